"""Batched device trainer: R independent CGNN models in one set of kernels.

The unit of GPU work is a *batch of models* (runs x candidates x pairs),
not one TF session.  Buffers are PyTorch tensors on the target
device; the step sequence is owned by the native ``CgnnEngine`` (C++), which
replays chunks of steps through hipGraphs.  Nothing is copied back to the host
until the final scores are read.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch

from .. import native
from .program import Program, pack_programs, pack_schedules

# padded variable counts with compiled kernels; above 64 only the matrix-core MMD, above
# 256 its dimension-grouped form and the wide (scratch-image) Fourier-feature MMD
SUPPORTED_D = (1, 2, 3, 4, 6, 8, 12, 16, 20, 24, 32, 48, 64, 80, 96, 128, 160, 192, 224, 256,
               320, 384, 448, 512, 640, 768, 896, 1024)
MAX_D = 16384             # above 1024: every multiple of 256 (runtime-width grouped MMD)
# above: rff_kernels.hip's wide form (theta scratch image); at and below: the forms compiled
# per width.  The wide form is 2-11x faster from D = 64 up (tools/ab_rff.py, profiles/r05_rff)
WIDE_RFF_D = 32
MAX_VALU_D = 64
MMD_TILE = 256
TARGET_WGS = 2048


def padded_dim(d: int) -> int:
    for D in SUPPORTED_D:
        if D >= d:
            return D
    if d <= MAX_D:
        return (d + 255) // 256 * 256
    raise ValueError("CGNN device path supports at most %d variables (got %d)" % (MAX_D, d))


def mmd_geometry(N: int, R: int = 0):
    """(row_tiles, n_chunks, tiles_per_chunk) of the vector MMD kernel.  A function
    of N only -- never of the batch size R -- so the fixed-order sums (and hence every
    score) are bitwise independent of how jobs are batched or sharded over GPUs:
    one 256-column tile per chunk."""
    row_tiles = (N + MMD_TILE - 1) // MMD_TILE
    ct = 2 * row_tiles
    return row_tiles, ct, 1


MFMA_ROWS = 128     # generated rows per workgroup of the matrix-core MMD
MFMA_TILE = 32      # joint columns per LDS tile


def mmd_mfma_geometry(N: int, R: int = 0):
    """(row_blocks, n_chunks, tiles_per_chunk) of the matrix-core MMD; like
    ``mmd_geometry`` a function of N only (batch-independent sums): small N get a
    few column chunks so that one model still spreads over >= 8 workgroups."""
    rb = (N + MFMA_ROWS - 1) // MFMA_ROWS
    ct = 2 * ((N + MFMA_TILE - 1) // MFMA_TILE)
    n_chunks = min(ct, max(1, math.ceil(8 / rb)))
    tpc = math.ceil(ct / n_chunks)
    n_chunks = math.ceil(ct / tpc)
    return rb, n_chunks, tpc


def mmd_mirror_slots(D: int, N: int, symmetric: bool = True) -> int:
    """Extra gradient slots of a symmetric vector-kernel training launch (0: the launch
    evaluates the full pred-pred block; ``symmetric=False`` forces that)."""
    if not symmetric:
        return 0
    return int(native.hip().mmd_mirror_slots(D, N))


def mmd_kernel_choice(D: int, mmd_kernel: str = "auto") -> str:
    """'mfma' (matrix cores, D >= 8) or 'valu' (packed-fp32 vector kernel).
    ``CGNN_MMD_KERNEL=valu|mfma`` overrides 'auto'."""
    import os
    choice = mmd_kernel
    if choice == "auto":
        choice = os.environ.get("CGNN_MMD_KERNEL", "auto")
    hip = native.hip()
    if choice == "auto":
        choice = "mfma" if hip.mmd_mfma_supported(D) else "valu"
    if choice == "mfma" and not hip.mmd_mfma_supported(D):
        raise ValueError("matrix-core MMD needs a padded D >= 8 from engine.batch.SUPPORTED_D, got %d" % D)
    if choice == "valu" and D > MAX_VALU_D:
        raise ValueError("the vector MMD kernel covers D <= %d (got %d): use the matrix-core one" % (MAX_VALU_D, D))
    if choice not in ("mfma", "valu"):
        raise ValueError("mmd_kernel must be auto|mfma|valu")
    return choice


def _prog_stride(prog_len: int) -> int:
    return (int(prog_len) + 3) // 4 * 4              # pack_programs' stride


def kernel_family(d: int, H: int, max_in: int, prog_len: int = 0) -> int:
    """Generator-kernel family of a batch of ``d``-variable programs: 1 the per-sample
    kernels (sample state in LDS), 2 the level-scheduled ones, 0 neither.  The scorer
    evaluates it per program and batches programs of one family together, so the kernels
    that train a model -- and its score -- do not depend on its batch-mates."""
    return int(native.hip().gen_bwd_variant(int(H), int(max_in), int(d), _prog_stride(prog_len)))


def device_supported(d: int, H: int, max_in: int, prog_len: int = 0, fast_mmd: bool = False) -> bool:
    """True when the device kernels cover a batch of ``d``-variable programs with hidden
    width ``H``, at most ``max_in`` generator inputs per node and programs of at most
    ``prog_len`` ints: the variable count up to MAX_D, and either the
    per-sample generator kernels (sample state in LDS) or the level-scheduled ones.
    Otherwise ``score_jobs`` trains the batch on the CPU reference path (with a warning)."""
    if d > MAX_D:
        return False
    variant = kernel_family(d, H, max_in, prog_len)
    if variant == 1:
        return native.hip().gen_fwd_lds(padded_dim(d), _prog_stride(prog_len)) <= 160 * 1024
    return variant == 2


def staged_setup(programs: Sequence[Program], H: int, max_in: int, d: int, prog_stride: int):
    """Schedule + launch plan of the level-scheduled generator kernels for a batch:
    (schedule [R, stride] int32, stride, waves per block, dL/dx in global memory)."""
    sched, sstride, width = pack_schedules(programs)
    W = 8
    while W > 1 and W // 2 >= width:
        W //= 2
    # the launchers plan with the same arguments (no program words are staged in LDS), so
    # the dL/dx placement chosen here is the one they launch
    plan = native.hip().staged_plan(int(d), int(H), int(max_in), W, 0)
    if not plan:
        raise native.NativeExtensionError("staged generator kernels: no LDS plan for d=%d H=%d" % (d, H))
    return sched, sstride, W, bool(plan[2])


PARAM_PAD = 64    # floats past the last model (cgnn_staged.hip tail-chunk weight loads)


def param_buffer(R: int, P: int, device) -> torch.Tensor:
    """[R, P] fp32 zeros whose storage runs PARAM_PAD floats past the last model."""
    return torch.zeros(R * P + PARAM_PAD, dtype=torch.float32, device=device)[:R * P].view(R, P)


def _keys_tensor(keys, device):
    arr = np.asarray(keys, dtype=np.uint64).astype(np.uint32).reshape(-1)
    return torch.from_numpy(arr.view(np.int32).copy()).to(device)


class DeviceTrainer:
    """Train + evaluate R models on one GPU; returns per-model scores."""

    def __init__(self, programs: Sequence[Program], datas: Sequence[np.ndarray],
                 keys: Sequence[tuple], H: int, device, learning_rate=0.01, init_std=0.05,
                 use_fast_mmd=False, nb_vectors=100, record_history=0, graph_chunk=50,
                 mmd_kernel="auto", generator="auto"):
        # generator: "auto" (kernel_family of the batch), "staged" (the level-scheduled
        # kernels even where the per-sample ones fit: equivalence tests, A/B tools)
        hip = native.hip()
        self.hip = hip
        self.device = torch.device(device)
        R = len(programs)
        d = programs[0].n_vars
        if any(p.n_vars != d for p in programs):
            raise ValueError("all models in a device batch must share the variable count")
        N = int(np.asarray(datas[0]).shape[1])
        if any(np.asarray(x).shape != (d, N) for x in datas):
            raise ValueError("all models in a device batch must share the data shape [d, N]")
        D = padded_dim(d)
        self.R, self.N, self.d, self.D, self.H = R, N, d, D, int(H)
        prog, stride, P, max_in = pack_programs(programs)
        self.P, self.prog_stride, self.max_in = P, stride, max_in
        if generator not in ("auto", "staged"):
            raise ValueError("generator must be auto|staged")
        self.bwd_variant = hip.gen_bwd_variant(int(H), int(max_in), int(d), int(stride))
        if generator == "staged":
            self.bwd_variant = 2 if hip.gen_staged_supported(int(H), int(max_in), int(d)) else 0
        if self.bwd_variant == 0:
            raise native.NativeExtensionError(
                "generator backward: H=%d with %d inputs per node does not fit in LDS" % (H, max_in))
        self.staged = self.bwd_variant == 2
        if self.staged:
            sched, sstride, self.stage_w, dx_global = staged_setup(programs, H, max_in, d, stride)
        else:
            sched, sstride, self.stage_w, dx_global = np.zeros((1, 4), np.int32), 4, 8, False
        self.sched_stride = sstride
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            self.prog = torch.from_numpy(prog).to(dev)
            data = np.zeros((R, D, N), dtype=np.float32)
            for r, x in enumerate(datas):
                data[r, :d] = np.asarray(x, dtype=np.float32)
            self.data = torch.from_numpy(data).to(dev)
            self.keys = _keys_tensor(keys, dev)
            self.params = param_buffer(R, P, dev)
            self.m = torch.zeros(R, P, **f32)
            self.v = torch.zeros(R, P, **f32)
            self.xhat = torch.zeros(R, D, N, **f32)
            # forward noise draws, reused by the backward: [R][D + confounder streams][N]
            self.NS = D + max(int(p.n_conf) for p in programs)
            self.noise = torch.zeros(R, self.NS, N, **f32)
            row_tiles, n_chunks, tpc = mmd_geometry(N, R)
            self.geometry = (row_tiles, n_chunks, tpc)
            self.rff_k = int(nb_vectors) if use_fast_mmd else 0
            self.mmd_kernel = "rff" if self.rff_k else mmd_kernel_choice(D, mmd_kernel)
            mf_rb, mf_chunks, mf_tpc = mmd_mfma_geometry(N, R)
            F = 7 * self.rff_k
            n_parts = max(row_tiles * n_chunks, mf_rb * mf_chunks, (F + 255) // 256 if F else 0)
            # symmetric pred-pred training on the vector kernel: extra gradient slots for
            # the mirrored column sums
            self.mirror = mmd_mirror_slots(D, N) if self.mmd_kernel == "valu" else 0
            self.gradp = torch.zeros(max(n_chunks + self.mirror, mf_chunks, 1), R, D, N, **f32)
            self.lpart = torch.zeros(R, n_parts, **f32)
            G = hip.staged_tiles(N) if self.staged else hip.gen_bwd_blocks(N)
            self.gpart = torch.zeros(R, G, P, **f32)
            self.sched = torch.from_numpy(sched).to(dev)
            self.tt = torch.zeros(R, **f32)
            self.loss_last = torch.zeros(R, **f32)
            self.loss_acc = torch.zeros(R, **f32)
            self.hist_len = int(record_history)
            self.hist = torch.zeros(R, max(self.hist_len, 1), **f32)
            self.step = torch.zeros(2, dtype=torch.int32, device=dev)
            self.rff_w = torch.zeros(R, max(F, 1), D + 1, **f32)
            self.rff_diff = torch.zeros(R, max(F, 1), **f32)
            # wide joints: theta of the generated samples + cos-sum partials
            self.rff_scratch = (torch.zeros(hip.rff_wide_scratch_floats(N, F, R), **f32)
                                if self.rff_k and D > WIDE_RFF_D else None)
            # squared row norms for the Gram-form (matrix-core) MMD
            self.xnorm = torch.zeros(R, N, **f32)
            self.ynorm = (self.data * self.data).sum(1).contiguous()
            # dL/dx scratch of a staged backward whose sample state does not fit in LDS
            self.dxs = torch.zeros(R, d, N, **f32) if dx_global else None
            # a dedicated (non-default) stream: hipGraph capture is not allowed on
            # the legacy null stream, and batches on different devices overlap
            self.stream = torch.cuda.Stream(dev)
            stream = self.stream
            icfg = [R, N, D, self.H, P, stride, max_in, row_tiles, n_chunks, tpc, self.hist_len,
                    self.rff_k, d, self.NS, int(self.mmd_kernel == "mfma"), mf_chunks, mf_tpc, self.mirror,
                    int(self.staged), sstride, self.stage_w]
            fcfg = [float(learning_rate), 0.9, 0.999, 1e-8, float(init_std)]
            ptrs = [t.data_ptr() for t in (self.prog, self.params, self.m, self.v, self.data,
                                           self.xhat, self.noise, self.gradp, self.lpart, self.gpart,
                                           self.tt, self.loss_last, self.loss_acc)]
            ptrs.append(self.hist.data_ptr() if self.hist_len else 0)
            ptrs += [self.step.data_ptr(), self.keys.data_ptr(), self.rff_w.data_ptr(),
                     self.rff_diff.data_ptr(), self.xnorm.data_ptr(), self.ynorm.data_ptr(),
                     self.dxs.data_ptr() if self.dxs is not None else 0, self.sched.data_ptr(),
                     self.rff_scratch.data_ptr() if self.rff_scratch is not None else 0]
            self.engine = hip.CgnnEngine(icfg, fcfg, ptrs, stream.cuda_stream)
        self.graph_chunk = int(graph_chunk)

    def start(self):
        """Initialise parameters and the constant true-true MMD block (async)."""
        with torch.cuda.device(self.device):
            self.step.zero_()
            self.loss_acc.zero_()
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            self.engine.init()
            self.engine.tt()

    def train(self, epochs: int):
        with torch.cuda.device(self.device):
            self.engine.run(0, int(epochs), self.graph_chunk, self.hist_len > 0)

    def evaluate(self, epochs: int, log_every: int = 0, log=None):
        """Enqueue ``epochs`` evaluation steps (the score accumulates in ``loss_acc``).
        ``log_every`` > 0: ``log(it, losses[R])`` with the loss of every step
        ``it % log_every == 0`` (the reference's verbose evaluate, CGNN.py:147-149); the
        steps run in the same order with the same draws, in chunks that end at those
        steps (one host read of ``loss_last`` each)."""
        epochs = int(epochs)
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            self.loss_acc.zero_()
            if log_every <= 0 or log is None:
                self.engine.run(1, epochs, self.graph_chunk, False)
                return
            it = 0
            while it < epochs:
                self.engine.run(1, 1, 0, False)
                log(it, self.loss_last.cpu().numpy())
                k = min(int(log_every) - 1, epochs - it - 1)
                self.engine.run(1, k, self.graph_chunk, False)
                it += 1 + k

    def _join(self):
        torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def launch(self, train_epochs: int, test_epochs: int):
        """Enqueue the whole train+eval schedule without synchronising."""
        self.start()
        self.train(train_epochs)
        self.evaluate(test_epochs)
        self._test_epochs = max(int(test_epochs), 1)

    def collect(self) -> np.ndarray:
        self._join()
        scores = (self.loss_acc / float(self._test_epochs)).cpu().numpy().astype(np.float64)
        return scores

    def history(self) -> np.ndarray:
        self._join()
        return self.hist[:, :self.hist_len].cpu().numpy()

    def run(self, train_epochs: int, test_epochs: int, verbose=False) -> np.ndarray:
        self.launch(train_epochs, test_epochs)
        scores = self.collect()
        if verbose and self.hist_len:
            h = self.history()
            for r in range(self.R):
                for it in range(0, self.hist_len, 100):
                    print('Run:{}, Iter:{}, score:{}'.format(r, it, h[r, it]))
        return scores

    def generated(self) -> np.ndarray:
        """Last generated samples, [R, d, N]."""
        self._join()
        return self.xhat[:, :self.d].cpu().numpy()
