"""Long-N CGNN training: the samples of one job split over the ranks of a process group.

The reference caps every run at ``max_nb_points`` = 1500 samples by subsampling
(CGNN.py:183-185) because TF materialises seven [2N, 2N] kernel matrices.  The
fused MMD kernels never materialise them (O(N d) memory), so one MI355X already
trains far longer sample sets; this trainer spreads one job's N samples over W
ranks (SURVEY §5 "long-context"):

* rank r owns samples [row0, row0 + N/W) of the data and GENERATES exactly those
  rows: generator noise is keyed by the global sample index (``row0`` of the
  generator kernel), so the generated set does not depend on W;
* per step the generated rows are all-gathered (O(R d N) bytes, against the
  O(R d N^2 / W) kernel work of the rank), the MMD kernels evaluate the rank's
  rows against all 2N columns (``row_begin`` / ``n_rows``), and the gradient of the
  global loss w.r.t. the rank's generated rows needs only those rows
  (``parallel/sharded_mmd.py``);
* the generator backward runs on the local rows; the parameter gradients are
  SUM-all-reduced (one [R, P] collective per step) and every rank applies the same
  TF1 Adam update, so the replicated parameters stay identical;
* the loss is a sum of per-rank partials: accumulated locally over the evaluation
  steps and all-reduced once at the end.

On a GPU every step is the HIP kernels (generator forward / backward, vector or
matrix-core MMD, Adam) plus RCCL; on the CPU the same decomposition runs on the
PyTorch oracle pieces (gloo tests).  With W = 1 it is simply the long-N trainer.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .. import native
from ..parallel.sharded_mmd import _mfma_geometry, _valu_geometry, row_partials
from .batch import _keys_tensor, mmd_kernel_choice, padded_dim, param_buffer, staged_setup
from .program import Program, pack_programs
from .reference import ReferenceTrainer


def shard_range(N: int, rank: int, world: int):
    """Equal contiguous sample blocks (N must be a multiple of the rank count)."""
    if N % world:
        raise ValueError("sample-sharded training needs N (%d) divisible by the rank count (%d)" % (N, world))
    per = N // world
    return rank * per, per


class SampleShardedTrainer:
    """Train + evaluate R models whose N samples are split over ``group``.

    ``datas_local``: this rank's data rows, one [d, N/W] array per model.  Without an
    initialised process group (or W = 1) it trains the whole sample set locally."""

    def __init__(self, programs: Sequence[Program], datas_local: Sequence[np.ndarray], keys: Sequence[tuple],
                 H: int, device, N: int, group=None, learning_rate=0.01, init_std=0.05, mmd_kernel="auto"):
        self.group = group
        self.dist = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist else 1
        self.rank = dist.get_rank(group) if self.dist else 0
        self.row0, self.n_loc = shard_range(int(N), self.rank, self.world)
        self.N = int(N)
        self.programs = list(programs)
        self.keys = list(keys)
        self.H = int(H)
        self.lr, self.init_std = float(learning_rate), float(init_std)
        self.R = len(self.programs)
        self.d = self.programs[0].n_vars
        if any(np.asarray(x).shape != (self.d, self.n_loc) for x in datas_local):
            raise ValueError("every model needs this rank's [d, N/W] = [%d, %d] data rows" % (self.d, self.n_loc))
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.rng_step = 0
        self.opt_step = 0
        if self.cuda:
            self._init_device(datas_local, mmd_kernel)
        else:
            self._init_cpu(datas_local)

    # ------------------------------------------------------------------ collectives
    def _all_reduce(self, t):
        if self.world > 1:
            dist.all_reduce(t, group=self.group)
        return t

    def _gather_cols(self, loc: torch.Tensor) -> torch.Tensor:
        """[R, D, n_loc] on every rank -> [R, D, N] (samples in global order)."""
        if self.world == 1:
            return loc
        R, D, n = loc.shape
        if loc.is_cuda:
            buf = torch.empty(self.world, R, D, n, dtype=loc.dtype, device=loc.device)
            dist.all_gather_into_tensor(buf, loc.contiguous(), group=self.group)
        else:
            parts = [torch.empty_like(loc) for _ in range(self.world)]
            dist.all_gather(parts, loc.contiguous(), group=self.group)
            buf = torch.stack(parts)
        return buf.permute(1, 2, 0, 3).reshape(R, D, self.world * n)

    # ------------------------------------------------------------------ GPU path
    def _init_device(self, datas_local, mmd_kernel):
        hip = native.hip()
        self.hip = hip
        R, d, n, N = self.R, self.d, self.n_loc, self.N
        D = padded_dim(d)
        self.D = D
        prog, stride, P, max_in = pack_programs(self.programs)
        self.P, self.stride, self.max_in = P, stride, max_in
        variant = hip.gen_bwd_variant(int(self.H), int(max_in), int(d), int(stride))
        if variant == 0:
            raise native.NativeExtensionError(
                "generator backward: H=%d with %d inputs per node does not fit in LDS" % (self.H, max_in))
        self.staged = variant == 2
        dx_global = False
        if self.staged:
            sched, self.sstride, self.stage_w, dx_global = staged_setup(self.programs, self.H, max_in, d, stride)
            self.sched = torch.from_numpy(sched).to(self.device)
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.prog = torch.from_numpy(prog).to(dev)
        data = np.zeros((R, D, n), dtype=np.float32)
        for r, x in enumerate(datas_local):
            data[r, :d] = np.asarray(x, dtype=np.float32)
        self.data_loc = torch.from_numpy(data).to(dev)
        self.data_all = self._gather_cols(self.data_loc).contiguous()
        self.keys_t = _keys_tensor(self.keys, dev)
        self.params = param_buffer(R, P, dev)
        self.m = torch.zeros(R, P, **f32)
        self.v = torch.zeros(R, P, **f32)
        self.xhat = torch.zeros(R, D, n, **f32)
        self.NS = D + max(int(p.n_conf) for p in self.programs)
        self.noise = torch.zeros(R, self.NS, n, **f32)
        self.xnorm = torch.zeros(R, n, **f32)
        self.step = torch.zeros(2, dtype=torch.int32, device=dev)
        self.kernel = mmd_kernel_choice(D, mmd_kernel)
        self.vgeo = _valu_geometry(n, N, R)
        self.mgeo = _mfma_geometry(n, N, R)
        G = hip.staged_tiles(n) if self.staged else hip.gen_bwd_blocks(n)
        self.gpart = torch.zeros(R, G, P, **f32)
        self.dxs = torch.zeros(R, d, n, **f32) if dx_global else None
        self.dnorm = (self.data_all * self.data_all).sum(1).contiguous()
        self.st = torch.cuda.current_stream(dev).cuda_stream
        hip.init_params(self.params.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), self.prog.data_ptr(), stride, P,
                        self.keys_t.data_ptr(), self.init_std, R, self.st)
        # constant true-true block of this rank's rows
        dummy = torch.empty(1, **f32)
        if hip.mmd_supported_d(D):
            rt, nc, tpc = self.vgeo
            lp = torch.empty(R, rt * nc, **f32)
            hip.mmd(2, D, self.data_all.data_ptr(), self.data_all.data_ptr(), dummy.data_ptr(), lp.data_ptr(), N, R,
                    rt, nc, tpc, 0.0, self.st, row_begin=self.row0, n_rows=n)
        else:                         # wide joints: the matrix-core kernel's true-true mode
            rb, nc, tpc = self.mgeo
            lp = torch.empty(R, rb * nc, **f32)
            hip.mmd_mfma(2, D, self.data_all.data_ptr(), self.data_all.data_ptr(), self.dnorm.data_ptr(),
                         self.dnorm.data_ptr(), dummy.data_ptr(), lp.data_ptr(), N, R, nc, tpc, 0.0, self.st,
                         row_begin=self.row0, n_rows=n)
        self.tt_part = lp.sum(1)

    def _device_step(self, train: bool) -> torch.Tensor:
        hip, R, D, n, N = self.hip, self.R, self.D, self.n_loc, self.N
        if self.staged:
            hip.gen_noise(self.prog.data_ptr(), self.stride, self.keys_t.data_ptr(), self.step.data_ptr(), 0,
                          self.noise.data_ptr(), self.NS, n, D, self.d, R, self.row0, self.st)
            hip.gen_fwd_staged(self.prog.data_ptr(), self.stride, self.sched.data_ptr(), self.sstride,
                               self.params.data_ptr(), self.P, self.data_loc.data_ptr(), self.xhat.data_ptr(),
                               self.noise.data_ptr(), self.NS, self.xnorm.data_ptr(), n, D, self.d, self.H,
                               self.max_in, R, self.stage_w, self.st)
        else:
            hip.gen_fwd(self.prog.data_ptr(), self.stride, self.params.data_ptr(), self.P, self.data_loc.data_ptr(),
                        self.xhat.data_ptr(), self.noise.data_ptr(), self.NS, self.xnorm.data_ptr(),
                        self.keys_t.data_ptr(), self.step.data_ptr(), 0, n, D, self.H, R, self.st, row0=self.row0)
        xall = self._gather_cols(self.xhat).contiguous()
        scale = 4.0 / (N * N) if train else 0.0
        mode = 0 if train else 1
        if self.kernel == "mfma":
            rb, nc, tpc = self.mgeo
            gp = torch.empty(nc, R, D, n, dtype=torch.float32, device=self.device)
            lp = torch.empty(R, rb * nc, dtype=torch.float32, device=self.device)
            xn = (xall * xall).sum(1).contiguous()
            hip.mmd_mfma(mode, D, xall.data_ptr(), self.data_all.data_ptr(), xn.data_ptr(), self.dnorm.data_ptr(),
                         gp.data_ptr(), lp.data_ptr(), N, R, nc, tpc, scale, self.st, row_begin=self.row0, n_rows=n)
        else:
            rt, nc, tpc = self.vgeo
            gp = torch.empty(nc, R, D, n, dtype=torch.float32, device=self.device)
            lp = torch.empty(R, rt * nc, dtype=torch.float32, device=self.device)
            hip.mmd(mode, D, xall.data_ptr(), self.data_all.data_ptr(), gp.data_ptr(), lp.data_ptr(), N, R, rt, nc,
                    tpc, scale, self.st, row_begin=self.row0, n_rows=n)
        part = lp.sum(1) + self.tt_part                      # this rank's share of the loss (x N^2)
        if train:
            if self.staged:
                hip.gen_bwd_staged(self.prog.data_ptr(), self.stride, self.sched.data_ptr(), self.sstride,
                                   self.params.data_ptr(), self.P, self.xhat.data_ptr(), self.noise.data_ptr(),
                                   self.NS, gp.data_ptr(), nc, R, n, D, self.d, self.H, self.max_in, self.stage_w,
                                   self.gpart.data_ptr(), self.dxs.data_ptr() if self.dxs is not None else 0,
                                   self.st)
            else:
                hip.gen_bwd(self.prog.data_ptr(), self.stride, self.params.data_ptr(), self.P, self.xhat.data_ptr(),
                            self.noise.data_ptr(), self.NS, gp.data_ptr(), nc, R, n, D, self.d, self.H,
                            self.max_in, self.gpart.data_ptr(), self.st)
            g = self.gpart.sum(1, keepdim=True).contiguous()     # [R, 1, P], fixed order
            self._all_reduce(g)
            hip.adam(self.params.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), g.data_ptr(), 1, self.prog.data_ptr(),
                     self.stride, self.P, self.step.data_ptr(), 0, self.lr, 0.9, 0.999, 1e-8, R, self.st)
            hip.advance(self.step.data_ptr(), 1, 1, self.st)
        else:
            hip.advance(self.step.data_ptr(), 1, 0, self.st)
        return part

    # ------------------------------------------------------------------ CPU path
    def _init_cpu(self, datas_local):
        self.ref = ReferenceTrainer(self.programs, datas_local, self.keys, self.H, learning_rate=self.lr,
                                    init_std=self.init_std)
        self.ref.row0 = self.row0
        self.data_loc = [torch.as_tensor(np.asarray(x), dtype=torch.float64) for x in datas_local]   # [d, n]
        self.data_all = [self._gather_cols(x[None]).squeeze(0) for x in self.data_loc]                # [d, N]
        self.ms = [torch.zeros_like(p) for p in self.ref.params]
        self.vs = [torch.zeros_like(p) for p in self.ref.params]

    def _cpu_step(self, train: bool) -> torch.Tensor:
        ref, R = self.ref, self.R
        ref.rng_step = self.rng_step
        parts, grads = [], []
        for r in range(R):
            theta = ref.params[r].clone().requires_grad_(train)
            with torch.set_grad_enabled(train):
                xg = ref.generate(r, theta)                                   # [d, n] local rows
            P_all = self._gather_cols(xg.detach()[None]).squeeze(0)           # [d, N]
            loss, g = row_partials(xg.detach().T[None], self.data_loc[r].T[None], P_all.T[None],
                                   self.data_all[r].T[None], self.row0)
            parts.append(loss[0])
            if train:
                (gt,) = torch.autograd.grad(xg, theta, grad_outputs=g[0].T.to(xg.dtype))
                grads.append(gt)
        if train:
            flat = torch.stack(grads)
            self._all_reduce(flat)
            t = self.opt_step + 1
            b1, b2, eps = 0.9, 0.999, 1e-8
            lr_t = self.lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
            for r in range(R):
                g = flat[r]
                self.ms[r] = b1 * self.ms[r] + (1 - b1) * g
                self.vs[r] = b2 * self.vs[r] + (1 - b2) * g * g
                ref.params[r] = ref.params[r] - lr_t * self.ms[r] / (self.vs[r].sqrt() + eps)
            self.opt_step += 1
        self.rng_step += 1
        return torch.stack(parts)

    # ------------------------------------------------------------------ driver
    def _step(self, train):
        return self._device_step(train) if self.cuda else self._cpu_step(train)

    def train(self, epochs: int):
        for _ in range(int(epochs)):
            self._step(True)

    def evaluate(self, epochs: int) -> np.ndarray:
        acc = None
        for _ in range(int(epochs)):
            p = self._step(False)
            acc = p if acc is None else acc + p
        acc = self._all_reduce(acc.to(torch.float64).clone())
        return (acc / (self.N * self.N * max(int(epochs), 1))).cpu().numpy()

    def run(self, train_epochs: int, test_epochs: int) -> np.ndarray:
        self.train(train_epochs)
        return self.evaluate(test_epochs)
