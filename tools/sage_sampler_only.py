"""GraphSAGE sampler throughput without training (diagnostic only): products-sage3's
pipelined sampler (native worker, side stream, 3 slots) run over one epoch's batches
with nothing else on the GPU.  If its wall per batch is near the pipelined epoch's
(~500 us), the sampler's launch chain -- not the training -- sets the batch time.

    python tools/sage_sampler_only.py
"""
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from cgnn_amd.gnn.data import reorder, synthetic
    from cgnn_amd.gnn.sage import SAGETrainer
    dev = torch.device("cuda", 0)
    g, _ = reorder(synthetic("ogbn-products", seed=0, device=dev), seed=0)
    tr = SAGETrainer(g, hidden=256, layers=3, dropout=0.5, lr=0.003, fanouts=(15, 10, 5), batch_size=1024)
    ps = tr._psampler
    batches = tr._batches()
    flat = torch.as_tensor(np.concatenate(batches).astype(np.int32), device=dev)
    seeds, o = [], 0
    for b in batches:
        seeds.append(flat[o:o + len(b)])
        o += len(b)
    res = {}
    for rep in range(3):
        torch.cuda.synchronize()
        ready = torch.cuda.Event()
        ready.record()
        t0 = time.perf_counter()
        depth, nb = len(ps.slots) - 1, len(seeds)
        pend = collections.deque(ps.enqueue(seeds[j], 1000 * rep + j, ready) for j in range(min(depth, nb)))
        for k in range(nb):                    # the epoch loop of SAGETrainer, minus the step
            if k + depth < nb:
                pend.append(ps.enqueue(seeds[k + depth], 1000 * rep + k + depth, ready))
            cur = pend.popleft()
            cur.resolve()
            torch.cuda.current_stream(dev).wait_event(cur.slot.done)
            ps.consumed(cur)
        torch.cuda.synchronize()
        res["rep%d_us_per_batch" % rep] = round(1e6 * (time.perf_counter() - t0) / len(seeds), 1)
    print(json.dumps({"sampler_only": res, "batches": len(seeds)}))


if __name__ == "__main__":
    main()
