"""A/B of the pipelined GraphSAGE loop's sampler settings on the products-sage3 shape:
sampler stream priority (-1 high / 0 normal) x slots (3: two batches sampled ahead, 4:
three).  One graph, one trainer per setting, 4 timed epochs after 1 warm-up, twice in
alternating order.  One JSON line per run.

    python tools/ab_sage_prio.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from cgnn_amd.gnn import sampler as smp
    from cgnn_amd.gnn.data import reorder, synthetic
    from cgnn_amd.gnn.sage import SAGETrainer
    dev = torch.device("cuda", 0)
    g = synthetic("ogbn-products", seed=0, device=dev, scale=1.0)
    g, _ = reorder(g)
    settings = [(-1, 3), (0, 3), (-1, 4), (0, 4)]
    for rep in range(2):
        for prio, slots in (settings if rep == 0 else settings[::-1]):
            smp.STREAM_PRIORITY = prio
            orig = smp.PipelinedSampler.__init__

            def init(self, *a, _orig=orig, _slots=slots, **k):
                k["slots"] = _slots
                _orig(self, *a, **k)
            smp.PipelinedSampler.__init__ = init
            try:
                tr = SAGETrainer(g, hidden=256, layers=3, dropout=0.5, lr=0.003, fanouts=(15, 10, 5),
                                 batch_size=1024, seed=0)
            finally:
                smp.PipelinedSampler.__init__ = orig
            tr.train_epoch()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(4):
                tr.train_epoch()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / 4
            print(json.dumps({"rep": rep, "priority": prio, "slots": slots, "epochs_per_s": round(1.0 / dt, 3)}),
                  flush=True)
            del tr
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
