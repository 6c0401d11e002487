"""Record the exact outcomes of the three reference example workloads (the accuracy
gates of tests/test_examples_gpu.py) at the gates' fixed settings, as JSON.

    python tools/pin_examples.py tests/data/expected_examples.json
    python tools/pin_examples.py --compat compat_examples.json     (SETTINGS.compat_scores)

Scores are deterministic on a given device and kernel build (counter-based RNG,
fixed-order reductions, bitwise independent of batching), so the gates compare the
outcome exactly; re-run this after a deliberate numerics change of the CGNN kernels
and commit the new file with the change that caused it."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    args = [a for a in sys.argv[1:] if a != "--compat"]
    compat = "--compat" in sys.argv[1:]
    out = args[0] if args else "expected_examples.json"
    import pandas as pd
    import cgnn
    from conftest import example
    from cgnn_amd.utils.formats import CCEPC_PairsFileReader
    from cgnn_amd.utils.metrics import orientation_scores, shd, sign_accuracy
    from test_examples_gpu import REFERENCE_SETTINGS, run_confounders, run_graph, run_pairwise
    for k, v in REFERENCE_SETTINGS.items():
        setattr(cgnn.SETTINGS, k, v)
    cgnn.SETTINGS.compat_scores = compat
    wall = {}
    t0 = time.perf_counter()
    pred, targets = run_pairwise()
    wall["pairwise"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    dag, target = run_graph()
    wall["graph"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    cdag, ctarget = run_confounders()
    wall["confounders"] = time.perf_counter() - t0
    rec = {
        "settings": dict(REFERENCE_SETTINGS, compat_scores=compat),
        "pairwise": {"signs": [int(x > 0) - int(x < 0) for x in pred], "predictions": [float(x) for x in pred],
                     "sign_accuracy": float(sign_accuracy(pred, targets))},
        "graph": {"edges": sorted([a, b] for a, b, _ in dag.get_list_edges()), "shd": int(shd(dag, target))},
        "confounders": {"edges": sorted([a, b] for a, b, _ in cdag.get_list_edges()),
                        "scores": orientation_scores(cdag, ctarget)},
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({"pairwise_sign_accuracy": rec["pairwise"]["sign_accuracy"], "graph_shd": rec["graph"]["shd"],
                      "confounders": rec["confounders"]["scores"],
                      "wall_s": {k: round(v, 2) for k, v in wall.items()}}))


if __name__ == "__main__":
    main()
