"""Wall time of one reference example script run through the framework (pairwise, graph
or confounders; tests/test_examples_gpu.py runners), for profiling (cProfile /
rocprofv3 --stats around it).

    python tools/profile_example.py confounders
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "confounders"
    import test_examples_gpu as ex
    fn = {"pairwise": ex.run_pairwise, "graph": ex.run_graph, "confounders": ex.run_confounders}[which]
    t = time.perf_counter()
    fn()
    print('{"example": "%s", "wall_s": %.3f}' % (which, time.perf_counter() - t), flush=True)


if __name__ == "__main__":
    main()
