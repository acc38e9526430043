"""Debug aid: run a small dependent chain with GEMV_CHAIN and GEMV_ROWS and report,
per node, how many outputs differ (and the bus hand-off status)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from oracle import kq_oracle_np as npo  # noqa: E402
from test_gpu_chain import SMALL, Graph  # noqa: E402


SPECS = {
    "2st": [(None, [(12, 512)]), (0, [(12, 1024)])],
    "2st-2d": [(None, [(12, 512)]), (0, [(12, 1024), (12, 1024)])],
    "3st": [(None, [(12, 512)]), (0, [(12, 512)]), (1, [(12, 1024), (12, 1024)])],
    "small": SMALL,
}


def main():
    import torch
    torch.cuda.init()
    for name, spec in SPECS.items():
        print("==", name)
        run(spec)


def run(spec):
    rng = np.random.default_rng(5)
    be = g.Backend(0)
    G = Graph(g, be, rng, npo, spec, 512)
    res = {}
    for name, impl in (("rows", g.GEMV_ROWS), ("chain", g.GEMV_CHAIN)):
        g.gemv_impl(impl)
        assert be.graph_compute(G.nodes, use_graph=False) == 0
        try:
            be.synchronize()
        except Exception as e:  # noqa: BLE001
            print(name, "sync:", e)
        res[name] = G.outputs()
    for i, (a, b) in enumerate(zip(res["rows"], res["chain"])):
        bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
        print(f"node {i} meta {G.meta[i]} mismatches {len(bad)} first {bad[:8].tolist()}")
    G.close()


if __name__ == "__main__":
    main()
