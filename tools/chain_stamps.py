"""Per-stage timeline of one persistent kq_chain launch (the bench's TinyLlama token):
per (workgroup, stage) s_memrealtime stamps when the stage's activation is in LDS
(after the workgroup barrier) and when the workgroup finished the stage.
Prints, per stage, the spread of x-ready times over workgroups, the stage's compute
span and the hand-off (first x-ready of stage s+1 minus the last done of stage s)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from bench import Chain  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    g.gemv_impl(g.GEMV_CHAIN)
    chain = Chain(os.environ.get("MODEL", "tinyllama-1.1b"), dev, seed=1)
    be = g.Backend(0)
    S = len(chain.stages)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    buf = torch.zeros(cus * S * 8 + 64, dtype=torch.int64, device=dev)
    for _ in range(20):
        assert be.graph_compute(chain.nodes, use_graph=False) == 0
    be.synchronize()
    runs = []
    for r in range(5):
        for i in range(10):
            if i == 9:
                be.synchronize()
                buf.zero_()
                torch.cuda.synchronize()
                g.lib().mi355x_diag_stamps(buf.data_ptr(), buf.numel() * 8)
            assert be.graph_compute(chain.nodes, use_graph=False) == 0
        be.synchronize()
        g.lib().mi355x_diag_stamps(None, 0)
        st = buf[:cus * S * 8].cpu().numpy().astype(np.int64).reshape(cus, S, 8)
        npoll = st[:, :, 7].copy()
        t0 = st[:, 0, 3].min()
        rel = (st - t0) * 10 / 1000.0  # 100 MHz ticks -> us
        rel[:, :, 7] = npoll
        runs.append(rel)
    R = np.median(np.stack(runs), axis=0)  # [wg, stage, 8]
    # per (workgroup, stage): 0 first poll, 1 poll ok, 2 quantized (wave 0, a poller);
    # 3 activation ready, 4 computed, 5 flushed, 6 next ring issued (last wave, streams rows); 7 polls
    med = lambda v: float(np.median(v))  # noqa: E731
    cols = ("gap", "poll", "npoll", "quant", "barrier", "compute", "flush", "pref", "vis", "span")
    print(f"{'st':>3} {'matrices':<22} " + " ".join(f"{c:>7}" for c in cols))
    tot = {}
    for s, stage in enumerate(chain.stages):
        row = dict(
            gap=med(R[:, s, 0] - R[:, s - 1, 6]) if s else 0.0,       # own streamers done -> first poll
            poll=med(R[:, s, 1] - R[:, s, 0]) if s else 0.0, npoll=med(R[:, s, 7]),
            quant=med(R[:, s, 2] - R[:, s, 1]) if s else 0.0,
            barrier=med(R[:, s, 3] - R[:, s, 2]) if s else 0.0,
            compute=med(R[:, s, 4] - R[:, s, 3]), flush=med(R[:, s, 5] - R[:, s, 4]),
            pref=med(R[:, s, 6] - R[:, s, 5]),
            vis=(R[:, s, 1].min() - R[:, s - 1, 5].max()) if s else 0.0,  # last flush anywhere -> first poll ok
            span=R[:, s, 3].max() - (R[:, s - 1, 3].max() if s else 0.0))
        names = "+".join(n.split(".")[-1].replace("attn_", "").replace("ffn_", "") for n, *_ in stage)
        for k, v in row.items():
            tot.setdefault(names, {}).setdefault(k, []).append(v)
        if s < 6 or s >= S - 2:
            print(f"{s:3d} {names:<22} " + " ".join(f"{row[c]:7.2f}" for c in cols))
    print(f"token: {R[:, -1, 6].max():.1f} us (from the first workgroup's stage-0 activation)")
    for names, d in tot.items():
        print(f"  median {names:<22} " + " ".join(f"{k}={np.median(v):.2f}" for k, v in d.items()))


if __name__ == "__main__":
    main()
