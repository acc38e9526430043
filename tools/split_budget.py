"""Multi-GPU budget of the row split (DESIGN.md §6 worksheet), measured on ONE GPU.

For a world of N GPUs a decode token takes T(N) = T_rank(N) + C(N) * c(N): the compute of
one rank (its row / K slices, every launch of its graph) plus C collectives of latency c
each. T_rank(N) is measured here exactly: rank 0's graph of the N-way split runs on this
GPU with the collectives emulated as no-ops (mi355x_backend_set_comm_loopback with
MI355X_LOOPBACK_NOCOPY: timing only, the exchanged vectors stay stale). C(N) is the node
count of the schedule (gather: 4 per layer + 1; reduce: 2 per layer + 1). c(1) — an RCCL
collective on a 1-rank communicator in the hipGraph — is measured too; c(N > 1) over xGMI
needs the 8-GPU node. The output gives, per model / mode / N, the largest c that still
reaches a target speedup (3.5x at N = 4, the north_star's), so the scaling run can be read
against it.

    python tools/split_budget.py > gpurun_out/split_budget.json
"""
import json
import os
import sys
import time

os.environ.setdefault("MI355X_LOOPBACK_NOCOPY", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import ggml_mi355x as g  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()  # the MI355X_* A/B environment -> explicit library calls



def time_token(model, dev, world, mode, steps, warmup=4):
    be = g.Backend(0)
    if world > 1:
        be.set_comm_loopback(0, world)
    n_ctx = 128
    tk = bench.Token(model, dev, 0x51A7, be, n_ctx, split=(world, 0, mode) if world > 1 else None)
    for i in range(warmup):
        tk.dec.step(tk.tokens[i], i)
    be.synchronize()
    tk.dec.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tk.dec.step(tk.tokens[i], i)
    be.synchronize()
    el = time.perf_counter() - t0
    out = {"ms_per_token": round(el / steps * 1e3, 4), "launches": tk.launches(),
           "collectives": tk.split.collectives_per_token() if tk.split is not None else 0,
           "weights_MB_per_gpu": round(tk.bytes_per_token / 1e6, 1)}
    del tk, be
    torch.cuda.empty_cache()
    return out


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    res = {"note": "T_rank(N): rank 0's split graph with no-op collectives (loopback, no copy); "
                   "c_max_us: largest per-collective latency that reaches `speedup_target` x the 1-GPU token"}
    try:
        res["collective_us_world1"] = bench.collective_side(dev, 1, 0, 0, lambda: None)
    except Exception as e:  # noqa: BLE001
        res["collective_us_world1"] = {"error": str(e)}
    for model, steps in (("tinyllama-1.1b", 64), ("llama-3-70b", 8)):
        base = time_token(model, dev, 1, "gather", steps)
        rows = {"1": base}
        for world in (2, 4, 8):
            for mode in ("gather", "reduce"):
                try:
                    r = time_token(model, dev, world, mode, steps)
                except ValueError as e:
                    rows[f"{world}-{mode}"] = {"error": str(e)}
                    continue
                t1 = base["ms_per_token"]
                r["compute_speedup"] = round(t1 / r["ms_per_token"], 3)
                target = {2: 1.8, 4: 3.5, 8: 6.0}[world]
                r["speedup_target"] = target
                # T(N) = T_rank + C * c <= t1 / target  ->  c <= (t1 / target - T_rank) / C
                slack_ms = t1 / target - r["ms_per_token"]
                r["c_max_us"] = round(slack_ms * 1e3 / r["collectives"], 2) if r["collectives"] else None
                rows[f"{world}-{mode}"] = r
                print(model, world, mode, r, file=sys.stderr, flush=True)
        res[model] = rows
    print(json.dumps(res))


if __name__ == "__main__":
    main()
