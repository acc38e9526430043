"""A/B of the persistent decode layer (csrc/kq_layer.hip) against the per-node launches on
one box, interleaved: the bench's full decode token (synthetic Q4_K_M weights of the real
shapes, graph replay, tokens 0..steps-1 from an empty cache) with mi355x_backend_set_layer_engine
off / on, rounds alternating. Prints one JSON line per model.

    python tools/layer_ab.py [--models tinyllama-1.1b,llama-3-8b] [--rounds 3] [--steps 64]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ggml-neon-opt_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import ggml_mi355x as g  # noqa: E402


def run(tk, be, steps):
    tk.dec.reset()
    torch.cuda.synchronize()
    st = torch.cuda.ExternalStream(be.stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for i in range(steps):
        tk.dec.step(tk.tokens[i], i)
    e1.record(st)
    be.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="tinyllama-1.1b,llama-3-8b")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--mix", default="q4_k_m")
    ap.add_argument("--layer-profile", action="store_true", help="also per-launch event timing of one eager token")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for model in args.models.split(","):
        be = g.Backend(0)
        tk = bench.Token(model, dev, 0x51A7, be, max(128, args.steps), mix=args.mix)
        for i in range(8):
            tk.dec.step(tk.tokens[i], i)
        be.synchronize()
        res = {"off": [], "on": []}
        for r in range(args.rounds):
            for mode in ("off", "on"):
                be.set_layer_engine(mode == "on")
                run(tk, be, 8)  # capture + warm
                res[mode].append(run(tk, be, args.steps))
                if mode == "on":
                    err = be.layer_error()
                    if err:
                        res["error"] = "a persistent-layer wait gave up"
        out = {"model": model, "mix": args.mix, "steps": args.steps,
               "ms_per_token": {k: [round(x, 4) for x in v] for k, v in res.items() if k != "error"},
               "tok_s": {k: round(1e3 / min(v), 1) for k, v in res.items() if k != "error"},
               "error": res.get("error")}
        if args.layer_profile:
            kinds = {}
            for mode in ("off", "on"):
                be.set_layer_engine(mode == "on")
                tk.dec.reset()
                tk.dec.step(tk.tokens[0], 0, use_graph=False)
                be.synchronize()
                g.timing_enable(True)
                for i in range(1, 4):
                    tk.dec.step(tk.tokens[i], i, use_graph=False)
                be.synchronize()
                rows = g.timing_read()
                g.timing_enable(False)
                agg = {}
                for name, nbytes, ms in rows:
                    a = agg.setdefault(name, [0, 0.0, 0.0])
                    a[0] += 1
                    a[1] += ms
                    a[2] += nbytes
                kinds[mode] = {k: {"launches": v[0], "us_per_launch": round(v[1] * 1e3 / v[0], 2),
                                   "MB_per_launch": round(v[2] / v[0] / 1e6, 2)} for k, v in agg.items()}
            out["eager_kernels"] = kinds
        print(json.dumps(out), flush=True)
        del tk, be
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
