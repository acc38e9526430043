"""Phase timeline of the persistent decode layer (csrc/kq_layer.hip) from the stamps build:
    make -C ggml-neon-opt_amd variant-layer NAME=lst VFLAGS="-DKQ_LAYER_STAMPS=1"
    python tools/layer_stamps.py [--model llama-3-8b] [--tokens 8]
Decodes a few eager tokens of the bench's model with the engine on; for one layer launch
per token (the middle layer) prints, per phase, the median / max over workgroups of the
stamp relative to the launch's first stamp (us). Slots (control wave, lane 0):
0 entry, 1 stage-0 loads landed, 2 stage-0 activation, 3 C0 (q/k/v records), 4 E1 signalled,
5 E1 passed (attention workgroups), 6 E2 signalled (attention done), 7 E2 passed, 8 B2,
9 C2, 10 E3 signalled, 11 E3 passed, 12 B3, 13 C3, 14 E4 signalled, 15 E4 passed, 16 B4,
17 C4, 18 end."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
os.environ.setdefault("MI355X_LIB", os.path.join(ROOT, "ggml-neon-opt_amd/lib/variants/liblst.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import ggml_mi355x as g  # noqa: E402

NAMES = ["entry", "x0 in", "act0", "C0", "E1 sig", "E1 pass", "E2 sig", "E2 pass", "B2", "C2", "E3 sig",
         "E3 pass", "B3", "C3", "E4 sig", "E4 pass", "B4", "C4", "end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tokens", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    be = g.Backend(0)
    tk = bench.Token(args.model, dev, 0x51A7, be, 128)
    be.set_layer_engine(True)
    G = 256
    buf = torch.zeros(G * 32, dtype=torch.int64, device=dev)
    for i in range(4):  # warm: graph capture etc.
        tk.dec.step(tk.tokens[i], i)
    be.synchronize()
    out = []
    L = bench.MODELS[args.model]["L"]
    for t in range(args.tokens):
        # stamps are overwritten by every layer launch: run the layers eagerly up to the
        # middle one by the graph, then read (the last launch of the token is the head, not
        # a layer: the buffer holds the LAST layer's stamps)
        buf.zero_()
        torch.cuda.synchronize()
        assert g.lib().mi355x_diag_stamps(buf.data_ptr(), buf.numel() * 8) == 0
        tk.dec.step(tk.tokens[4 + t], 4 + t, use_graph=False)
        be.synchronize()
        g.lib().mi355x_diag_stamps(None, 0)
        full = buf.cpu().numpy().reshape(G, 32).astype(np.int64)
        s = full[:, :19]
        t0 = s[:, 0][s[:, 0] > 0].min()
        rel = np.where(s > 0, (s - t0) / 100.0, np.nan)  # 100 MHz -> us
        row = {}
        for i, nm in enumerate(NAMES):
            col = rel[:, i]
            col = col[~np.isnan(col)]
            if col.size:
                row[nm] = (round(float(np.median(col)), 2), round(float(col.max()), 2), int(col.size))
        # slots 20..31: stream wave 0's first 12 gate/up steps (start of each)
        st = full[:, 20:32].astype(np.float64)
        d = np.diff(np.where(st > 0, st, np.nan), axis=1) / 100.0
        row["gate/up step us"] = [round(float(v), 3) for v in np.nanmedian(d, axis=0)] if np.isfinite(d).any() else []
        out.append(row)
    assert be.layer_error() == 0
    print(json.dumps({"model": args.model, "layers": L, "note": "last layer of each eager token; (median, max, n) us",
                      "tokens": out}))
    for nm in NAMES:
        vals = [r.get(nm) for r in out if r.get(nm)]
        if vals:
            med = np.median([v[0] for v in vals])
            mx = np.median([v[1] for v in vals])
            print(f"{nm:8s} median {med:7.2f} us   max {mx:7.2f} us   (workgroups {vals[0][2]})")
    print("gate/up per-step (stream wave 0, median over workgroups):", out[-1].get("gate/up step us"))


if __name__ == "__main__":
    main()
