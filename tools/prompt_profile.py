"""Per-kernel time of one prompt batch through the graph (eager, launch-timing hook):
where pp512 goes beyond the GEMMs. usage: python tools/prompt_profile.py [model] [n_tok]"""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from bench import Token  # noqa: E402
from ggml_mi355x.llama import LlamaDecoder  # noqa: E402


def main(model="tinyllama-1.1b", n_tok=512):
    dev = torch.device("cuda:0")
    be = g.Backend()
    tk = Token(model, dev, 0x51A7, be, 128)
    dec = LlamaDecoder(be, tk.hp, tk.w, n_tok)
    toks = np.random.default_rng(1).integers(0, tk.hp["n_vocab"], size=n_tok).tolist()
    dec.prompt(toks, 0, use_graph=False)
    be.synchronize()
    g.timing_enable(True)
    dec.prompt(toks, 0, use_graph=False)
    be.synchronize()
    rows = g.timing_read()
    g.timing_enable(False)
    agg = defaultdict(lambda: [0, 0.0])
    for name, _, ms in rows:
        agg[name][0] += 1
        agg[name][1] += ms
    tot = sum(v[1] for v in agg.values())
    for name, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{name:32s} {n:5d} launches {ms * 1e3:10.1f} us  {ms / tot * 100:5.1f} %")
    print(f"{'total':32s} {len(rows):5d} launches {tot * 1e3:10.1f} us")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "tinyllama-1.1b", int(sys.argv[2]) if len(sys.argv) > 2 else 512)
