"""Prompt graph on the f16 GEMMs: fused (multi-matrix launches, ADD epilogue) against
unfused and against the exact path, per layer cache and logits (diagnostics)."""
import os
import sys

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "ggml-neon-opt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from tests.test_gpu_ops import _decoder  # noqa: E402
from ggml_mi355x.llama import hparams  # noqa: E402

dev = torch.device("cuda:0")
hp = hparams(2048, 2, 32, 4, 5632, 4096)
tokens = np.random.default_rng(13).integers(0, hp["n_vocab"], size=37).tolist()
res = {}
for name, f16, fuse in (("exact", 0, True), ("f16_fused", 1, True), ("f16_unfused", 1, False)):
    g.prefill_precision(f16)
    w, b, dec = _decoder(dev, hp, 7, 64, fuse)
    lg = dec.prompt(tokens, 0)
    b.synchronize()
    res[name] = [lg.cpu().numpy().astype(np.float64).ravel().copy()]
    for i in range(2):
        res[name].append(dec.k_cache[i][:37].view(torch.float16).float().cpu().numpy())
        res[name].append(dec.v_cache[i].view(torch.float16).float().cpu().numpy())
    b.close()
g.prefill_precision(0)


def rel(a, c):
    return float(np.linalg.norm(a - c) / max(np.linalg.norm(c), 1e-30))


names = ["logits", "k0", "v0", "k1", "v1"]
for a, c in (("f16_fused", "f16_unfused"), ("f16_fused", "exact"), ("f16_unfused", "exact")):
    print(a, "vs", c, " ".join(f"{n} {rel(x, y):.3e}" for n, x, y in zip(names, res[a], res[c])))
