import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "ggml-neon-opt_amd")]
import numpy as np, torch
import ggml_mi355x as g
from tests import llama_model as LM
from tests.test_gpu_ops import _decoder
from ggml_mi355x.llama import hparams
from oracle import kq_ops_oracle as O
O.lib()
dev = torch.device("cuda:0")
hp = hparams(2048, 2, 32, 4, 5632, 4096)
tokens = np.random.default_rng(13).integers(0, hp["n_vocab"], size=37).tolist()
res = {}
for name, f16, fuse in (("exact", 0, True), ("f16_fused", 1, True), ("f16_unfused", 1, False)):
    g.prefill_precision(f16)
    w, b, dec = _decoder(dev, hp, 7, 64, fuse)
    lg = dec.prompt(tokens, 0); b.synchronize()
    res[name] = lg.cpu().numpy().astype(np.float64).ravel().copy()
    res[name + "_k0"] = dec.k_cache[0][:37].view(torch.float16).float().cpu().numpy()
    res[name + "_k1"] = dec.k_cache[1][:37].view(torch.float16).float().cpu().numpy()
    b.close()
g.prefill_precision(0)
model, cache = LM.oracle_model(hp, w, 64)
for p, tok in enumerate(tokens):
    ref, _ = O.decode_token(model, tok, p, cache)
ref = np.asarray(ref, np.float64).ravel()
def rel(a, b): return float(np.linalg.norm(a - b) / np.linalg.norm(b))
for n in ("exact", "f16_fused", "f16_unfused"):
    print(n, "logits rel vs oracle", rel(res[n], ref), "k0 rel vs exact", rel(res[n + "_k0"], res["exact_k0"]), "k1", rel(res[n + "_k1"], res["exact_k1"]))
print("fused vs unfused logits", rel(res["f16_fused"], res["f16_unfused"]))
print("max |logit|", np.abs(ref).max(), "argmax eq", int(np.argmax(ref)) == int(np.argmax(res["f16_fused"])))
