"""Three graph-replayed 512-token prompts of `model` (after a capture run): the command
tools/prof_prompt.sh traces."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from bench import Token  # noqa: E402
from ggml_mi355x.llama import LlamaDecoder  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "tinyllama-1.1b"
dev = torch.device("cuda:0")
be = g.Backend()
tk = Token(model, dev, 0x51A7, be, 128)
dec = LlamaDecoder(be, tk.hp, tk.w, 512)
toks = np.random.default_rng(1).integers(0, tk.hp["n_vocab"], size=512).tolist()
for _ in range(4):
    dec.prompt(toks, 0)
be.synchronize()
print("ok", model)
