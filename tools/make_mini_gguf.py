"""Writes a small llama-architecture Q4_K_M-style GGUF file (tests/gguf_writer.py)
for exercising `bench.py --gguf` without a downloaded model:
    python tools/make_mini_gguf.py OUT.gguf [E L KV FF V]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

from gguf_writer import mini_llama  # noqa: E402
from oracle import kq_oracle_np as npo  # noqa: E402

if __name__ == "__main__":
    dims = [int(v) for v in sys.argv[2:7]] or [512, 2, 256, 1024, 1000]
    E, L, KV, FF, V = dims
    mini_llama(sys.argv[1], np.random.default_rng(0), npo, E=E, L=L, KV=KV, FF=FF, V=V)
    print(f"wrote {sys.argv[1]} ({os.path.getsize(sys.argv[1]) / 1e6:.1f} MB)")
