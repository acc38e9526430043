"""Generates tests/golden/*.npz: seeded synthetic K-quant rows, f32 activations,
their Q8_K quantization and the expected mul_mat outputs / integer partials,
computed by the C oracle (oracle/kq_oracle.c) and cross-checked bit-for-bit
against the independent numpy restatement (oracle/kq_oracle_np.py) before saving.

The reference ships no fixtures for this path (parity unpinned),
so these are this repo's own golden vectors. Regenerate with:
    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import kq_oracle as O  # noqa: E402
from oracle import kq_oracle_np as N  # noqa: E402

CASES = [
    # (name, type, K, N, M, seed)
    ("q4K_k256_n16_m2", 12, 256, 16, 2, 1),
    ("q4K_k2048_n16_m2", 12, 2048, 16, 2, 2),
    ("q4K_k5632_n8_m1", 12, 5632, 8, 1, 3),
    ("q5K_k2048_n16_m2", 13, 2048, 16, 2, 4),
    ("q6K_k2048_n16_m2", 14, 2048, 16, 2, 5),
    ("q6K_k768_n9_m3", 14, 768, 9, 3, 6),
]


def edge_activations(rng, M, K):
    x = rng.standard_normal((M, K)).astype(np.float32)
    # block 0 of column 0: all zero (the !amax branch)
    x[0, :256] = 0
    if K >= 512:
        # block 1: a +/- tie for the max magnitude (first index must win)
        x[0, 256:512] = rng.uniform(-1, 1, 256).astype(np.float32)
        x[0, 300] = -3.0
        x[0, 400] = 3.0
    if M > 1:
        # column 1: upstream-style 0.1 + 2cos(i) data (tests/test-quantize-fns.cpp [U])
        x[1] = (0.1 + 2 * np.cos(np.arange(K) + 1.0)).astype(np.float32)
    return x


def main():
    manifest = {}
    for name, t, K, Nr, M, seed in CASES:
        rng = np.random.default_rng(seed)
        w = N.random_blocks(rng, t, Nr, K)
        x = edge_activations(rng, M, K)
        q8 = O.quantize_q8_K(x)
        q8n = N.q8_K_to_bytes(N.quantize_q8_K(x))
        assert (q8 == q8n).all(), name
        dst = O.mul_mat(t, w, x)
        dstn = N.mul_mat_q8(w, t, K, N.q8_K_from_bytes(q8, K // 256))
        assert (dst.view(np.uint32) == dstn.view(np.uint32)).all(), name
        parts = np.stack([O.block_partials(t, w, q8[j], K) for j in range(M)])
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, type=np.int32(t), K=np.int32(K), w=w, x=x, q8=q8, dst=dst, partials=parts)
        manifest[name] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    # quantizer edge cases (one block each)
    rng = np.random.default_rng(99)
    rows = [
        np.zeros(256, np.float32),
        np.full(256, 1e-40, np.float32),                  # subnormal inputs
        np.where(np.arange(256) % 2 == 0, 1.0, -1.0).astype(np.float32),  # all ties, first is +
        np.where(np.arange(256) % 2 == 0, -1.0, 1.0).astype(np.float32),  # all ties, first is -
        rng.uniform(-1e30, 1e30, 256).astype(np.float32),
        (rng.integers(-127, 128, 256) * np.float32(0.5)).astype(np.float32),  # .5 boundaries after scaling
        np.linspace(-1, 1, 256, dtype=np.float32),
    ]
    xq = np.stack(rows)
    q8 = O.quantize_q8_K(xq)
    assert (q8 == N.q8_K_to_bytes(N.quantize_q8_K(xq))).all()
    q8u = O.quantize_q8_K(xq, fused=False)
    path = os.path.join(HERE, "q8K_edges.npz")
    np.savez_compressed(path, x=xq, q8=q8, q8_unfused=q8u)
    manifest["q8K_edges"] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
