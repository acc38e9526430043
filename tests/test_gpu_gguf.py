"""GPU: weights loaded from a GGUF file (native reader, mi355x_gguf_upload — bytes
unchanged) drive the decode GEMV and the prefill GEMM bit-exactly against the
oracle on the same file bytes."""
import numpy as np
import pytest

from gguf_writer import mini_llama
from test_gpu_parity import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu


def test_gguf_tensors_through_the_kernels(dev, oracle, npo, tmp_path):
    import torch
    import ggml_mi355x as g
    import ggml_mi355x.gguf as G
    path = tmp_path / "mini.gguf"
    mini_llama(path, np.random.default_rng(11), npo)
    rng = np.random.default_rng(12)
    with G.GGUFFile(path) as f:
        checked = 0
        for name, info in f.tensors.items():
            if info["type"] not in (12, 13, 14) or len(info["ne"]) != 2:
                continue
            K, N = info["ne"]
            w = f.to_device(name, dev)
            torch.cuda.synchronize()
            host = f.bytes(name).reshape(N, -1)
            assert np.array_equal(w.cpu().numpy(), host)
            for M in (1, 16):
                x = rng.standard_normal((M, K)).astype(np.float32)
                y = g.mul_mat(info["type"], w, K, torch.from_numpy(x).to(dev)).cpu().numpy()
                want = oracle.mul_mat(info["type"], host, x)
                assert bits_equal(y, want), (name, M, first_mismatch(y, want))
            checked += 1
        assert checked == 2 + 2 * 7  # token_embd, output, 7 matrices per layer
