"""The bench's synthetic workload matches SURVEY.md §8d (CPU only): the Q4_K_M type
mix of llama-quant.cpp [U] (use_more_bits layers: attn_v / ffn_down Q6_K; output
Q6_K) and the per-token weight bytes the roofline and tok/s figures are quoted on."""
import pytest

import bench
import ggml_mi355x as g


def _bytes(model):
    return sum(N * (K // 256) * g.BLOCK_BYTES[t] for stage in bench.q4km_chain(model) for _, t, K, N in stage)


@pytest.mark.parametrize("model,mb,more_bits", [("tinyllama-1.1b", 629.8, 10), ("llama-3-8b", 4616.3, 16),
                                                ("llama-3-70b", 41916.3, 40)])
def test_q4km_mix_bytes_and_more_bits_layers(model, mb, more_bits):
    L = bench.MODELS[model]["L"]
    assert sum(bench.use_more_bits(i, L) for i in range(L)) == more_bits
    assert round(_bytes(model) / 1e6, 1) == mb


def test_tinyllama_type_mix():
    """attn_v / ffn_down are Q6_K exactly in the use_more_bits layers, the output head is
    Q6_K, every other matrix Q4_K, at the real TinyLlama shapes (K -> N)."""
    types = {}
    for stage in bench.q4km_chain("tinyllama-1.1b"):
        for name, t, K, N in stage:
            types[name] = (t, K, N)
    L = bench.MODELS["tinyllama-1.1b"]["L"]
    for i in range(L):
        q6 = bench.use_more_bits(i, L)
        assert types[f"blk.{i}.attn_v"] == (g.TYPE_Q6_K if q6 else g.TYPE_Q4_K, 2048, 256)
        assert types[f"blk.{i}.ffn_down"] == (g.TYPE_Q6_K if q6 else g.TYPE_Q4_K, 5632, 2048)
        assert types[f"blk.{i}.attn_q"] == (g.TYPE_Q4_K, 2048, 2048)
        assert types[f"blk.{i}.ffn_gate"] == (g.TYPE_Q4_K, 2048, 5632)
    assert types["output"] == (g.TYPE_Q6_K, 2048, 32000)


def test_tinyllama_model_size_matches_published():
    """llama-bench reports the TinyLlama-1.1B Q4_K_M model as 636.18 MiB (README.md:192,
    the sum of ggml_nbytes over every tensor). The bench's mix — the matmul chain, the
    Q4_K token_embd and the f32 norms (2 per layer + output_norm) — must reproduce it
    within the print's rounding and a 6 KB residual (667,078,656 B = 636.174 MiB)."""
    m = bench.MODELS["tinyllama-1.1b"]
    E, L, V = m["E"], m["L"], m["V"]
    total = _bytes("tinyllama-1.1b")                      # every MUL_MAT weight incl. output
    total += V * (E // 256) * g.BLOCK_BYTES[g.TYPE_Q4_K]  # token_embd (Q4_K)
    total += (2 * L + 1) * E * 4                          # attn_norm, ffn_norm, output_norm (f32)
    mib = total / 2 ** 20
    assert abs(mib - 636.18) <= 0.01, mib


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_multi_gpu_headline_is_the_row_split(world):
    """at N > 1 the driver's scaling line measures the north_star's row-split
    path (one TinyLlama token stream, reduce schedule, strong scaling), not replicas; at
    N = 1 the line stays one stream on one GPU. Explicit --mode values are kept."""
    m = bench.resolve_mode("auto", world)
    h = bench.headline_fields(m, world)
    if world == 1:
        assert m == "replicas" and h == {"scaling": "weak", "parallelism": "replicas x1", "tokens_per_step": 1}
    else:
        assert m == "rowsplit-reduce"
        assert h == {"scaling": "strong", "parallelism": f"rowsplit-reduce{world}", "tokens_per_step": 1}
    assert bench.resolve_mode("replicas", world) == "replicas"
    assert bench.headline_fields("replicas", world)["tokens_per_step"] == world
    assert bench.headline_fields("rowsplit", world)["parallelism"] == f"rowsplit-gather{world}"
