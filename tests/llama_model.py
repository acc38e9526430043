"""Synthetic llama models for the decode-graph tests: host (numpy) weights for the CPU
oracle and the same bytes on the device for ggml_mi355x.llama.LlamaDecoder.

Q4_K_M type mix [U] (llama-quant.cpp): attn_v / ffn_down Q6_K in the
use_more_bits layers, output Q6_K, every other matrix (token_embd too) Q4_K. Block
scales keep the activation RMS O(1) down the layers (d ~ 1/sqrt(K * E[w^2]/d^2),
dmin = d * mean quant)."""
from __future__ import annotations

import numpy as np

Q4_K, Q5_K, Q6_K = 12, 13, 14
W2 = {Q4_K: 66727.0, Q5_K: 277630.0, Q6_K: 1.865e6}
BB = {Q4_K: 144, Q5_K: 176, Q6_K: 210}


def use_more_bits(i, n):
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def kquant(rng, type_, N, K, rms_keep=True):
    nb = K // 256
    B = BB[type_]
    raw = rng.integers(0, 256, size=(N, nb, B), dtype=np.uint8)
    if rms_keep:
        d = rng.uniform(0.75, 1.25, size=(N, nb)) / np.sqrt(1.0208 * K * W2[type_])
    else:
        d = rng.uniform(2.0 ** -14, 2.0 ** -6, size=(N, nb))
    dh = d.astype(np.float16).view(np.uint8).reshape(N, nb, 2)
    if type_ in (Q4_K, Q5_K):
        dmin = (d * (7.5 if type_ == Q4_K else 15.5)) if rms_keep else rng.uniform(2.0 ** -14, 2.0 ** -6, size=(N, nb))
        raw[..., 0:2] = dh
        raw[..., 2:4] = dmin.astype(np.float16).view(np.uint8).reshape(N, nb, 2)
    else:
        raw[..., 208:210] = dh
    return raw.reshape(N, nb * B)


def build(hp, seed=0, v_type=Q4_K, mix="q4_k_m"):
    """Host weights: dict name -> (type, uint8 array) for matrices, f32 arrays for norms.
    v_type: attn_v outside the use_more_bits layers (Q4_K; Q5_K in Llama-3-70B's
    Q4_K_M mix). mix "q5_k_m": llama-quant.cpp's Q5_K_M [U] — every
    matrix Q5_K (token_embd too) except attn_v / ffn_down of the use_more_bits layers and
    the output, Q6_K (BASELINE config 5)."""
    rng = np.random.default_rng(seed)
    E, F, V, L = hp["n_embd"], hp["n_ff"], hp["n_vocab"], hp["n_layer"]
    kvw = hp["n_head_kv"] * hp["head_dim"]
    base = Q5_K if mix == "q5_k_m" else Q4_K
    if mix == "q5_k_m":
        v_type = Q5_K
    w = {"token_embd": (base, kquant(rng, base, V, E, rms_keep=False)),
         "output": (Q6_K, kquant(rng, Q6_K, V, E)),
         "output_norm": rng.uniform(0.8, 1.2, E).astype(np.float32)}
    for i in range(L):
        p = f"blk.{i}."
        mb = use_more_bits(i, L)
        w[p + "attn_norm"] = rng.uniform(0.8, 1.2, E).astype(np.float32)
        w[p + "ffn_norm"] = rng.uniform(0.8, 1.2, E).astype(np.float32)
        w[p + "attn_q"] = (base, kquant(rng, base, E, E))
        w[p + "attn_k"] = (base, kquant(rng, base, kvw, E))
        vt = Q6_K if mb else v_type
        w[p + "attn_v"] = (vt, kquant(rng, vt, kvw, E))
        w[p + "attn_output"] = (base, kquant(rng, base, E, E))
        w[p + "ffn_gate"] = (base, kquant(rng, base, F, E))
        w[p + "ffn_up"] = (base, kquant(rng, base, F, E))
        dt = Q6_K if mb else base
        w[p + "ffn_down"] = (dt, kquant(rng, dt, E, F))
    return w


def to_device(w, dev):
    import torch
    out = {}
    for k, v in w.items():
        if isinstance(v, tuple):
            out[k] = (v[0], torch.from_numpy(v[1]).to(dev))
        else:
            out[k] = torch.from_numpy(v).to(dev)
    return out


def oracle_model(hp, w, n_ctx):
    """The dict oracle/kq_ops_oracle.decode_token expects (+ a fresh zero KV cache)."""
    from oracle import kq_ops_oracle as O
    layers = []
    for i in range(hp["n_layer"]):
        p = f"blk.{i}."
        layers.append({"attn_norm": w[p + "attn_norm"], "ffn_norm": w[p + "ffn_norm"], "wq": w[p + "attn_q"],
                       "wk": w[p + "attn_k"], "wv": w[p + "attn_v"], "wo": w[p + "attn_output"],
                       "w_gate": w[p + "ffn_gate"], "w_up": w[p + "ffn_up"], "w_down": w[p + "ffn_down"]})
    model = {"hp": hp, "tok_embd": w["token_embd"], "output": w["output"], "output_norm": w["output_norm"],
             "layers": layers, "rope_table": O.rope_table(n_ctx, hp["head_dim"], hp["freq_base"])}
    kvw = hp["n_head_kv"] * hp["head_dim"]
    cache = [(np.zeros((n_ctx, kvw), np.uint16), np.zeros((kvw, n_ctx), np.uint16)) for _ in range(hp["n_layer"])]
    return model, cache
