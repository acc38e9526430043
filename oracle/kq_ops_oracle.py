"""ctypes binding of the decode-op oracle (oracle/kq_ops_oracle.c) and the CPU
restatement of one llama decode token (llm_build_llama, out.folded:249-251).

TEST INFRASTRUCTURE ONLY — the checker used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg. The product package never imports this.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import kq_oracle as KO

_bound = False


def lib():
    global _bound
    L = KO.lib()
    if not _bound:
        vp, i64, i32, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
        u16 = ctypes.c_uint16
        L.kqo_f16_fma.argtypes = [u16, u16, u16]
        L.kqo_f16_fma.restype = u16
        L.kqo_f16_add.argtypes = [u16, u16]
        L.kqo_f16_add.restype = u16
        L.kqo_fp32_to_fp16_row.argtypes = [vp, vp, i64]
        L.kqo_vec_dot_f16.argtypes = [i32, vp, vp]
        L.kqo_vec_dot_f16.restype = f32
        L.kqo_v_expf.argtypes = [f32]
        L.kqo_v_expf.restype = f32
        L.kqo_vec_swiglu_f32.argtypes = [i32, vp, vp, vp]
        L.kqo_soft_max_row.argtypes = [i32, vp, vp, vp, f32]
        L.kqo_rms_norm_f32.argtypes = [vp, vp, i64, f32]
        L.kqo_mul_f32.argtypes = [vp, vp, vp, i64]
        L.kqo_add_f32.argtypes = [vp, vp, vp, i64]
        L.kqo_rope_theta_scale.argtypes = [f32, i32]
        L.kqo_rope_theta_scale.restype = f32
        L.kqo_rope_table.argtypes = [vp, i32, i32, f32, f32]
        L.kqo_rope_norm.argtypes = [vp, vp, i32, i32, i32, i32, vp]
        L.kqo_get_rows.argtypes = [i32, vp, i64, ctypes.c_size_t, vp, i64, vp]
        L.kqo_attn_n_kv.argtypes = [i32, i32]
        L.kqo_attn_n_kv.restype = i32
        L.kqo_attn_decode.argtypes = [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, f32, vp]
        L.kqo_attn_decode_fast.argtypes = [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, f32, vp, i32]
        L.kqo_f16_fma_fast.argtypes = [u16, u16, u16]
        L.kqo_f16_fma_fast.restype = u16
        L.kqo_f16_fast_check.argtypes = [ctypes.c_long, ctypes.c_uint64]
        L.kqo_f16_fast_check.restype = ctypes.c_long
        _bound = True
    return L


_p = KO._p


def _f32(a):
    return np.ascontiguousarray(a, np.float32)


def f16_fma(a: int, b: int, c: int) -> int:
    return lib().kqo_f16_fma(a, b, c)


def f16_add(a: int, b: int) -> int:
    return lib().kqo_f16_add(a, b)


def fp32_to_fp16(x):
    x = _f32(x)
    y = np.empty(x.shape, np.uint16)
    lib().kqo_fp32_to_fp16_row(_p(x), _p(y), x.size)
    return y


def vec_dot_f16(x16, y16) -> float:
    x16 = np.ascontiguousarray(x16, np.uint16)
    y16 = np.ascontiguousarray(y16, np.uint16)
    return np.float32(lib().kqo_vec_dot_f16(x16.size, _p(x16), _p(y16)))


def v_expf(x) -> np.ndarray:
    x = _f32(x).ravel()
    return np.array([lib().kqo_v_expf(float(v)) for v in x], np.float32)


def swiglu(x, g):
    x, g = _f32(x), _f32(g)
    y = np.empty_like(x)
    lib().kqo_vec_swiglu_f32(x.size, _p(y), _p(x), _p(g))
    return y


def soft_max_row(s, mask=None, scale=1.0):
    s = _f32(s)
    d = np.empty_like(s)
    m = _f32(mask) if mask is not None else None
    lib().kqo_soft_max_row(s.size, _p(d), _p(s), _p(m) if m is not None else None, scale)
    return d


def rms_norm(x, eps):
    x = _f32(x)
    y = np.empty_like(x)
    for r in range(x.shape[0] if x.ndim == 2 else 1):
        xr = x[r] if x.ndim == 2 else x
        yr = y[r] if y.ndim == 2 else y
        lib().kqo_rms_norm_f32(_p(xr), _p(yr), xr.size, eps)
    return y


def mul(a, b):
    a, b = _f32(a), _f32(b)
    y = np.empty_like(a)
    lib().kqo_mul_f32(_p(a), _p(b), _p(y), a.size)
    return y


def add(a, b):
    a, b = _f32(a), _f32(b)
    y = np.empty_like(a)
    lib().kqo_add_f32(_p(a), _p(b), _p(y), a.size)
    return y


def rope_table(n_pos, n_dims, freq_base=10000.0, freq_scale=1.0):
    t = np.empty((n_pos, n_dims // 2, 2), np.float32)
    lib().kqo_rope_table(_p(t), n_pos, n_dims, freq_base, freq_scale)
    return t


def rope(x, head_dim, n_dims, pos, table):
    x = _f32(x)
    y = np.empty_like(x)
    lib().kqo_rope_norm(_p(x), _p(y), head_dim, n_dims, x.size // head_dim, pos, _p(np.ascontiguousarray(table)))
    return y


def get_rows(type_, table, k, ids):
    table = np.ascontiguousarray(table)
    ids = np.ascontiguousarray(ids, np.int32)
    out = np.empty((ids.size, k), np.float32)
    row_stride = table.strides[0] if table.ndim == 2 else k * 4
    lib().kqo_get_rows(type_, _p(table), k, row_stride, _p(ids), ids.size, _p(out))
    return out


def attn_n_kv(pos, n_ctx):
    return lib().kqo_attn_n_kv(pos, n_ctx)


def attn_decode(q, k, v, k_cache, v_cache, pos, n_head, n_head_kv, head_dim, scale, fast_threads=0):
    """Updates k_cache ([n_ctx, n_head_kv*hd] u16) and v_cache ([n_head_kv*hd, n_ctx] u16) in place.
    fast_threads > 0: the CPU-baseline form (kq_cpu_simd.c: double-based binary16 ops,
    heads over the worker pool), bit-identical to the restatement."""
    q, k, v = _f32(q), _f32(k), _f32(v)
    assert k_cache.flags.c_contiguous and v_cache.flags.c_contiguous
    out = np.empty(n_head * head_dim, np.float32)
    n_ctx = k_cache.shape[0]
    if fast_threads > 0:
        lib().kqo_attn_decode_fast(_p(q), _p(k), _p(v), _p(k_cache), _p(v_cache), pos, n_ctx, n_head, n_head_kv,
                                   head_dim, scale, _p(out), fast_threads)
    else:
        lib().kqo_attn_decode(_p(q), _p(k), _p(v), _p(k_cache), _p(v_cache), pos, n_ctx, n_head, n_head_kv,
                              head_dim, scale, _p(out))
    return out


# ------------------------------------------------------------ one decode token
def decode_token(model, token, pos, cache, n_threads=8, variant="neon", full_trace=None):
    """The llama graph for one token (llm_build_llama, non-flash attention), ggml-cpu
    semantics op by op: get_rows -> [rms_norm*attn_norm -> q/k/v mul_mat -> rope ->
    attention -> wo mul_mat -> add -> rms_norm*ffn_norm -> gate/up mul_mat -> swiglu ->
    down mul_mat -> add] x n_layer -> rms_norm*output_norm -> output mul_mat.
    `model`: dict as built by tests/llama_model.py; `cache`: list of (k_cache, v_cache)
    per layer, updated in place. `variant`: the vec_dot form of the matmuls ("neon"
    scalar, or "simd": AVX2 integer parts, bit-identical). Returns (logits,
    per-layer residual outputs). `full_trace` (a list) receives per layer a dict of
    the attention output, ffn_inp, the swiglu output and the layer output."""
    hp = model["hp"]
    E, hd = hp["n_embd"], hp["head_dim"]
    eps = hp["eps"]
    t, w = model["tok_embd"]
    x = get_rows(t, w, E, [token])[0]
    table = model["rope_table"]
    scale = np.float32(1.0) / np.sqrt(np.float32(hd))
    trace = []
    for li, L in enumerate(model["layers"]):
        inp = x
        cur = mul(rms_norm(x, eps), L["attn_norm"])
        q = KO.mul_mat(L["wq"][0], L["wq"][1], cur, n_threads, variant)[0]
        k = KO.mul_mat(L["wk"][0], L["wk"][1], cur, n_threads, variant)[0]
        v = KO.mul_mat(L["wv"][0], L["wv"][1], cur, n_threads, variant)[0]
        q = rope(q, hd, hd, pos, table)
        k = rope(k, hd, hd, pos, table)
        kc, vc = cache[li]
        att = attn_decode(q, k, v, kc, vc, pos, hp["n_head"], hp["n_head_kv"], hd, float(scale),
                          fast_threads=n_threads if variant == "simd" else 0)
        cur = KO.mul_mat(L["wo"][0], L["wo"][1], att, n_threads, variant)[0]
        ffn_inp = add(cur, inp)
        cur = mul(rms_norm(ffn_inp, eps), L["ffn_norm"])
        g = KO.mul_mat(L["w_gate"][0], L["w_gate"][1], cur, n_threads, variant)[0]
        u = KO.mul_mat(L["w_up"][0], L["w_up"][1], cur, n_threads, variant)[0]
        glu = swiglu(g, u)
        cur = KO.mul_mat(L["w_down"][0], L["w_down"][1], glu, n_threads, variant)[0]
        x = add(cur, ffn_inp)
        trace.append(x)
        if full_trace is not None:
            full_trace.append({"att": att, "ffn_inp": ffn_inp, "glu": glu, "x": x})
    cur = mul(rms_norm(x, eps), model["output_norm"])
    logits = KO.mul_mat(model["output"][0], model["output"][1], cur, n_threads, variant)[0]
    return logits, trace
