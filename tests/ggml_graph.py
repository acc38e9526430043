"""llm_build_llama's decode graph (one token, KV cache, non-flash attention) as the
ggml_tensor mirror a ggml backend adapter hands to mi355x_lower_ggml_graph — test
infrastructure. Restated from llama.cpp [U] (llama-model.cpp llm_build_llama,
llama-graph.cpp build_norm / build_attn / build_attn_mha / build_ffn, llama-kv-cache
cpy_k / cpy_v / get_k / get_v) in its ggml_build_forward_expand order: build_attn
expands q_cur, k_cur, v_cur, then the two cache stores, then the attention product.
"""
from __future__ import annotations

import ctypes

import numpy as np

import ggml_mi355x as g

F32, F16, I32, I64 = 0, 1, 26, 27
ELT = {F32: 4, F16: 2, I32: 4, I64: 8}


def f32_bits(v):
    return int(np.array([v], np.float32).view(np.int32)[0])


class Graph:
    """Tensors are GTensor structs; `nodes` is the cgraph's node list (graph order)."""

    def __init__(self, alloc=None):
        """alloc(nbytes) -> device pointer for node outputs (None: distinct fake addresses)."""
        self.keep, self.nodes = [], []
        self._fake = 0x7f0000000000
        self._alloc = alloc

    def _new(self, type_, ne, nb=None, data=None, op=g.GOP_NONE, srcs=(), params=(), view_src=None, flags=0,
             name=""):
        t = g.GTensor()
        t.type, t.op = type_, op
        ne = list(ne) + [1] * (4 - len(ne))
        for d in range(4):
            t.ne[d] = ne[d]
        if nb is None:
            if type_ in g.BLOCK_BYTES:
                nb0 = g.BLOCK_BYTES[type_]
                nb = [nb0, ne[0] // 256 * nb0]
            else:
                nb = [ELT[type_], ne[0] * ELT[type_]]
            nb = nb + [nb[-1] * ne[1], nb[-1] * ne[1] * ne[2]]
        for d in range(4):
            t.nb[d] = nb[d]
        for i, s in enumerate(srcs):
            t.src[i] = ctypes.pointer(s) if s is not None else ctypes.POINTER(g.GTensor)()
        for i, p in enumerate(params):
            t.op_params[i] = p
        if view_src is not None:
            t.view_src = ctypes.pointer(view_src)
        if data is None:  # a node output: a buffer of its own (ggml-alloc's)
            if self._alloc is not None:
                data = self._alloc(int(np.prod(ne)) * ELT.get(type_, 4))
            else:
                self._fake += 1 << 20
                data = self._fake
        t.data = data
        t.flags = flags
        t.name = name.encode()[:63]
        self.keep.append(t)
        return t

    def leaf(self, type_, ne, data, nb=None, name=""):
        return self._new(type_, ne, nb=nb, data=data, name=name)

    def node(self, op, type_, ne, srcs, params=(), view_src=None, flags=0, name="", data=None):
        t = self._new(type_, ne, data=data, op=op, srcs=srcs, params=params, view_src=view_src, flags=flags,
                      name=name)
        self.nodes.append(t)
        return t

    def alias(self, op, src, ne, nb=None):
        """RESHAPE / VIEW / PERMUTE / TRANSPOSE: a view of src (same data)."""
        return self.node(op, src.type, ne, [src], view_src=src, data=src.data)


def rope_params(n_dims, freq_base, freq_scale=1.0, n_ctx_orig=0):
    p = [0, n_dims, 0, 0, n_ctx_orig]  # n_past, n_dims, mode (NORMAL), n_ctx, n_ctx_orig
    p += [f32_bits(freq_base), f32_bits(freq_scale), f32_bits(0.0), f32_bits(1.0), f32_bits(32.0), f32_bits(1.0)]
    return p


def llama_decode_graph(hp, L, n_ctx, alloc=None, n_tokens=1):
    """hp: ggml_mi355x.llama.hparams; L: leaf data pointers — "token_embd", "output",
    "output_norm", "blk.i.<mat|norm>" -> (type, ne0, ne1, data, row_bytes) / (data,),
    "k_cache.i" / "v_cache.i" -> data, "inp_tokens", "inp_pos", "kq_mask" (and
    "inp_out_ids" for n_tokens > 1). n_tokens > 1: a prompt ubatch whose logits are wanted
    for its last token only (llm_build_llama's inp_out_ids GET_ROWS after the last layer's
    attention). Returns Graph."""
    G = Graph(alloc)
    E, V, hd, nh, nkv = hp["n_embd"], hp["n_vocab"], hp["head_dim"], hp["n_head"], hp["n_head_kv"]
    kvw = nkv * hd
    eps = f32_bits(hp["eps"])
    T = n_tokens

    def mat(name):
        t, ne0, ne1, data, rb = L[name]
        return G.leaf(t, [ne0, ne1], data, nb=[g.BLOCK_BYTES[t], rb, rb * ne1, rb * ne1], name=name)

    def vec(name, n):
        return G.leaf(F32, [n], L[name], name=name)

    tok = G.leaf(I32, [T], L["inp_tokens"], name="inp_tokens")
    pos = G.leaf(I32, [T], L["inp_pos"], name="inp_pos")
    mask = G.leaf(F16, [n_ctx, T], L["kq_mask"], name="kq_mask")
    out_ids = G.leaf(I32, [1], L["inp_out_ids"], name="inp_out_ids") if T > 1 else None
    inpL = G.node(g.GOP_GET_ROWS, F32, [E, T], [mat("token_embd"), tok], name="inp_embd")
    scale = f32_bits(np.float32(1.0) / np.sqrt(np.float32(hd)))
    for il in range(hp["n_layer"]):
        p = f"blk.{il}."
        inpSA = inpL
        cur = G.node(g.GOP_RMS_NORM, F32, [E, T], [inpL], [eps], name="norm")
        cur = G.node(g.GOP_MUL, F32, [E, T], [cur, vec(p + "attn_norm", E)], name="attn_norm")
        q = G.node(g.GOP_MUL_MAT, F32, [nh * hd, T], [mat(p + "attn_q"), cur], name="Qcur")
        q = G.alias(g.GOP_RESHAPE, q, [hd, nh, T])
        q = G.node(g.GOP_ROPE, F32, [hd, nh, T], [q, pos], rope_params(hd, hp["freq_base"]), name="Qcur_rope")
        k = G.node(g.GOP_MUL_MAT, F32, [kvw, T], [mat(p + "attn_k"), cur], name="Kcur")
        k = G.alias(g.GOP_RESHAPE, k, [hd, nkv, T])
        k = G.node(g.GOP_ROPE, F32, [hd, nkv, T], [k, pos], rope_params(hd, hp["freq_base"]), name="Kcur_rope")
        v = G.node(g.GOP_MUL_MAT, F32, [kvw, T], [mat(p + "attn_v"), cur], name="Vcur")
        v = G.alias(g.GOP_RESHAPE, v, [hd, nkv, T])
        kc = G.leaf(F16, [kvw, n_ctx], L[f"k_cache.{il}"], name=f"cache_k_l{il}")
        vc = G.leaf(F16, [n_ctx, kvw], L[f"v_cache.{il}"], name=f"cache_v_l{il}")
        k_idxs = G.leaf(I64, [T], L["k_idxs"], name="k_idxs")
        v_idxs = G.leaf(I64, [kvw * T], L["v_idxs"], name="v_idxs")
        # cpy_k: set_rows(k cache [kvw, kv_size], reshape_2d(k_cur, kvw, n_tokens), k_idxs)
        kview = G.alias(g.GOP_VIEW, kc, [kvw, n_ctx])
        G.node(g.GOP_SET_ROWS, F16, [kvw, n_ctx], [G.alias(g.GOP_RESHAPE, k, [kvw, T]), k_idxs], view_src=kview,
               data=kc.data, name="k_store")
        # cpy_v (transposed V): set_rows(reshape_2d(v cache, 1, kvw*kv_size), reshape_2d(v_cur, 1, kvw*T), v_idxs)
        vview = G.alias(g.GOP_RESHAPE, vc, [1, kvw * n_ctx])
        G.node(g.GOP_SET_ROWS, F16, [1, kvw * n_ctx], [G.alias(g.GOP_RESHAPE, v, [1, kvw * T]), v_idxs],
               view_src=vview, data=vc.data, name="v_store")
        # build_attn_mha
        qp = G.alias(g.GOP_PERMUTE, q, [hd, T, nh])
        kv = G.alias(g.GOP_VIEW, kc, [hd, n_ctx, nkv])
        kq = G.node(g.GOP_MUL_MAT, F32, [n_ctx, T, nh], [kv, qp], name="kq")
        kq = G.node(g.GOP_SOFT_MAX, F32, [n_ctx, T, nh], [kq, mask], [scale, f32_bits(0.0)], name="kq_soft_max")
        vv = G.alias(g.GOP_VIEW, vc, [n_ctx, hd, nkv])
        kqv = G.node(g.GOP_MUL_MAT, F32, [hd, T, nh], [vv, kq], name="kqv")
        cur = G.alias(g.GOP_PERMUTE, kqv, [hd, nh, T])
        cur = G.node(g.GOP_CONT, F32, [hd * nh, T], [cur], name="kqv_out")
        cur = G.node(g.GOP_MUL_MAT, F32, [E, T], [mat(p + "attn_output"), cur], name="attn_out")
        R = T
        if il == hp["n_layer"] - 1 and out_ids is not None:  # skip computing output for unused tokens
            cur = G.node(g.GOP_GET_ROWS, F32, [E, 1], [cur, out_ids], name="attn_out_sel")
            inpSA = G.node(g.GOP_GET_ROWS, F32, [E, 1], [inpSA, out_ids], name="inpSA_sel")
            R = 1
        ffn_inp = G.node(g.GOP_ADD, F32, [E, R], [cur, inpSA], name="ffn_inp")
        cur = G.node(g.GOP_RMS_NORM, F32, [E, R], [ffn_inp], [eps], name="norm")
        cur = G.node(g.GOP_MUL, F32, [E, R], [cur, vec(p + "ffn_norm", E)], name="ffn_norm")
        F = hp["n_ff"]
        tmp = G.node(g.GOP_MUL_MAT, F32, [F, R], [mat(p + "ffn_up"), cur], name="ffn_up")
        gt = G.node(g.GOP_MUL_MAT, F32, [F, R], [mat(p + "ffn_gate"), cur], name="ffn_gate")
        cur = G.node(g.GOP_GLU, F32, [F, R], [gt, tmp], [g.GLU_SWIGLU, 0], name="ffn_swiglu")
        cur = G.node(g.GOP_MUL_MAT, F32, [E, R], [mat(p + "ffn_down"), cur], name="ffn_out")
        inpL = G.node(g.GOP_ADD, F32, [E, R], [cur, ffn_inp], name="l_out")
    cur = G.node(g.GOP_RMS_NORM, F32, [E, 1], [inpL], [eps], name="norm")
    cur = G.node(g.GOP_MUL, F32, [E, 1], [cur, vec("output_norm", E)], name="result_norm")
    G.node(g.GOP_MUL_MAT, F32, [V, 1], [mat("output"), cur], flags=g.FLAG_OUTPUT, name="result_output")
    return G
