"""The row-split decode token restated on the CPU oracle (test infrastructure):
rank `split.rank` of `split.world` computes exactly the node list LlamaDecoder builds
with `split=` (ggml_mi355x/rowsplit.py TokenSplit) — its q/k/v rows, the attention of
its heads on its KV-cache slice, its attn_output / gate / up / down / output rows —
and `gather(local) -> full` stands in for the ALL_GATHER node (RCCL on GPUs, gloo
here). The reference's own split is the same rows across threads
(ggml_compute_forward_mul_mat chunks, README.md:125-131)."""
from __future__ import annotations

import numpy as np

from oracle import kq_oracle as KO
from oracle import kq_ops_oracle as OO


def local_model(model, split):
    """Row slices of an oracle model dict (tests/llama_model.oracle_model layout)."""
    rows = split.rows
    lay = []
    for L in model["layers"]:
        d = dict(L)
        for key, name in (("wq", "attn_q"), ("wk", "attn_k"), ("wv", "attn_v"), ("wo", "attn_output"),
                          ("w_gate", "ffn_gate"), ("w_up", "ffn_up"), ("w_down", "ffn_down")):
            r0, r1 = rows[name]
            d[key] = (L[key][0], np.ascontiguousarray(L[key][1][r0:r1]))
        lay.append(d)
    r0, r1 = rows["output"]
    out = dict(model)
    out["layers"] = lay
    out["output"] = (model["output"][0], np.ascontiguousarray(model["output"][1][r0:r1]))
    return out


def local_cache(hp, split, n_ctx):
    kvw = split.n_head_kv * hp["head_dim"]
    return [(np.zeros((n_ctx, kvw), np.uint16), np.zeros((kvw, n_ctx), np.uint16)) for _ in range(hp["n_layer"])]


def split_decode_token(lmodel, split, token, pos, cache, gather, n_threads=2, full_trace=None):
    hp = lmodel["hp"]
    E, hd, eps = hp["n_embd"], hp["head_dim"], hp["eps"]
    t, w = lmodel["tok_embd"]
    x = OO.get_rows(t, w, E, [token])[0]
    table = lmodel["rope_table"]
    scale = np.float32(1.0) / np.sqrt(np.float32(hd))
    e0, e1 = split.rows["attn_output"]
    for li, L in enumerate(lmodel["layers"]):
        cur = OO.mul(OO.rms_norm(x, eps), L["attn_norm"])
        q = KO.mul_mat(L["wq"][0], L["wq"][1], cur, n_threads)[0]
        k = KO.mul_mat(L["wk"][0], L["wk"][1], cur, n_threads)[0]
        v = KO.mul_mat(L["wv"][0], L["wv"][1], cur, n_threads)[0]
        q = OO.rope(q, hd, hd, pos, table)
        k = OO.rope(k, hd, hd, pos, table)
        kc, vc = cache[li]
        att = OO.attn_decode(q, k, v, kc, vc, pos, split.n_head, split.n_head_kv, hd, float(scale))
        att = gather(att)
        o = KO.mul_mat(L["wo"][0], L["wo"][1], att, n_threads)[0]
        ffn_inp = gather(OO.add(o, x[e0:e1]))
        cur = OO.mul(OO.rms_norm(ffn_inp, eps), L["ffn_norm"])
        g = KO.mul_mat(L["w_gate"][0], L["w_gate"][1], cur, n_threads)[0]
        u = KO.mul_mat(L["w_up"][0], L["w_up"][1], cur, n_threads)[0]
        glu = gather(OO.swiglu(g, u))
        dn = KO.mul_mat(L["w_down"][0], L["w_down"][1], glu, n_threads)[0]
        x = gather(OO.add(dn, ffn_inp[e0:e1]))
        if full_trace is not None:
            full_trace.append({"att": att, "ffn_inp": ffn_inp, "glu": glu, "x": x})
    cur = OO.mul(OO.rms_norm(x, eps), lmodel["output_norm"])
    return gather(KO.mul_mat(lmodel["output"][0], lmodel["output"][1], cur, n_threads)[0])
