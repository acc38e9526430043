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
    """Row slices (and, in reduce mode, superblock-column slices of attn_output /
    ffn_down) of an oracle model dict (tests/llama_model.oracle_model layout)."""
    rows = split.rows
    lay = []
    for L in model["layers"]:
        d = dict(L)
        for key, name in (("wq", "attn_q"), ("wk", "attn_k"), ("wv", "attn_v"), ("wo", "attn_output"),
                          ("w_gate", "ffn_gate"), ("w_up", "ffn_up"), ("w_down", "ffn_down")):
            r0, r1 = rows[name]
            w = L[key][1][r0:r1]
            if name in split.cols:
                c0, c1 = split.cols[name]
                B = KO.BLOCK_BYTES[L[key][0]]
                w = w[:, c0 * B:c1 * B]
            d[key] = (L[key][0], np.ascontiguousarray(w))
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



def _ksplit_gen(lmodel, split, token, pos, cache, n_threads, full_trace, variant="neon"):
    """Reduce mode (TokenSplit(mode="reduce"), the K-split Megatron pairing) as a
    generator that yields ("reduce" | "gather", local f32 vector) at every collective and
    receives the exchanged vector: the rank's q/k/v heads and attention, its K slice of
    attn_output (partial chain over its superblocks, + x on rank 0) -> reduce; its ffn
    rows (gate / up / swiglu) = its K slice of ffn_down (+ ffn_inp on rank 0) -> reduce;
    output rows -> gather. Returns the logits."""
    hp = lmodel["hp"]
    E, hd, eps = hp["n_embd"], hp["head_dim"], hp["eps"]
    t, w = lmodel["tok_embd"]
    x = OO.get_rows(t, w, E, [token])[0]
    table = lmodel["rope_table"]
    scale = np.float32(1.0) / np.sqrt(np.float32(hd))
    for li, L in enumerate(lmodel["layers"]):
        cur = OO.mul(OO.rms_norm(x, eps), L["attn_norm"])
        q = KO.mul_mat(L["wq"][0], L["wq"][1], cur, n_threads, variant)[0]
        k = KO.mul_mat(L["wk"][0], L["wk"][1], cur, n_threads, variant)[0]
        v = KO.mul_mat(L["wv"][0], L["wv"][1], cur, n_threads, variant)[0]
        q = OO.rope(q, hd, hd, pos, table)
        k = OO.rope(k, hd, hd, pos, table)
        kc, vc = cache[li]
        att = OO.attn_decode(q, k, v, kc, vc, pos, split.n_head, split.n_head_kv, hd, float(scale))
        o = KO.mul_mat(L["wo"][0], L["wo"][1], att, n_threads, variant)[0]
        po = OO.add(o, x) if split.rank == 0 else o
        ffn_inp = yield ("reduce", po)
        cur = OO.mul(OO.rms_norm(ffn_inp, eps), L["ffn_norm"])
        g = KO.mul_mat(L["w_gate"][0], L["w_gate"][1], cur, n_threads, variant)[0]
        u = KO.mul_mat(L["w_up"][0], L["w_up"][1], cur, n_threads, variant)[0]
        glu = OO.swiglu(g, u)
        dn = KO.mul_mat(L["w_down"][0], L["w_down"][1], glu, n_threads, variant)[0]
        pd = OO.add(dn, ffn_inp) if split.rank == 0 else dn
        x = yield ("reduce", pd)
        if full_trace is not None:
            full_trace.append({"att": att, "p_ffn_inp": po, "ffn_inp": ffn_inp, "glu": glu, "p_x": pd, "x": x})
    cur = OO.mul(OO.rms_norm(x, eps), lmodel["output_norm"])
    lg = KO.mul_mat(lmodel["output"][0], lmodel["output"][1], cur, n_threads, variant)[0]
    return (yield ("gather", lg))


def ksplit_decode_token(lmodel, split, token, pos, cache, allreduce, gather, n_threads=2, full_trace=None):
    """One rank of the reduce-mode token with real collectives (allreduce / gather
    callables: gloo in tests/test_dist.py)."""
    gen = _ksplit_gen(lmodel, split, token, pos, cache, n_threads, full_trace)
    try:
        kind, v = next(gen)
        while True:
            kind, v = gen.send(allreduce(v) if kind == "reduce" else gather(v))
    except StopIteration as e:
        return e.value


def rank_ordered_sum(parts):
    """The deterministic stand-in for ncclAllReduce(sum): ((p0 + p1) + p2) + ... in f32."""
    acc = np.asarray(parts[0], np.float32).copy()
    for p in parts[1:]:
        acc = (acc + np.asarray(p, np.float32)).astype(np.float32)
    return acc


def ksplit_reference(model, hp, world, tokens, n_ctx, n_threads=2, variant="neon"):
    """Every rank of a reduce-mode split in one process, in lock step, the all-reduce a
    rank-ordered f32 sum: the restatement the per-rank GPU emulation is checked against
    bit for bit. Returns per token (logits, traces[rank] -> per layer dict)."""
    from ggml_mi355x.rowsplit import TokenSplit
    splits = [TokenSplit(hp, world, r, mode="reduce") for r in range(world)]
    lms = [local_model(model, sp) for sp in splits]
    caches = [local_cache(hp, sp, n_ctx) for sp in splits]
    out = []
    for pos, tok in enumerate(tokens):
        traces = [[] for _ in range(world)]
        gens = [_ksplit_gen(lms[r], splits[r], tok, pos, caches[r], n_threads, traces[r], variant)
                for r in range(world)]
        reqs = [next(gen) for gen in gens]
        while True:
            kinds = {k for k, _ in reqs}
            assert len(kinds) == 1, kinds
            kind = kinds.pop()
            parts = [v for _, v in reqs]
            val = rank_ordered_sum(parts) if kind == "reduce" else np.concatenate(parts).astype(np.float32)
            done, nxt = [], []
            for gen in gens:
                try:
                    nxt.append(gen.send(val.copy()))
                except StopIteration as e:
                    done.append(e.value)
            if done:
                assert len(done) == world
                break
            reqs = nxt
        assert all((d.view(np.uint32) == done[0].view(np.uint32)).all() for d in done)
        out.append((done[0], traces))
    return out
