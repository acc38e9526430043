"""CPU tests of the ggml graph lowering (mi355x_lower_ggml_graph, csrc/kq_lower.cpp):
llm_build_llama's decode graph, as a ggml backend adapter would mirror it
(tests/ggml_graph.py), lowers to exactly the node list LlamaDecoder builds for the
backend — same ops, shapes, op_params, flags, operands — so a llama.cpp graph runs on
the same fused launches the bench measures. Host only: no device is touched."""
import numpy as np
import pytest
import torch

import ggml_mi355x as g
from ggml_mi355x.llama import LlamaDecoder, hparams
from tests import ggml_graph as GG
from tests import llama_model as LM


def _describe(hp, n_ctx, seed=0):
    w = LM.build(hp, seed)
    wt = {k: ((v[0], torch.from_numpy(v[1])) if isinstance(v, tuple) else torch.from_numpy(v)) for k, v in w.items()}
    dec = LlamaDecoder(None, hp, wt, n_ctx, rope_src="table")
    return wt, dec


def _leaves(hp, wt, dec):
    L = {}
    for k, v in wt.items():
        if isinstance(v, tuple):
            t, a = v
            L[k] = (t, a.shape[1] // g.BLOCK_BYTES[t] * 256, a.shape[0], a.data_ptr(), a.stride(0))
        else:
            L[k] = v.data_ptr()
    for i in range(hp["n_layer"]):
        L[f"k_cache.{i}"] = dec.k_cache[i].data_ptr()
        L[f"v_cache.{i}"] = dec.v_cache[i].data_ptr()
    L["inp_tokens"] = dec.token.data_ptr()
    L["inp_pos"] = dec.pos.data_ptr()
    L["kq_mask"] = L["k_idxs"] = L["v_idxs"] = 0x1000
    return L


def canon(nodes):
    """(op, ne, op_params, flags, operands) per node; an operand is the index of the
    node producing it, or a leaf's (type, ne0, ne1, nb1, data)."""
    idx = {ctypes_addr(n): i for i, n in enumerate(nodes)}
    out = []
    for n in nodes:
        srcs = []
        for s in range(g.MAX_SRC):
            if not n.src[s]:
                break
            t = n.src[s].contents
            a = ctypes_addr(t)
            srcs.append(("node", idx[a]) if a in idx else ("leaf", t.type, t.ne[0], t.ne[1], t.nb[1], t.data))
        out.append((n.op, tuple(n.ne), tuple(n.op_params), n.flags, tuple(srcs)))
    return out


def ctypes_addr(t):
    import ctypes
    return ctypes.addressof(t)


@pytest.mark.parametrize("hp", [hparams(512, 2, 8, 2, 768, 1024), hparams(2048, 3, 32, 4, 5632, 4096),
                                hparams(1024, 2, 8, 8, 1536, 512)],
                         ids=["small-gqa4", "tinyllama-width", "mha"])
def test_llama_graph_lowers_to_decoder_nodes(hp):
    n_ctx = 64
    wt, dec = _describe(hp, n_ctx)
    G = GG.llama_decode_graph(hp, _leaves(hp, wt, dec), n_ctx)
    rc, nodes, keep = g.lower_ggml_graph(G.nodes, dec.table.data_ptr(), n_ctx, hp["freq_base"])
    assert rc == 0
    assert len(nodes) == len(dec.nodes) == 2 + 15 * hp["n_layer"] + 2
    got, want = canon(nodes), canon(dec.nodes)
    for i, (a, b) in enumerate(zip(got, want)):
        assert a == b, (i, a, b)


def test_lowering_rejects_what_it_cannot_run():
    """Patterns outside the backend's op set are refused (the scheduler keeps them on
    another backend): NEOX rope, a max_bias softmax, a swapped GLU, an unknown op."""
    hp = hparams(512, 1, 8, 2, 768, 1024)
    wt, dec = _describe(hp, 32)
    L = _leaves(hp, wt, dec)

    def lower(mutate):
        G = GG.llama_decode_graph(hp, L, 32)
        mutate(G)
        return g.lower_ggml_graph(G.nodes, dec.table.data_ptr(), 32, hp["freq_base"])[0]

    assert lower(lambda G: None) == 0

    def first(G, op):
        return next(t for t in G.nodes if t.op == op)

    assert lower(lambda G: first(G, g.GOP_ROPE).op_params.__setitem__(2, 2)) == g.E_UNSUPPORTED  # NEOX
    assert lower(lambda G: first(G, g.GOP_SOFT_MAX).op_params.__setitem__(1, GG.f32_bits(8.0))) == g.E_UNSUPPORTED
    assert lower(lambda G: first(G, g.GOP_GLU).op_params.__setitem__(1, 1)) == g.E_UNSUPPORTED  # swapped
    assert lower(lambda G: setattr(first(G, g.GOP_ADD), "op", 99)) == g.E_UNSUPPORTED
    # the rope table must match the graph's rope
    G = GG.llama_decode_graph(hp, L, 32)
    assert g.lower_ggml_graph(G.nodes, dec.table.data_ptr(), 32, 500000.0)[0] == g.E_UNSUPPORTED
    # an arena too small is reported, not overrun
    assert g.lower_ggml_graph(G.nodes, dec.table.data_ptr(), 32, hp["freq_base"], arena_cap=8)[0] == g.E_WORKSPACE


def test_lowering_rejects_attention_it_would_misplace():
    """ATTN_DECODE writes cell == pos and attends causally over [0, pos]. The lowering
    cannot read the device-resident k_idxs / mask, so it lowers an attention block only
    under the adapter's cells_eq_pos promise (one sequence, k_idxs == inp_pos, causal
    mask), and refuses what the table cannot express: rope freq_factors (Llama-3.1+
    rope_freqs, ROPE src[2]), index operands of the wrong shape, KQ views not at cell 0."""
    hp = hparams(512, 1, 8, 2, 768, 1024)
    wt, dec = _describe(hp, 32)
    L = _leaves(hp, wt, dec)
    tab = dec.table.data_ptr()

    def lower(mutate, **kw):
        G = GG.llama_decode_graph(hp, L, 32)
        mutate(G)
        return g.lower_ggml_graph(G.nodes, tab, 32, hp["freq_base"], **kw)[0]

    def nodes(G, op):
        return [t for t in G.nodes if t.op == op]

    assert lower(lambda G: None) == 0
    # several sequences / cells != positions (seq_rm, defrag, context shift): no promise
    assert lower(lambda G: None, cells_eq_pos=False) == g.E_UNSUPPORTED
    # rope with freq_factors on either the Q or the K rope
    ff = GG.Graph().leaf(GG.F32, [hp["head_dim"] // 2], 0x2000, name="rope_freqs")
    import ctypes
    for which in (0, 1):
        assert lower(lambda G: nodes(G, g.GOP_ROPE)[which].src.__setitem__(2, ctypes.pointer(ff))) == g.E_UNSUPPORTED
    # a K index operand that is not one row per token
    bad_idx = GG.Graph().leaf(GG.I64, [2], 0x1000, name="k_idxs")
    assert lower(lambda G: nodes(G, g.GOP_SET_ROWS)[0].src.__setitem__(1, ctypes.pointer(bad_idx))) == g.E_UNSUPPORTED
    # f32 indices are not indices
    f_idx = GG.Graph().leaf(GG.F32, [1], 0x1000, name="k_idxs")
    assert lower(lambda G: nodes(G, g.GOP_SET_ROWS)[0].src.__setitem__(1, ctypes.pointer(f_idx))) == g.E_UNSUPPORTED

    # a KQ view that starts past cell 0
    def shift_view(G):
        kq = next(t for t in G.nodes if t.op == g.GOP_MUL_MAT and t.name == b"kq")
        kq.src[0].contents.view_offs = 64

    assert lower(shift_view) == g.E_UNSUPPORTED


def test_lowering_supports_every_lowered_node():
    """Every node the lowering emits passes the backend's supports_op."""
    hp = hparams(512, 2, 8, 2, 768, 1024)
    wt, dec = _describe(hp, 64)
    G = GG.llama_decode_graph(hp, _leaves(hp, wt, dec), 64)
    rc, nodes, keep = g.lower_ggml_graph(G.nodes, dec.table.data_ptr(), 64, hp["freq_base"])
    assert rc == 0
    assert all(g.supports_op(n) for n in nodes)
    ops = [n.op for n in nodes]
    assert ops.count(g.OP_ATTN_DECODE) == hp["n_layer"]
    assert np.count_nonzero(np.array(ops) == g.OP_MUL_MAT) == 7 * hp["n_layer"] + 1


@pytest.mark.parametrize("n_tok", [2, 37])
def test_llama_prompt_graph_lowers_to_decoder_nodes(n_tok):
    """A prompt ubatch of llm_build_llama (T tokens, the inp_out_ids GET_ROWS of the last
    layer) lowers to exactly LlamaDecoder's prompt node list: batched MUL_MATs, the
    attention block -> one ATTN_DECODE node of T tokens, and every node passes supports_op."""
    hp = hparams(512, 2, 8, 2, 768, 1024)
    n_ctx = 64
    wt, dec = _describe(hp, n_ctx)
    pg = dec._prompt_graph(n_tok)
    L = _leaves(hp, wt, dec)
    L["inp_tokens"] = pg["inp"][:n_tok].data_ptr()
    L["inp_pos"] = pg["inp"][n_tok:2 * n_tok].data_ptr()
    L["inp_out_ids"] = pg["inp"][2 * n_tok:].data_ptr()
    G = GG.llama_decode_graph(hp, L, n_ctx, n_tokens=n_tok)
    rc, nodes, keep = g.lower_ggml_graph(G.nodes, dec.table.data_ptr(), n_ctx, hp["freq_base"])
    assert rc == 0
    got, want = canon(nodes), canon(pg["nodes"])
    assert len(got) == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert a == b, (i, a, b)
    assert all(g.supports_op(n) for n in nodes)
    assert [n.op for n in nodes].count(g.OP_ATTN_DECODE) == hp["n_layer"]
