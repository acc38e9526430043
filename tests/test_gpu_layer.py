"""GPU: every decode layer of llm_build_llama as ONE persistent launch (csrc/kq_layer.hip,
mi355x_backend_set_layer_engine). One workgroup per CU owns rows of every matrix; the
stream waves fetch the next stage's weights into LDS while the current stage's output is
handed between workgroups (sc1 stores, counters, sc1 loads); the control wave replays each
row's fp32 chain in superblock order. Checked here:
  * the engine really runs (one kq_layer launch per layer, no kq_rows / kq_attn_decode for
    the layers) and the engine-off path does not use it;
  * every token's logits and final hidden state are bit-exact with the oracle's
    llm_build_llama restatement AND with the per-node launches, over many positions through
    the captured graph (the counters and the epoch run launch after launch);
  * TinyLlama width (head_dim 64, 4 heads per attention workgroup, Q4_K_M and Q5_K_M mixes:
    Q5_K / Q6_K segments in one stage) and Llama-3-8B width (head_dim 128, GQA 32/8, n_ff
    14336: 56-superblock down rows);
  * no wait ever gave up (mi355x_backend_layer_error)."""
import numpy as np
import pytest

from tests.test_gpu_parity import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu


def _decoder(dev, hp, seed, n_ctx, mix="q4_k_m"):
    from tests import llama_model as LM
    import ggml_mi355x as g
    from ggml_mi355x.llama import LlamaDecoder
    w = LM.build(hp, seed, mix=mix)
    b = g.Backend()
    assert b.set_layer_engine(True) == 0  # opt-in
    dec = LlamaDecoder(b, hp, LM.to_device(w, dev), n_ctx, fuse=True)
    return w, b, dec


def _launch_names(dec, tok, pos):
    import ggml_mi355x as g
    g.timing_enable(True)
    dec.step(tok, pos, use_graph=False)
    names = [r[0] for r in g.timing_read()]
    g.timing_enable(False)
    return names


SHAPES = {
    "tinyllama": dict(args=(2048, 2, 32, 4, 5632, 4096), kw={}),
    "llama3_8b": dict(args=(4096, 2, 32, 8, 14336, 2048), kw=dict(freq_base=500000.0)),
}


@pytest.mark.parametrize("shape,mix,n_tok", [("tinyllama", "q4_k_m", 40), ("tinyllama", "q5_k_m", 12),
                                             ("llama3_8b", "q4_k_m", 24)])
def test_layer_engine_bit_exact(dev, shape, mix, n_tok):
    from oracle import kq_ops_oracle as O
    from tests import llama_model as LM
    from ggml_mi355x.llama import hparams
    O.lib()
    hp = hparams(*SHAPES[shape]["args"], **SHAPES[shape]["kw"])
    n_ctx = 64
    w, b, dec = _decoder(dev, hp, 31, n_ctx, mix)
    names = _launch_names(dec, 5, 0)
    n_layer = hp["n_layer"]
    assert sum("kq_layer" in n for n in names) == n_layer, names
    assert not any("kq_attn_decode" in n for n in names), names
    assert sum("kq_rows" in n for n in names) == 1, names  # the output head only
    assert b.layer_error() == 0
    dec.reset()
    model, cache = LM.oracle_model(hp, w, n_ctx)
    rng = np.random.default_rng(5)
    tokens = rng.integers(0, hp["n_vocab"], size=n_tok).tolist()
    outs = []
    for p, tok in enumerate(tokens):
        dec.step(tok, p)
        b.synchronize()
        got = dec.logits.cpu().numpy().copy()
        ref, trace = O.decode_token(model, tok, p, cache)
        assert bits_equal(got, ref), (p, first_mismatch(got, ref))
        hid = dec.last_hidden.cpu().numpy()
        assert bits_equal(hid, trace[-1]), (p, "hidden", first_mismatch(hid, trace[-1]))
        outs.append(got)
    assert b.layer_error() == 0
    # the per-node launches on the same backend, same tokens
    assert b.set_layer_engine(False) == 1
    dec.reset()
    names = _launch_names(dec, 5, 0)
    assert not any("kq_layer" in n for n in names), names
    dec.reset()
    for p, tok in enumerate(tokens[:6]):
        dec.step(tok, p)
        b.synchronize()
        assert bits_equal(dec.logits.cpu().numpy(), outs[p]), p
    b.close()


def test_layer_engine_long_cache(dev):
    """A 256-cell cache at head_dim 64 (the attention's multi-pass branch past 128 cells,
    the attention workgroups' LDS beside the weight ring): tokens past position 128
    bit-exact with the per-node path; eager steps and graph replays interleaved."""
    from ggml_mi355x.llama import hparams
    hp = hparams(2048, 1, 32, 4, 1024, 1024)
    n_ctx = 256
    _, b, dec = _decoder(dev, hp, 7, n_ctx)
    rng = np.random.default_rng(3)
    tokens = rng.integers(0, hp["n_vocab"], size=140).tolist()
    eng = []
    for p, tok in enumerate(tokens):
        dec.step(tok, p, use_graph=(p % 7 != 3))
        b.synchronize()
        eng.append(dec.logits.cpu().numpy().copy())
    assert b.layer_error() == 0
    assert b.set_layer_engine(False) == 1
    dec.reset()
    for p, tok in enumerate(tokens):
        dec.step(tok, p)
        b.synchronize()
        assert bits_equal(dec.logits.cpu().numpy(), eng[p]), p
    b.close()


def _per_node_logits(dev, hp, wdev, n_ctx, tokens):
    import ggml_mi355x as g
    from ggml_mi355x.llama import LlamaDecoder
    b = g.Backend()
    dec = LlamaDecoder(b, hp, wdev, n_ctx, fuse=True)
    out = []
    for p, tok in enumerate(tokens):
        dec.step(tok, p)
        b.synchronize()
        out.append(dec.logits.cpu().numpy().copy())
    b.close()
    return out


def test_layer_engine_tables_across_graphs(dev):
    """one backend, the engine on, graphs that (a) match MORE layers than the first
    one did (the counter blocks grow; every step table stays valid) and (b) share weights at a
    different KV-cache size (another ring depth and LDS layout, so another step table), steps
    of the three decoders interleaved: every token bit-exact with the per-node launches."""
    import ggml_mi355x as g
    from tests import llama_model as LM
    from ggml_mi355x.llama import LlamaDecoder, hparams
    hp1 = hparams(2048, 1, 32, 4, 1024, 1024)
    hp2 = hparams(2048, 2, 32, 4, 1024, 1024)
    w1 = LM.to_device(LM.build(hp1, 11), dev)
    w2 = LM.to_device(LM.build(hp2, 12), dev)
    rng = np.random.default_rng(9)
    tokens = rng.integers(0, hp1["n_vocab"], size=10).tolist()
    b = g.Backend()
    assert b.set_layer_engine(True) == 0
    decs = [LlamaDecoder(b, hp1, w1, 64, fuse=True),    # 1 layer
            LlamaDecoder(b, hp2, w2, 64, fuse=True),    # 2 layers: the blocks grow
            LlamaDecoder(b, hp2, w2, 256, fuse=True)]   # same weights, another cache size
    names = _launch_names(decs[2], 5, 0)
    assert sum("kq_layer" in n for n in names) == 2, names
    for d in decs:
        d.reset()
    refs = [_per_node_logits(dev, hp1, w1, 64, tokens), _per_node_logits(dev, hp2, w2, 64, tokens),
            _per_node_logits(dev, hp2, w2, 256, tokens)]
    for p, tok in enumerate(tokens):
        for i, d in enumerate(decs):
            d.step(tok, p, use_graph=(p % 3 != 1))
            b.synchronize()  # raises on a lost-co-residency error (MI355X_E_LAYER)
            got = d.logits.cpu().numpy()
            assert bits_equal(got, refs[i][p]), (i, p, first_mismatch(got, refs[i][p]))
    assert b.layer_error() == 0
    b.close()
