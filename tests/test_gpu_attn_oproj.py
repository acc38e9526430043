"""GPU: decode attention fused with the o-proj GEMV (+ residual ADD) in one launch
(csrc/kq_attn_oproj.hip, mi355x_backend_set_attn_oproj). Workgroup (s, rb) runs the
attention of the heads of the o-proj's K superblock s, quantizes them to that Q8_K
superblock and writes the exact records of row block rb; the last workgroup of each row
block replays every row's fp32 chain in superblock order. Checked here:
  * the fused kernel really runs (launch log) and the unfused path does not use it;
  * every token's logits and hidden state are bit-exact with the oracle's llm_build_llama
    restatement AND with the two-launch path (kq_attn_decode + kq_rows), over many positions
    (the arrival counters run round after round through the captured graph);
  * TinyLlama width (head_dim 64, 4 heads per superblock, Q4_K_M and Q5_K_M mixes) and
    Llama-3-8B width (head_dim 128, GQA 32/8, 2 heads per superblock);
  * a position outside the cache gives the same logits fused and unfused."""
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
    assert b.set_attn_oproj(True) == 0  # opt-in (the product default is the two launches)
    dec = LlamaDecoder(b, hp, LM.to_device(w, dev), n_ctx, fuse=True)
    return w, b, dec


def _launch_names(dec, tok, pos):
    import ggml_mi355x as g
    g.timing_enable(True)
    dec.step(tok, pos, use_graph=False)
    names = [r[0] for r in g.timing_read()]
    g.timing_enable(False)
    return names


@pytest.mark.parametrize("shape,mix", [("tinyllama", "q4_k_m"), ("tinyllama", "q5_k_m"), ("llama3_8b", "q4_k_m")])
def test_attn_oproj_bit_exact(dev, shape, mix):
    from oracle import kq_ops_oracle as O
    from tests import llama_model as LM
    from ggml_mi355x.llama import hparams
    O.lib()
    if shape == "tinyllama":
        hp = hparams(2048, 2, 32, 4, 5632, 4096)
    else:  # Llama-3-8B width (E 4096, GQA 32/8, hd 128), a short FF and vocabulary
        hp = hparams(4096, 2, 32, 8, 2048, 2048, freq_base=500000.0)
    n_ctx = 64
    w, b, dec = _decoder(dev, hp, 23, n_ctx, mix)
    names = _launch_names(dec, 5, 0)
    n_layer = hp["n_layer"]
    assert sum("kq_attn_oproj" in n for n in names) == n_layer, names
    assert not any("kq_attn_decode" in n for n in names), names
    dec.reset()
    model, cache = LM.oracle_model(hp, w, n_ctx)
    rng = np.random.default_rng(5)
    tokens = rng.integers(0, hp["n_vocab"], size=40).tolist()
    fused = []
    for p, tok in enumerate(tokens):
        dec.step(tok, p)
        b.synchronize()
        got = dec.logits.cpu().numpy().copy()
        ref, trace = O.decode_token(model, tok, p, cache)
        assert bits_equal(got, ref), (p, first_mismatch(got, ref))
        hid = dec.last_hidden.cpu().numpy()
        assert bits_equal(hid, trace[-1]), (p, "hidden", first_mismatch(hid, trace[-1]))
        fused.append(got)
    # the two-launch path on the same backend, same tokens
    assert b.set_attn_oproj(False) == 1
    dec.reset()
    names = _launch_names(dec, 5, 0)
    assert not any("kq_attn_oproj" in n for n in names) and any("kq_attn_decode" in n for n in names), names
    dec.reset()
    for p, tok in enumerate(tokens[:8]):
        dec.step(tok, p)
        b.synchronize()
        assert bits_equal(dec.logits.cpu().numpy(), fused[p]), p
    b.close()


def test_attn_oproj_position_outside_cache(dev):
    """pos >= n_ctx (set straight into the graph's input, past LlamaDecoder.step's guard):
    the attention writes NaN and stores no cell; the o-proj then quantizes what it gets (an
    all-NaN superblock quantizes to zeros: quantize_row_q8_K's amax skips NaN). Fused and
    unfused give the same logits bit for bit."""
    import torch
    import ggml_mi355x as g
    from ggml_mi355x.llama import hparams
    hp = hparams(2048, 1, 32, 4, 5632, 4096)
    n_ctx = 32
    outs = []
    for fused in (True, False):
        _, b, dec = _decoder(dev, hp, 3, n_ctx)
        b.set_attn_oproj(fused)
        for p in range(3):
            dec.step(7 + p, p)
        b.synchronize()
        row = torch.zeros(dec.inp.numel(), dtype=torch.int32)
        row[0], row[1] = 11, n_ctx + 5
        row[2:] = dec._table_host[0]
        assert g.lib().mi355x_backend_set_tensor(b.h, dec.inp.data_ptr(), row.data_ptr(), 4 * row.numel()) == 0
        assert g.lib().mi355x_backend_graph_compute(b.h, dec._arr, len(dec.nodes), 1) == 0
        b.synchronize()
        outs.append(dec.logits.cpu().numpy().copy())
        b.close()
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


@pytest.mark.parametrize("nrb", [0, 12])
def test_attn_oproj_long_cache_and_row_blocks(dev, nrb):
    """the fused kernel admits KV caches of up to 256 cells. At head_dim 64 a head
    runs on 128 threads, so n_kv > 128 takes attn_head's multi-pass branch: decode past
    position 128 of a 256-cell cache, fused against unfused bit for bit (and against the
    oracle at the positions around the 128-cell edge). nrb = 12 (AO_NRB): row blocks whose
    workgroups are not a multiple of 8 apart, so one row block's workgroups sit on several
    XCDs and the hand-off crosses them."""
    from oracle import kq_ops_oracle as O
    from tests import llama_model as LM
    import ggml_mi355x as g
    from ggml_mi355x.llama import hparams
    O.lib()
    hp = hparams(2048, 1, 32, 4, 1024, 1024)
    n_ctx = 256
    prev = g.debug_knob("AO_NRB", nrb) if nrb else None
    try:
        w, b, dec = _decoder(dev, hp, 29, n_ctx)
        model, cache = LM.oracle_model(hp, w, n_ctx)
        rng = np.random.default_rng(11)
        tokens = rng.integers(0, hp["n_vocab"], size=150).tolist()
        fused = []
        for p, tok in enumerate(tokens):
            dec.step(tok, p)
            b.synchronize()
            got = dec.logits.cpu().numpy().copy()
            ref, _ = O.decode_token(model, tok, p, cache)
            if p in (0, 1, 126, 127, 128, 129, 130, 149):
                assert bits_equal(got, ref), (p, first_mismatch(got, ref))
            fused.append(got)
        assert b.set_attn_oproj(False) == 1
        dec.reset()
        for p, tok in enumerate(tokens):
            dec.step(tok, p)
            b.synchronize()
            assert bits_equal(dec.logits.cpu().numpy(), fused[p]), p
        b.close()
    finally:
        if nrb:
            g.debug_knob("AO_NRB", prev if prev else float("nan"))
