"""GPU: the f16 prefill path (kq_mmf, mi355x_prefill_precision(PREFILL_F16)) against the
bit-exact reference restatement within the stated tolerance (oracle/kq_oracle_np.py
mmf_bound; csrc/kq_mmf.hip header), and against the f16 emulation of the same operands
(only the f32 accumulation order differs: 2^-12 of the bound's sum). The default stays
the bit-exact kq_mmq (tests/test_gpu_parity.py test_prefill_*)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.fixture
def f16path():
    """The f16 kernel on every shape (PREFILL_F16_ALL), so that each test exercises kq_mmf."""
    import ggml_mi355x as g
    prev = g.prefill_precision(g.PREFILL_F16_ALL)
    yield
    g.prefill_precision(prev)


def check(got, w, type_, K, x, oracle, npo, rows=None, cols=None):
    wr = w if rows is None else w[rows]
    xc = x if cols is None else x[cols]
    g = got if rows is None else got[np.ix_(cols, rows)]
    g = g.astype(np.float64)
    ref = oracle.mul_mat(type_, wr, xc).astype(np.float64)
    bound = npo.mmf_bound(wr, type_, K, xc)
    assert np.isfinite(g).all()
    err = np.abs(g - ref)
    assert (err <= bound).all(), ("vs reference", float((err / bound).max()))
    emu = npo.mmf_emulate(wr, type_, K, xc)
    assert (np.abs(g - emu) <= bound * 2.0 ** -4).all(), ("vs emulation", float((np.abs(g - emu) / bound).max()))


@pytest.mark.parametrize("type_", [12, 13, 14], ids=["q4_K", "q5_K", "q6_K"])
@pytest.mark.parametrize("K,N,M", [
    (256, 32, 16),      # one superblock, one partial tile
    (768, 200, 37),     # odd superblock count (Q6_K rows 2-B aligned), ragged rows / columns
    (2048, 256, 128),   # split-K (grid below the CU count)
    (4096, 384, 200),   # split-K, three row tiles, two column tiles
    (1024, 130, 129),   # one row and one column past a tile edge
])
def test_mmf_within_stated_tolerance(dev, oracle, npo, f16path, type_, K, N, M):
    import ggml_mi355x as g
    rng = np.random.default_rng(K + 7 * N + 13 * M + type_)
    w = npo.random_blocks(rng, type_, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    x[1, :256] = 0.0  # an all-zero activation block (d = 0)
    got = g.mul_mat(type_, t(w, dev), K, t(x, dev)).cpu().numpy()
    check(got, w, type_, K, x, oracle, npo)


@pytest.mark.parametrize("type_,K,N", [(12, 4096, 14336), (14, 14336, 4096), (13, 4096, 4096)],
                         ids=["8b_ffn_up_q4K", "8b_ffn_down_q6K", "8b_q_q5K"])
def test_mmf_bench_size_subset(dev, oracle, npo, f16path, type_, K, N):
    """Llama-3-8B shapes at pp512: every output finite, a row x column subset checked."""
    import ggml_mi355x as g
    M = 512
    rng = np.random.default_rng(N + type_)
    w = npo.random_blocks(rng, type_, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    got = g.mul_mat(type_, t(w, dev), K, t(x, dev)).cpu().numpy()
    assert got.shape == (M, N) and np.isfinite(got).all()
    rows = np.unique(np.concatenate([rng.integers(0, N, 24), [0, 127, 128, N - 1]]))
    cols = np.unique(np.concatenate([rng.integers(0, M, 12), [0, 127, 128, M - 1]]))
    check(got, w, type_, K, x, oracle, npo, rows, cols)


def test_prefill_precision_selector(dev):
    import ggml_mi355x as g
    prev = g.prefill_precision(-1)
    assert prev == g.PREFILL_EXACT  # the default: bit-exact kq_mmq
    assert g.prefill_precision(g.PREFILL_F16) == prev
    assert g.prefill_precision(-1) == g.PREFILL_F16
    assert g.prefill_precision(g.PREFILL_F16_ALL) == g.PREFILL_F16
    assert g.prefill_precision(prev) == g.PREFILL_F16_ALL
    assert g.lib().mi355x_prefill_precision(7) == g.E_INVAL


def test_prefill_f16_per_shape_choice(dev, oracle, npo):
    """PREFILL_F16 runs kq_mmf where it is the faster kernel (Q5_K / Q6_K, large Q4_K) and
    the bit-exact kq_mmq elsewhere: the launch names say which, every result within the
    stated bound (and the exact ones bit-exact)."""
    import ggml_mi355x as g
    prev = g.prefill_precision(g.PREFILL_F16)
    try:
        rng = np.random.default_rng(21)
        for type_, K, N, want in ((12, 2048, 256, "kq_mmq"), (14, 2048, 256, "kq_mmf"), (13, 512, 64, "kq_mmf"),
                                  (12, 8192, 4096, "kq_mmf")):
            M = 32
            w = npo.random_blocks(rng, type_, N, K)
            x = rng.standard_normal((M, K)).astype(np.float32)
            g.timing_enable(True)
            got = g.mul_mat(type_, t(w, dev), K, t(x, dev)).cpu().numpy()
            names = [r[0] for r in g.timing_read()]
            g.timing_enable(False)
            assert any(want in n for n in names), (type_, K, N, names)
            if want == "kq_mmq":
                assert np.array_equal(got.view(np.uint32), oracle.mul_mat(type_, w, x).view(np.uint32))
            else:
                ref = oracle.mul_mat(type_, w, x).astype(np.float64)
                assert (np.abs(got - ref) <= npo.mmf_bound(w, type_, K, x)).all()
    finally:
        g.prefill_precision(prev)


@pytest.mark.parametrize("mix", ["q4_k_m", "q5_k_m"])
def test_llama_prompt_f16(dev, f16path, mix):
    """The prompt graph on the f16 GEMMs (every MUL_MAT at ne11 = 37 through kq_mmf, the
    norm / swiglu as their own nodes, the residual ADD as the GEMM's epilogue):
    * a replay of the captured graph repeats its logits exactly, and the fused graph
      (multi-matrix launches, ADD epilogue, one activation image per activation) gives
      layer 0's K cache of the unfused one bit for bit;
    * layer 0's K cache (one GEMM deep) is within a relative L2 error of 2^-9 of the
      bit-exact prompt's;
    * the logits are within 2^-5 (relative L2) of the oracle's sequential llm_build_llama.
      The synthetic model's random attention is sharp (|q.k| scores in the tens), so a
      GEMM-level difference of ~2^-11 grows ~10x per layer (layer 1's K cache: ~2^-7);
      the GEMM-level tolerance itself is test_mmf_within_stated_tolerance's."""
    import torch
    from oracle import kq_ops_oracle as O
    from tests import llama_model as LM
    from tests.test_gpu_ops import _decoder
    import ggml_mi355x as g
    from ggml_mi355x.llama import hparams
    O.lib()
    hp = hparams(2048, 2, 32, 4, 5632, 4096)
    n_ctx, n = 64, 37
    tokens = np.random.default_rng(13).integers(0, hp["n_vocab"], size=n).tolist()
    out = {}
    for name, prec, fuse in (("exact", g.PREFILL_EXACT, True), ("f16", g.PREFILL_F16_ALL, True),
                             ("f16_unfused", g.PREFILL_F16_ALL, False), ("f16_auto", g.PREFILL_F16, True)):
        g.prefill_precision(prec)
        w, b, dec = _decoder(dev, hp, 7, n_ctx, fuse, mix=mix)
        lg = dec.prompt(tokens, 0)
        b.synchronize()
        first = lg.cpu().numpy().copy()
        lg = dec.prompt(tokens, 0)  # replay of the captured graph
        b.synchronize()
        assert np.array_equal(first.view(np.uint32), lg.cpu().numpy().view(np.uint32)), name
        out[name] = (first.astype(np.float64).ravel(),
                     [c[:n].view(torch.float16).float().cpu().numpy() for c in dec.k_cache])
        b.close()
    g.prefill_precision(g.PREFILL_F16_ALL)
    got = out["f16_auto"][0]  # the per-shape choice (kq_mmq on TinyLlama's small Q4_K GEMMs)
    assert np.isfinite(got).all()
    # fused (q/k/v and gate/up as multi-matrix launches) vs unfused: layer 0's K cache (one
    # GEMM deep, the same K split either way) bit for bit; later values differ by the f32
    # summation order of other splits, grown by the model (test_mmf_multi_matrix_launch
    # checks the multi-matrix GEMM itself)
    assert np.array_equal(out["f16"][1][0], out["f16_unfused"][1][0])
    k0, k0e = out["f16"][1][0], out["exact"][1][0]
    assert np.isfinite(k0).all() and np.linalg.norm(k0 - k0e) <= 2.0 ** -9 * np.linalg.norm(k0e)
    model, cache = LM.oracle_model(hp, w, n_ctx)
    for p, tok in enumerate(tokens):
        ref, _ = O.decode_token(model, tok, p, cache)
    ref = np.asarray(ref, np.float64).ravel()
    assert np.array_equal(out["exact"][0], ref)  # the default path stays bit-exact
    got = out["f16"][0]
    assert np.isfinite(got).all()
    assert np.linalg.norm(got - ref) <= 2.0 ** -5 * np.linalg.norm(ref)
    torch.cuda.synchronize()


def test_llama_prompt_f16_auto_then_exact_prologue(dev, f16path):
    """PREFILL_F16 with the per-shape choice on 5 TinyLlama-width layers: layer 2 is a
    use_more_bits layer, so its Q6_K ffn_down runs on kq_mmf (f16); layer 3's q/k/v are
    Q4_K and stay on kq_mmq behind the fused rms_norm -> Q8L prologue. That prologue must
    publish int8 Q8L blocks even though the launch before it was an f16 GEMM (ADVICE r3:
    a stale `f16` flag made the q/k/v GEMMs re-quantize a never-written f32 buffer).
    Checked: layers 0-2 (no f16 GEMM before them) bit-exact; layer 3's K cache, the first
    behind ONE f16 GEMM (layer 2's ffn_down), within a relative L2 error of 2^-7 of the
    bit-exact prompt's (one GEMM's stated bound carried through a residual add, a norm and
    the k projection: a regression of one layer shows there); every layer's K cache within
    2^-5 (garbage or zeros there would be ~1); and the logits within 2^-5 of the oracle's
    sequential llm_build_llama (held to ADVICE r3's 2^-5)."""
    import torch
    from oracle import kq_ops_oracle as O
    from tests import llama_model as LM
    from tests.test_gpu_ops import _decoder
    import ggml_mi355x as g
    from ggml_mi355x.llama import hparams
    O.lib()
    hp = hparams(2048, 5, 32, 4, 5632, 4096)
    assert [LM.use_more_bits(i, 5) for i in range(5)] == [False, False, True, False, True]
    n_ctx, n = 64, 29
    tokens = np.random.default_rng(17).integers(0, hp["n_vocab"], size=n).tolist()
    out = {}
    for name, prec in (("exact", g.PREFILL_EXACT), ("f16_auto", g.PREFILL_F16)):
        g.prefill_precision(prec)
        w, b, dec = _decoder(dev, hp, 11, n_ctx, True)
        lg = dec.prompt(tokens, 0)
        b.synchronize()
        out[name] = (lg.cpu().numpy().astype(np.float64).ravel(),
                     [c[:n].view(torch.float16).float().cpu().numpy() for c in dec.k_cache])
        b.close()
    g.prefill_precision(g.PREFILL_F16_ALL)
    errs = []
    for li in range(5):
        k, ke = out["f16_auto"][1][li], out["exact"][1][li]
        assert np.isfinite(k).all(), li
        errs.append(float(np.linalg.norm(k - ke) / np.linalg.norm(ke)))
    print("K-cache relative L2 per layer:", errs)
    assert errs[0] == errs[1] == errs[2] == 0.0, errs
    assert errs[3] <= 2.0 ** -7, errs
    assert max(errs) <= 2.0 ** -5, errs
    model, cache = LM.oracle_model(hp, w, n_ctx)
    for p, tok in enumerate(tokens):
        ref, _ = O.decode_token(model, tok, p, cache)
    ref = np.asarray(ref, np.float64).ravel()
    assert np.array_equal(out["exact"][0], ref)
    got = out["f16_auto"][0]
    rel = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    print("logits relative L2:", rel)
    assert np.isfinite(got).all() and rel <= 2.0 ** -5, rel
    torch.cuda.synchronize()


@pytest.mark.parametrize("K,Ns,M", [(2048, (2048, 256, 256), 37), (4096, (4096, 1024, 1024), 128),
                                    (1024, (300, 130), 200)], ids=["tl_qkv", "l3_qkv", "ragged"])
def test_mmf_multi_matrix_launch(dev, oracle, npo, f16path, K, Ns, M):
    """Several MUL_MATs on one activation in one backend graph run as ONE f16 launch (row
    tiles per matrix, slab columns per matrix for split-K): every output within the stated
    bound of the oracle, and equal to the single-matrix launches up to f32 summation order."""
    import ggml_mi355x as g
    rng = np.random.default_rng(K + sum(Ns) + M)
    be = g.Backend()
    x = rng.standard_normal((M, K)).astype(np.float32)
    xp = be.alloc(x.nbytes)
    be.set_tensor(xp, x)
    xt = g.make_tensor(g.TYPE_F32, K, M, xp)
    ws, nodes, outs, keep = [], [], [], [xt]
    for N in Ns:
        w = npo.random_blocks(rng, 12, N, K)
        p = be.alloc(w.nbytes)
        be.set_tensor(p, w)
        wt = g.make_tensor(12, K, N, p)
        y = be.alloc(M * N * 4)
        nodes.append(g.make_tensor(g.TYPE_F32, N, M, y, op=g.OP_MUL_MAT, src0=wt, src1=xt))
        ws.append(w)
        outs.append(y)
        keep.append(wt)
    assert be.graph_compute(nodes, use_graph=True) == 0
    be.synchronize()
    for w, y, N in zip(ws, outs, Ns):
        got = np.zeros((M, N), np.float32)
        be.get_tensor(got, y)
        be.synchronize()
        check(got, w, 12, K, x, oracle, npo)
        single = g.mul_mat(12, t(w, dev), K, t(x, dev)).cpu().numpy().astype(np.float64)
        bound = npo.mmf_bound(w, 12, K, x)
        assert (np.abs(got.astype(np.float64) - single) <= bound * 2.0 ** -6).all()
    be.close()
