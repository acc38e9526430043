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
    import ggml_mi355x as g
    prev = g.prefill_precision(g.PREFILL_F16)
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
    assert g.prefill_precision(prev) == g.PREFILL_F16
    assert g.lib().mi355x_prefill_precision(7) == g.E_INVAL
