"""CPU: the stated tolerance of the f16 prefill path (kq_mmf, MI355X_PREFILL_F16).

oracle/kq_oracle_np.py mmf_emulate restates what kq_mmf feeds its f16 matrix core (the
reference's Q8_K activation d*q rounded to f16 once, the weight f16(d*sc)*q rounded once,
the mins / q-32 offset as per-16-element-group products) in float64; mmf_bound is the
tolerance the GPU tests hold the kernel to. Here the emulation is checked against the
bit-exact reference restatement (kq_oracle.mul_mat, README.md:686-779 order) with a
30x margin, so the bound is a property of the design and not of one kernel build.
"""
import numpy as np
import pytest


@pytest.mark.parametrize("type_", [12, 13, 14], ids=["q4_K", "q5_K", "q6_K"])
@pytest.mark.parametrize("K,N,M", [(256, 40, 17), (768, 33, 16), (2048, 64, 24)])
def test_mmf_emulation_within_stated_bound(oracle, npo, type_, K, N, M):
    rng = np.random.default_rng(K + 3 * N + 5 * M + type_)
    w = npo.random_blocks(rng, type_, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    x[0, :256] = 0.0                     # an all-zero Q8_K block (d = 0)
    x[1, 256 % K:] *= 1e3                # a wide dynamic range across blocks
    ref = oracle.mul_mat(type_, w, x).astype(np.float64)
    emu = npo.mmf_emulate(w, type_, K, x)
    bound = npo.mmf_bound(w, type_, K, x)
    assert np.isfinite(emu).all()
    assert (np.abs(emu - ref) <= bound / 30).all(), float((np.abs(emu - ref) / bound).max())


def test_mmf_bound_is_not_vacuous(oracle, npo):
    """An indexing slip (the two 16-element halves of every 32-element sub-block swapped on
    the activation side) must break the bound on most outputs."""
    rng = np.random.default_rng(9)
    K, N, M = 512, 8, 16
    w = npo.random_blocks(rng, 12, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    ref = oracle.mul_mat(12, w, x).astype(np.float64)
    xs = x.reshape(M, K // 32, 2, 16)[:, :, ::-1].reshape(M, K).copy()
    bad = npo.mmf_emulate(w, 12, K, xs)
    assert (np.abs(bad - ref) > npo.mmf_bound(w, 12, K, x)).mean() > 0.5
