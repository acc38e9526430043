"""CPU checks of the decode-op oracle (oracle/kq_ops_oracle.c) and of the host side
of the decode graph: the exact binary16 arithmetic against rational arithmetic,
ggml_v_expf's accuracy, each op against a float64 statement of its math, a whole
tiny llama token, and supports_op for the new node types."""
import math
from fractions import Fraction

import numpy as np
import pytest


@pytest.fixture(scope="module")
def O():
    from oracle import kq_ops_oracle
    kq_ops_oracle.lib()
    return kq_ops_oracle


def h2f(h):
    return float(np.array([h], np.uint16).view(np.float16)[0])


def nearest_f16(x: Fraction, neg_zero=False):
    """Correctly rounded (RNE) binary16 of an exact rational, as bits."""
    if x == 0:
        return 0x8000 if neg_zero else 0
    best = None
    # candidates around float(x)
    f = float(x)
    c = int(np.array([f], np.float16).view(np.uint16)[0])
    for d in range(-2, 3):
        h = (c + d) & 0xFFFF
        if (h & 0x7C00) == 0x7C00:
            continue
        if (h & 0x8000) != (0x8000 if x < 0 else 0) and (h & 0x7FFF):
            continue
        err = abs(Fraction(h2f(h)) - x)
        key = (err, (h & 1))  # ties -> even mantissa
        if best is None or key < best[0]:
            best = (key, h)
    return best[1]


def test_f16_fma_add_exact(O):
    rng = np.random.default_rng(0)
    for _ in range(4000):
        a, b, c = (int(v) for v in rng.integers(0, 0x7C00, 3))
        a |= int(rng.integers(0, 2)) << 15
        c |= int(rng.integers(0, 2)) << 15
        ex = Fraction(h2f(a)) * Fraction(h2f(b)) + Fraction(h2f(c))
        r = O.f16_fma(a, b, c)
        if abs(ex) >= 65520:
            assert (r & 0x7FFF) == 0x7C00
            continue
        if ex != 0:
            assert r == nearest_f16(ex), (hex(a), hex(b), hex(c), hex(r))
        s = Fraction(h2f(a)) + Fraction(h2f(c))
        if s != 0 and abs(s) < 65520:
            assert O.f16_add(a, c) == nearest_f16(s)
    # signed zeros: (-0)+(-0) = -0, x + (-x) = +0, fma(-1, 0, -0) = -0
    assert O.f16_add(0x8000, 0x8000) == 0x8000
    assert O.f16_add(0x3C00, 0xBC00) == 0
    assert O.f16_fma(0xBC00, 0x0000, 0x8000) == 0x8000
    assert O.f16_fma(0x0001, 0x0001, 0x0000) == 0  # 2^-48 rounds to +0


def test_v_expf_accuracy(O):
    x = np.concatenate([np.linspace(-87, 88, 50001), np.array([0.0, -0.0, 1e-8, -1e-8])]).astype(np.float32)
    e = O.v_expf(x)
    ref = np.exp(x.astype(np.float64))
    rel = np.abs(e - ref) / ref
    assert rel.max() < 4 * 2.0 ** -24  # a few ulp (ggml's polynomial)
    assert O.v_expf(np.array([-np.inf, -200.0], np.float32)).tolist() == [0.0, 0.0]


def test_vec_dot_f16(O):
    rng = np.random.default_rng(1)
    for n in (32, 64, 96, 128, 256, 70):
        x = O.fp32_to_fp16(rng.standard_normal(n))
        y = O.fp32_to_fp16(rng.standard_normal(n))
        ref = float(np.dot(x.view(np.float16).astype(np.float64), y.view(np.float16).astype(np.float64)))
        got = float(O.vec_dot_f16(x, y))
        assert abs(got - ref) <= 2e-3 * (1 + math.sqrt(n)), (n, got, ref)


def test_soft_max_rms_swiglu_rope(O):
    rng = np.random.default_rng(2)
    s = (rng.standard_normal(96) * 5).astype(np.float32)
    m = np.where(np.arange(96) < 70, 0.0, -np.inf).astype(np.float32)
    p = O.soft_max_row(s, m, 0.125)
    w = s.astype(np.float64) * 0.125 + m
    ref = np.exp(w - w.max())
    ref /= ref.sum()
    assert np.abs(p - ref).max() < 1e-6 and (p[70:] == 0).all()
    x = rng.standard_normal(2048).astype(np.float32)
    assert np.allclose(O.rms_norm(x, 1e-5), x / np.sqrt((x.astype(np.float64) ** 2).mean() + 1e-5), rtol=1e-6)
    g, u = rng.standard_normal(512).astype(np.float32), rng.standard_normal(512).astype(np.float32)
    ref = g / (1 + np.exp(-g.astype(np.float64))) * u
    assert np.allclose(O.swiglu(g, u), ref, rtol=1e-6, atol=1e-7)
    tab = O.rope_table(64, 64)
    q = rng.standard_normal(128).astype(np.float32)
    th = 9 * 10000.0 ** (-np.arange(32) * 2 / 64)
    q2 = q.reshape(2, 32, 2).astype(np.float64)
    ref = np.stack([q2[..., 0] * np.cos(th) - q2[..., 1] * np.sin(th),
                    q2[..., 0] * np.sin(th) + q2[..., 1] * np.cos(th)], -1).ravel()
    assert np.abs(O.rope(q, 64, 64, 9, tab) - ref).max() < 1e-5


def test_attn_decode_matches_float_attention(O):
    rng = np.random.default_rng(3)
    nh, nkv, hd, n_ctx = 8, 2, 64, 64
    kc = np.zeros((n_ctx, nkv * hd), np.uint16)
    vc = np.zeros((nkv * hd, n_ctx), np.uint16)
    K, Vv = [], []
    for p in range(10):
        q = rng.standard_normal(nh * hd).astype(np.float32)
        k = rng.standard_normal(nkv * hd).astype(np.float32)
        v = rng.standard_normal(nkv * hd).astype(np.float32)
        K.append(k)
        Vv.append(v)
        out = O.attn_decode(q, k, v, kc, vc, p, nh, nkv, hd, 0.125)
        Ka, Va = np.stack(K).reshape(p + 1, nkv, hd), np.stack(Vv).reshape(p + 1, nkv, hd)
        for h in range(nh):
            gi = h // (nh // nkv)
            sc = Ka[:, gi] @ q[h * hd:(h + 1) * hd].astype(np.float64) * 0.125
            pr = np.exp(sc - sc.max())
            pr /= pr.sum()
            ref = pr @ Va[:, gi]
            assert np.abs(out[h * hd:(h + 1) * hd] - ref).max() < 3e-2  # f16 K/V/q/p and f16 accumulation
    assert O.attn_n_kv(0, 64) == 32 and O.attn_n_kv(31, 64) == 32 and O.attn_n_kv(32, 64) == 64


def test_tiny_llama_token_oracle(O):
    from tests import llama_model as LM
    import ggml_mi355x.llama as LL
    hp = LL.hparams(256, 2, 4, 2, 512, 300)
    w = LM.build(hp, 0)
    model, cache = LM.oracle_model(hp, w, 32)
    for p, tok in enumerate([3, 299, 3]):
        logits, trace = O.decode_token(model, tok, p, cache, n_threads=2)
        assert logits.shape == (300,) and np.isfinite(logits).all() and len(trace) == 2
        assert 0.05 < float(np.sqrt((trace[-1] ** 2).mean())) < 50


def test_supports_decode_ops():
    import ggml_mi355x as g
    E, F = 2048, 5632
    x = g.make_tensor(g.TYPE_F32, E, 1, 0x1000)
    wn = g.make_tensor(g.TYPE_F32, E, 1, 0x2000)
    assert g.supports_op(g.make_tensor(g.TYPE_F32, E, 1, 0x3000, op=g.OP_RMS_NORM, src0=x, op_params=[g.f32_bits(1e-5)]))
    assert not g.supports_op(g.make_tensor(g.TYPE_F32, E + 8, 1, 0x3000, op=g.OP_RMS_NORM,
                                           src0=g.make_tensor(g.TYPE_F32, E + 8, 1, 0x1000)))
    assert g.supports_op(g.make_tensor(g.TYPE_F32, E, 1, 0x3000, op=g.OP_MUL, src0=x, src1=wn))
    assert g.supports_op(g.make_tensor(g.TYPE_F32, E, 1, 0x3000, op=g.OP_ADD, src0=x, src1=wn))
    assert not g.supports_op(g.make_tensor(g.TYPE_F32, E, 1, 0x3000, op=g.OP_ADD, src0=x,
                                           src1=g.make_tensor(g.TYPE_F32, F, 1, 0x2000)))
    gt = g.make_tensor(g.TYPE_F32, F, 1, 0x1000)
    assert g.supports_op(g.make_tensor(g.TYPE_F32, F, 1, 0x3000, op=g.OP_SWIGLU, src0=gt, src1=gt))
    emb = g.make_tensor(g.TYPE_Q4_K, E, 32000, 0x4000)
    ids = g.make_tensor(g.TYPE_I32, 1, 1, 0x5000)
    assert g.supports_op(g.make_tensor(g.TYPE_F32, E, 1, 0x3000, op=g.OP_GET_ROWS, src0=emb, src1=ids))
    assert not g.supports_op(g.make_tensor(g.TYPE_F32, E, 1, 0x3000, op=g.OP_GET_ROWS, src0=emb, src1=x))
    n_ctx, hd, nh, nkv = 256, 64, 32, 4
    tab = g.make_tensor(g.TYPE_F32, hd, n_ctx, 0x6000)
    kc = g.make_tensor(g.TYPE_F16, nkv * hd, n_ctx, 0x7000)
    vc = g.make_tensor(g.TYPE_F16, n_ctx, nkv * hd, 0x8000)
    q = g.make_tensor(g.TYPE_F32, nh * hd, 1, 0x9000)
    kv = g.make_tensor(g.TYPE_F32, nkv * hd, 1, 0xa000)
    att = g.make_tensor(g.TYPE_F32, nh * hd, 1, 0xb000, op=g.OP_ATTN_DECODE, srcs=[q, kv, kv, ids, kc, vc, tab],
                        op_params=[nh, nkv, hd, g.f32_bits(0.125)])
    assert g.supports_op(att)
    bad = g.make_tensor(g.TYPE_F32, nh * hd, 1, 0xb000, op=g.OP_ATTN_DECODE, srcs=[q, kv, kv, ids, kc, vc, tab],
                        op_params=[nh, 3, hd, g.f32_bits(0.125)])
    assert not g.supports_op(bad)
    rope = g.make_tensor(g.TYPE_F32, hd, nh, 0xc000, op=g.OP_ROPE, srcs=[g.make_tensor(g.TYPE_F32, hd, nh, 0x9000),
                                                                         ids, tab], op_params=[hd])
    assert g.supports_op(rope)
    # layout the kernels assume: an unaligned or strided RMS_NORM source, a
    # strided GET_ROWS destination and a padded KV cache are declined up front
    assert not g.supports_op(g.make_tensor(g.TYPE_F32, E, 1, 0x3000, op=g.OP_RMS_NORM,
                                           src0=g.make_tensor(g.TYPE_F32, E, 1, 0x1004)))
    assert not g.supports_op(g.make_tensor(g.TYPE_F32, E, 2, 0x3000, op=g.OP_RMS_NORM,
                                           src0=g.make_tensor(g.TYPE_F32, E, 2, 0x1000, row_stride=E * 4 + 64)))
    ids2 = g.make_tensor(g.TYPE_I32, 2, 1, 0x5000)
    assert g.supports_op(g.make_tensor(g.TYPE_F32, E, 2, 0x3000, op=g.OP_GET_ROWS, src0=emb, src1=ids2))
    assert not g.supports_op(g.make_tensor(g.TYPE_F32, E, 2, 0x3000, row_stride=E * 4 + 16, op=g.OP_GET_ROWS,
                                           src0=emb, src1=ids2))
    kc_pad = g.make_tensor(g.TYPE_F16, nkv * hd, n_ctx, 0x7000, row_stride=nkv * hd * 2 + 32)
    assert not g.supports_op(g.make_tensor(g.TYPE_F32, nh * hd, 1, 0xb000, op=g.OP_ATTN_DECODE,
                                           srcs=[q, kv, kv, ids, kc_pad, vc, tab], op_params=[nh, nkv, hd, 0]))
    kc_mis = g.make_tensor(g.TYPE_F16, nkv * hd, n_ctx, 0x7008)
    assert not g.supports_op(g.make_tensor(g.TYPE_F32, nh * hd, 1, 0xb000, op=g.OP_ATTN_DECODE,
                                           srcs=[q, kv, kv, ids, kc_mis, vc, tab], op_params=[nh, nkv, hd, 0]))


@pytest.mark.parametrize("n", [1024, 2048, 4096, 8192])
def test_rms_norm_order_split_inputs(O, n):
    """The adversarial rows really separate the orders: the oracle (ggml's sequential
    double sum) gives the sequential mean, and the GPU's fast tree order would round the
    float mean the other way (tests/adversarial.py). The GPU tests feed these rows."""
    from tests.adversarial import order_split_rows
    rows, ms, mt = order_split_rows(n)
    assert (ms != mt).all()
    eps = np.float32(1e-5)
    for r, m in zip(rows, ms):
        y = O.rms_norm(r, float(eps))
        scale = np.float32(1.0) / np.sqrt(np.float32(m + eps))
        assert (y.view(np.uint32) == (r * scale).astype(np.float32).view(np.uint32)).all()


def test_fast_binary16_ops_match_restatement():
    """The CPU baseline's binary16 FMA / add (double TwoSum with the midpoint fix,
    oracle/kq_cpu_simd.c) equal the exact 128-bit restatement on 4M random finite
    triples (subnormals, signed zeros, same-exponent operands included)."""
    from oracle import kq_ops_oracle as O
    L = O.lib()
    assert L.kqo_f16_fast_check(4_000_000, 0x9E3779B97F4A7C15) == 0
    # exact ties broken by a tiny addend: p = 1 + 2^-11 (a binary16 midpoint), c tiny
    one_plus = 0x3C00 | 1  # 1 + 2^-10
    half_ulp = 0x3800      # 0.5
    for c in (0x0001, 0x8001, 0x0000, 0x8000):
        assert L.kqo_f16_fma_fast(one_plus, half_ulp, c) == L.kqo_f16_fma(one_plus, half_ulp, c)


@pytest.mark.parametrize("pos,n_threads", [(0, 1), (5, 3), (40, 4), (127, 8)])
def test_fast_attention_matches_restatement(pos, n_threads):
    """kqo_attn_decode_fast (heads over the pool) == kqo_attn_decode, output and caches."""
    from oracle import kq_ops_oracle as O
    rng = np.random.default_rng(pos)
    nh, nkv, hd, n_ctx = 8, 2, 64, 128
    kc = rng.integers(0, 0x4600, (n_ctx, nkv * hd)).astype(np.uint16)  # |x| < 6: finite sums
    vc = rng.integers(0, 0x4600, (nkv * hd, n_ctx)).astype(np.uint16)
    kc[:, ::3] |= 0x8000
    vc[::5] |= 0x8000
    q = rng.standard_normal(nh * hd).astype(np.float32)
    k = rng.standard_normal(nkv * hd).astype(np.float32)
    v = rng.standard_normal(nkv * hd).astype(np.float32)
    kc2, vc2 = kc.copy(), vc.copy()
    a = O.attn_decode(q, k, v, kc, vc, pos, nh, nkv, hd, 0.125)
    b = O.attn_decode(q, k, v, kc2, vc2, pos, nh, nkv, hd, 0.125, fast_threads=n_threads)
    assert (a.view(np.uint32) == b.view(np.uint32)).all()
    assert (kc == kc2).all() and (vc == vc2).all()


def test_softmax_group_sum_exactness_argument():
    """The argument behind softmax_group_sum (kq_ops_device.h): when every nonzero float
    group sum g <= 4 of n terms has exponent >= floor(log2(4n)) - 29, ggml's in-order
    double sum never rounds, so any order (the GPU's wave tree) gives the same bits;
    below the threshold the orders can differ (hence the in-order fallback)."""
    import math
    rng = np.random.default_rng(7)
    for n in (8, 32, 64, 128, 2048):
        thr = int(math.floor(math.log2(4 * n))) - 29
        for trial in range(200):
            ex = rng.integers(thr, 3, size=n)
            g = (rng.uniform(1, 2, size=n) * np.exp2(ex.astype(np.float64))).astype(np.float32)
            g = np.minimum(g, np.float32(4.0))
            g[rng.random(n) < 0.2] = 0
            d = g.astype(np.float64)
            seq = 0.0
            for v in d:
                seq += v
            assert seq == math.fsum(d)  # exact: equals the exactly rounded (here: exact) sum
            perm = rng.permutation(n)
            tree = d[perm].copy()
            while len(tree) > 1:
                if len(tree) % 2:
                    tree = np.append(tree, 0.0)
                tree = tree[0::2] + tree[1::2]
            assert tree[0] == seq
    # below the threshold the orders do differ: 1 + 2^-53 + 2^-53 rounds twice in order
    # ((1 + 2^-53) ties to 1), once as (2^-53 + 2^-53) + 1
    d = np.array([1.0, 2.0 ** -53, 2.0 ** -53], np.float64)
    seq = (d[0] + d[1]) + d[2]
    assert seq != d[0] + (d[1] + d[2])


def test_get_rows_q5K_matches_numpy_restatement(O):
    """get_rows on a Q5_K table (dequantize_row_q5_K [U], the fifth bit from qh, gcc's
    contraction of d1*q - m1 as in Q4_K) equals an independent numpy restatement with an
    exact float32 fma, bit for bit."""
    from oracle import kq_oracle_np as N
    rng = np.random.default_rng(5)
    K, R = 512, 6
    nb = K // 256
    raw = rng.integers(0, 256, size=(R, nb, 176), dtype=np.uint8)
    d = rng.uniform(2.0 ** -14, 2.0 ** -6, size=(R, nb)).astype(np.float16).view(np.uint8).reshape(R, nb, 2)
    dm = rng.uniform(2.0 ** -14, 2.0 ** -6, size=(R, nb)).astype(np.float16).view(np.uint8).reshape(R, nb, 2)
    raw[..., 0:2], raw[..., 2:4] = d, dm
    table = raw.reshape(R, nb * 176)
    ids = np.array([3, 0, 5], np.int32)
    got = O.get_rows(13, table, K, ids)
    for r, i in enumerate(ids):
        ref = []
        for b in range(nb):
            blk = table[i, 176 * b: 176 * (b + 1)]
            dd = N.fp16_to_f32(blk[0:2].view(np.uint16))[0]
            mn = N.fp16_to_f32(blk[2:4].view(np.uint16))[0]
            sc, qh, qs = blk[4:16].astype(np.int32), blk[16:48].astype(np.int32), blk[48:176].astype(np.int32)

            def scale_min(j):  # get_scale_min_k4 [U]
                if j < 4:
                    return sc[j] & 63, sc[j + 4] & 63
                return (sc[j + 4] & 0xF) | ((sc[j - 4] >> 6) << 4), (sc[j + 4] >> 4) | ((sc[j] >> 6) << 4)
            for j in range(4):
                for h in range(2):
                    s, m = scale_min(2 * j + h)
                    q = ((qs[32 * j: 32 * j + 32] >> (4 * h)) & 0xF) + ((qh >> (2 * j + h)) & 1) * 16
                    d1 = np.float32(dd * np.float32(s))
                    m1 = np.float32(mn * np.float32(m))
                    ref.append(N.fma_f32(np.full(32, d1, np.float32), q.astype(np.float32), np.full(32, -m1, np.float32)))
        ref = np.concatenate(ref)
        assert (got[r].view(np.uint32) == ref.view(np.uint32)).all(), r


def _seq_sum_wave_mirror(g):
    """numpy mirror of seq_sum_wave (csrc/kq_ops_device.h): 64 terms a round, one per lane, each
    RN(g / u) in ulp units u of the running sum's binade, an in-order scan over the lanes, the
    first lane that reaches the next binade or holds a tie or a non-finite term added as is."""
    import math
    n = len(g)
    s, i0, rounds = 0.0, 0, 0
    while i0 < n and rounds < (n >> 6) + 48:
        rounds += 1
        if not s < math.inf:
            break
        ln = min(64, n - i0)
        v = np.array(g[i0:i0 + ln], np.float64)
        if s == 0.0:
            nz = np.nonzero(v != 0.0)[0]
            if len(nz) == 0:
                i0 += ln
                continue
            k = int(nz[0])
        else:
            ex = int((np.float64(s).view(np.int64) >> 52) & 0x7FF)
            sc = np.int64((2098 - ex) << 52).view(np.float64)
            uu = np.int64((ex - 52) << 52).view(np.float64)
            su = s * sc
            with np.errstate(invalid="ignore", over="ignore"):
                x = v * sc
                fin = x < np.inf
                xf = np.where(fin, x, 0.0)
                fl = ~fin | (xf - np.floor(xf) == 0.5)
                q = np.cumsum(np.where(fin, np.rint(xf), x))
                fl |= su + q >= 2.0 ** 53
            if not fl.any():
                s = float((su + q[-1]) * uu)
                i0 += ln
                continue
            k = int(np.argmax(fl))
            s = float((su + (q[k - 1] if k > 0 else 0.0)) * uu)
        s += v[k]
        i0 += k + 1
    for i in range(i0, n):
        s += g[i]
    return s


def test_seq_sum_wave_mirror_matches_in_order():
    """The wave-parallel in-order double sum (seq_sum_wave) gives the plain loop's bits on
    soft_max-like group sums from flat to very peaked, leading zeros, exact ties against the
    running sum's ulp, and non-finite terms (mirror of the device algorithm; the GPU side is
    tests/test_gpu_ops.py's peaked soft_max cases)."""
    rng = np.random.default_rng(11)
    cases = []
    for n in (1, 2, 7, 63, 64, 65, 200, 1000, 1024, 1537):
        for spread in (1.0, 8.0, 30.0, 90.0):
            w = rng.standard_normal(4 * n).astype(np.float32) * np.float32(spread)
            e = np.exp((w - w.max()).astype(np.float64)).astype(np.float32).reshape(n, 4)
            gs = ((e[:, 0] + e[:, 1]) + (e[:, 2] + e[:, 3])).astype(np.float32)
            cases.append(gs.astype(np.float64))
    z = np.zeros(300)
    z[150:] = rng.random(150) * 1e-30
    cases.append(z)
    t = np.zeros(130)
    t[0] = 1.0
    t[1:] = 2.0 ** -53  # every add an exact tie against s = 1 (ulp 2^-52)
    cases.append(t)
    t2 = np.full(129, 3.0 * 2.0 ** -53)
    t2[0] = 1.0
    cases.append(t2)
    inf = np.ones(100)
    inf[70] = np.inf
    cases.append(inf)
    nan = np.ones(100)
    nan[3] = np.nan
    cases.append(nan)
    cases.append(np.zeros(0))
    for g in cases:
        ref = 0.0
        for v in g:
            ref += v
        got = _seq_sum_wave_mirror(list(g))
        assert np.float64(got).tobytes() == np.float64(ref).tobytes() or (np.isnan(got) and np.isnan(ref)), (len(g), got, ref)


def test_softmax_sum_bound_by_total():
    """Round 6's exactness test (sum_exact_ok, kq_ops_device.h): with G the exponent of a float
    term's last mantissa bit (max(biased exponent, 1) - 150) and S any-order total, S <= (1 -
    2^-40) 2^(Gmin + 53) proves every partial sum exact, so the wave tree equals ggml's in-order
    sum; the test admits far more peaked soft_max rows than rounds 1-5's 4n bound."""
    import math
    rng = np.random.default_rng(5)
    admitted_new = admitted_old = 0
    for trial in range(400):
        n = int(rng.integers(16, 1500))
        spread = float(rng.choice([2.0, 4.0, 6.0, 9.0]))
        w = (rng.standard_normal(4 * n) * spread).astype(np.float32)
        e = np.exp((w - w.max()).astype(np.float64)).astype(np.float32).reshape(n, 4)
        g = ((e[:, 0] + e[:, 1]) + (e[:, 2] + e[:, 3])).astype(np.float32)
        nz = g[g != 0]
        ef = (nz.view(np.uint32) >> 23) & 0xFF
        gmin = int((np.maximum(ef, 1).astype(np.int64) - 150).min()) if len(nz) else 1 << 20
        d = g.astype(np.float64)
        perm = rng.permutation(n)
        tree = d[perm].copy()
        while len(tree) > 1:
            if len(tree) % 2:
                tree = np.append(tree, 0.0)
            tree = tree[0::2] + tree[1::2]
        st = float(tree[0])
        ok_new = gmin >= (1 << 20) or st <= math.ldexp(1.0 - 2.0 ** -40, gmin + 53)
        thr = int(math.floor(math.log2(4 * n))) - 29
        ok_old = all(v == 0 or (((int(np.float32(v).view(np.uint32)) >> 23) & 0xFF) - 127 >= thr and
                                ((int(np.float32(v).view(np.uint32)) >> 23) & 0xFF) != 0) for v in g)
        assert not ok_old or ok_new  # the new test admits everything the old one did
        seq = 0.0
        for v in d:
            seq += v
        if ok_new:
            admitted_new += 1
            assert st == seq == math.fsum(d)
        admitted_old += ok_old
    assert admitted_new > admitted_old
