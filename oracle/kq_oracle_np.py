"""kq_oracle_np — independent numpy restatement of the K-quant x Q8_K path.

TEST INFRASTRUCTURE ONLY (the checker). Imported by tests/, the smoke check and
bench.py's cpu_baseline leg; never by the product package.

Written independently of oracle/kq_oracle.c (different formulation of every
step: get_scale_min_k4 instead of the kmask shuffle, per-element gathers instead
of the NEON lane structure, float16 via numpy instead of bit twiddling) so that
agreement between the two is evidence about the restatement, not a copy of it.

Reference semantics followed (file:line under /root/reference):
  * Q4_K dot, NEON listing README.md:725-777; FP order from the disassembly:
    sumf = fma(-(float)summins, dmin, sumf)  [fmsub, README.md:551]
    sumf = fma((float)sumi, d, sumf)         [fmadd, README.md:614]
    with d = y.d*fp16(x.d), dmin = y.d*fp16(x.dmin) (README.md:727-728, 538-540).
  * Block layouts from the disassembly offsets (README.md:459-460, 472, 480, 488,
    492, 507, 522, 529, 610-611).
  * quantize_row_q8_K_ref + nearest_int (out.folded:184-186), body per upstream
    ggml-quants.c @ a3cb0474 [U]; fused: iscale*x + 12582912.f as one fma.
  * Q6_K / Q5_K: upstream NEON @ a3cb0474 [U] (Q6_K profiled, README.md:369).
Parity status: unpinned (the reference has no tests or fixtures for this path).
"""
from __future__ import annotations

import numpy as np

QK_K = 256
Q4_K, Q5_K, Q6_K, Q8_K = 12, 13, 14, 15
BLOCK_BYTES = {Q4_K: 144, Q5_K: 176, Q6_K: 210, Q8_K: 292}

F32 = np.float32
F64 = np.float64


# --------------------------------------------------------------- exact fma
def fma_f32(a, b, c):
    """Correctly rounded float32 fma(a, b, c), elementwise, via float64.

    a*b is exact in float64 (24+24 bit significands). s = p + c is rounded to
    float64; TwoSum recovers the exact error e. Rounding s+e to float32 differs
    from rounding s only when s sits exactly on a float32 midpoint and e != 0.
    """
    a = np.asarray(a, F32)
    b = np.asarray(b, F32)
    c = np.asarray(c, F32)
    with np.errstate(over="ignore", invalid="ignore"):
        p = a.astype(F64) * b.astype(F64)
        cc = c.astype(F64)
        s = p + cc
        bb = s - p
        err = (p - (s - bb)) + (cc - bb)
        r = s.astype(F32)
        r64 = r.astype(F64)
        toward = np.where(s > r64, F32(np.inf), F32(-np.inf)).astype(F32)
        other = np.nextafter(r, toward)
        mid = (r64 + other.astype(F64)) * 0.5
    fix = (s != r64) & (s == mid) & (err != 0) & np.isfinite(s)
    if np.any(fix):
        up = np.maximum(r, other)
        dn = np.minimum(r, other)
        r = np.where(fix, np.where(err > 0, up, dn), r)
    return r


def fp16_to_f32(h):
    return np.asarray(h, np.uint16).view(np.float16).astype(F32)


# --------------------------------------------------------- Q8_K quantizer
def quantize_q8_K(x, fused=True):
    """x: (..., K) float32 -> dict(d (...,nb) f32, qs (...,nb,256) i8, bsums (...,nb,16) i16)."""
    x = np.asarray(x, F32)
    K = x.shape[-1]
    assert K % QK_K == 0
    xb = x.reshape(x.shape[:-1] + (K // QK_K, QK_K))
    ax = np.abs(xb)
    idx = np.argmax(ax, axis=-1)  # first occurrence of the largest |x|
    amax = np.take_along_axis(ax, idx[..., None], -1)[..., 0]
    mx = np.take_along_axis(xb, idx[..., None], -1)[..., 0]
    zero = amax == 0
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        iscale = (F32(-127.0) / np.where(zero, F32(1), mx)).astype(F32)
    if fused:
        v = fma_f32(iscale[..., None], xb, F32(12582912.0))
    else:
        v = (iscale[..., None] * xb).astype(F32) + F32(12582912.0)
    bits = np.asarray(v, F32).view(np.int32)
    q = (bits & 0x007FFFFF) - 0x00400000
    q = np.minimum(q, 127)
    q = np.where(zero[..., None], 0, q).astype(np.int8)
    bsums = q.reshape(q.shape[:-1] + (16, 16)).astype(np.int32).sum(-1).astype(np.int16)
    d = np.where(zero, F32(0), (F32(1.0) / iscale).astype(F32)).astype(F32)
    return {"d": d, "qs": q, "bsums": bsums}


def q8_K_to_bytes(q):
    d, qs, bs = q["d"], q["qs"], q["bsums"]
    lead = d.shape
    out = np.zeros(lead + (292,), np.uint8)
    out[..., 0:4] = d.astype("<f4").view(np.uint8).reshape(lead + (4,))
    out[..., 4:260] = qs.view(np.uint8)
    out[..., 260:292] = bs.astype("<i2").view(np.uint8).reshape(lead + (32,))
    return out.reshape(lead[:-1] + (lead[-1] * 292,))


def q8_K_from_bytes(buf, nb):
    b = np.asarray(buf, np.uint8).reshape(-1, nb, 292)
    return {
        "d": b[..., 0:4].copy().view("<f4")[..., 0].astype(F32),
        "qs": b[..., 4:260].copy().view(np.int8),
        "bsums": b[..., 260:292].copy().view("<i2"),
    }


# ------------------------------------------------------------- unpackers
def _scale_min_k4(scales12):
    """get_scale_min_k4 for j = 0..7. scales12: (..., 12) uint8 -> (sc, m) (..., 8) int32."""
    q = scales12.astype(np.int32)
    sc = np.empty(q.shape[:-1] + (8,), np.int32)
    mn = np.empty_like(sc)
    for j in range(8):
        if j < 4:
            sc[..., j] = q[..., j] & 63
            mn[..., j] = q[..., j + 4] & 63
        else:
            sc[..., j] = (q[..., j + 4] & 0xF) | ((q[..., j - 4] >> 6) << 4)
            mn[..., j] = (q[..., j + 4] >> 4) | ((q[..., j] >> 6) << 4)
    return sc, mn


def split_blocks(w, type_, K):
    """w: (N, nb*block_bytes) uint8 -> structured fields."""
    nb = K // QK_K
    B = BLOCK_BYTES[type_]
    b = np.asarray(w, np.uint8).reshape(-1, nb, B)
    if type_ == Q4_K:
        return {"d": b[..., 0:2].copy().view("<u2")[..., 0], "dmin": b[..., 2:4].copy().view("<u2")[..., 0],
                "scales": b[..., 4:16], "qs": b[..., 16:144]}
    if type_ == Q5_K:
        return {"d": b[..., 0:2].copy().view("<u2")[..., 0], "dmin": b[..., 2:4].copy().view("<u2")[..., 0],
                "scales": b[..., 4:16], "qh": b[..., 16:48], "qs": b[..., 48:176]}
    if type_ == Q6_K:
        return {"ql": b[..., 0:128], "qh": b[..., 128:192], "scales": b[..., 192:208].view(np.int8),
                "d": b[..., 208:210].copy().view("<u2")[..., 0]}
    raise ValueError(type_)


def weights_int(w, type_, K):
    """Per-element integer quant values q (N, nb, 256) and per-16/32 scales."""
    f = split_blocks(w, type_, K)
    if type_ in (Q4_K, Q5_K):
        qs = f["qs"].astype(np.int32)  # (N, nb, 128)
        q = np.empty(qs.shape[:-1] + (256,), np.int32)
        for j in range(4):
            lo = qs[..., 32 * j:32 * j + 32] & 0xF
            hi = qs[..., 32 * j:32 * j + 32] >> 4
            if type_ == Q5_K:
                qh = f["qh"].astype(np.int32)
                lo = lo + (((qh >> (2 * j)) & 1) << 4)
                hi = hi + (((qh >> (2 * j + 1)) & 1) << 4)
            q[..., 64 * j:64 * j + 32] = lo
            q[..., 64 * j + 32:64 * j + 64] = hi
        sc, mn = _scale_min_k4(f["scales"])
        return q, sc, mn, f
    if type_ == Q6_K:
        ql = f["ql"].astype(np.int32)
        qh = f["qh"].astype(np.int32)
        q = np.empty(ql.shape[:-1] + (256,), np.int32)
        for n in range(2):
            for l in range(32):
                b0 = ql[..., 64 * n + l]
                b1 = ql[..., 64 * n + 32 + l]
                h = qh[..., 32 * n + l]
                q[..., 128 * n + l] = (b0 & 0xF) | ((h & 3) << 4)
                q[..., 128 * n + 32 + l] = (b1 & 0xF) | (((h >> 2) & 3) << 4)
                q[..., 128 * n + 64 + l] = (b0 >> 4) | (((h >> 4) & 3) << 4)
                q[..., 128 * n + 96 + l] = (b1 >> 4) | (((h >> 6) & 3) << 4)
        return q, f["scales"].astype(np.int32), None, f
    raise ValueError(type_)


def block_partials(w, type_, K, q8):
    """Integer partials per (row, col, block): sumi, summins (int64 arrays (N, M, nb))."""
    q, sc, mn, _ = weights_int(w, type_, K)
    qs8 = q8["qs"].astype(np.int64)  # (M, nb, 256)
    bs = q8["bsums"].astype(np.int64)  # (M, nb, 16)
    N, nb, _ = q.shape
    if type_ in (Q4_K, Q5_K):
        # dot per 32-subblock: (N, M, nb, 8)
        d32 = np.einsum("nbsl,mbsl->nmbs", q.reshape(N, nb, 8, 32).astype(np.int64),
                        qs8.reshape(-1, nb, 8, 32))
        sumi = np.einsum("nmbs,nbs->nmb", d32, sc.astype(np.int64))
        bs32 = bs.reshape(-1, nb, 8, 2).sum(-1)
        summins = np.einsum("mbs,nbs->nmb", bs32, mn.astype(np.int64))
        return sumi, summins
    d16 = np.einsum("nbsl,mbsl->nmbs", q.reshape(N, nb, 16, 16).astype(np.int64),
                    qs8.reshape(-1, nb, 16, 16))
    isum = np.einsum("nmbs,nbs->nmb", d16, sc.astype(np.int64))
    isum_mins = np.einsum("mbs,nbs->nmb", bs, sc.astype(np.int64))
    return isum, isum_mins


def mul_mat_q8(w, type_, K, q8):
    """dst (M, N) float32 following the reference NEON fp order per (row, col)."""
    a, b = block_partials(w, type_, K, q8)
    f = split_blocks(w, type_, K)
    yd = q8["d"].astype(F32)  # (M, nb)
    N, M, nb = a.shape
    s = np.zeros((N, M), F32)
    if type_ == Q4_K:
        xd = fp16_to_f32(f["d"])
        xm = fp16_to_f32(f["dmin"])
        for i in range(nb):
            d = (yd[None, :, i] * xd[:, None, i]).astype(F32)
            dmin = (yd[None, :, i] * xm[:, None, i]).astype(F32)
            s = fma_f32(-(b[:, :, i].astype(F32)), dmin, s)
            s = fma_f32(a[:, :, i].astype(F32), d, s)
    elif type_ == Q5_K:
        xd = fp16_to_f32(f["d"])
        xm = fp16_to_f32(f["dmin"])
        for i in range(nb):
            d = (yd[None, :, i] * xd[:, None, i]).astype(F32)
            dmin = (yd[None, :, i] * xm[:, None, i]).astype(F32)
            t = fma_f32(d, a[:, :, i].astype(F32), -(dmin * b[:, :, i].astype(F32)).astype(F32))
            s = (s + t).astype(F32)
    else:
        xd = fp16_to_f32(f["d"])
        for i in range(nb):
            dd = (xd[:, None, i] * yd[None, :, i]).astype(F32)
            s = fma_f32(dd, (a[:, :, i] - 32 * b[:, :, i]).astype(F32), s)
    return s.T.copy()


def dequantize(w, type_, K):
    """float64 dequantized weights (exact products; for tolerance checks only)."""
    q, sc, mn, f = weights_int(w, type_, K)
    N, nb, _ = q.shape
    if type_ in (Q4_K, Q5_K):
        d = fp16_to_f32(f["d"]).astype(F64)[..., None]
        dm = fp16_to_f32(f["dmin"]).astype(F64)[..., None]
        scl = np.repeat(sc, 32, axis=-1).astype(F64)
        mnl = np.repeat(mn, 32, axis=-1).astype(F64)
        return (d * scl * q - dm * mnl).reshape(N, nb * 256)
    d = fp16_to_f32(f["d"]).astype(F64)[..., None]
    scl = np.repeat(sc, 16, axis=-1).astype(F64)
    return (d * scl * (q - 32)).reshape(N, nb * 256)


# ------------------------------------------------------------ generators
def random_blocks(rng, type_, N, K, d_lo=2.0 ** -14, d_hi=2.0 ** -6):
    """Random but valid K-quant rows: every qs/scales bit pattern is a legal
    block; d/dmin are fp16 of U[d_lo, d_hi] (finite, normal)."""
    nb = K // QK_K
    B = BLOCK_BYTES[type_]
    raw = rng.integers(0, 256, size=(N, nb, B), dtype=np.uint8)

    def f16(n):
        return rng.uniform(d_lo, d_hi, size=(N, nb)).astype(np.float16).view(np.uint16)

    if type_ in (Q4_K, Q5_K):
        raw[..., 0:2] = f16(0)[..., None].view(np.uint8).reshape(N, nb, 2)
        raw[..., 2:4] = f16(0)[..., None].view(np.uint8).reshape(N, nb, 2)
    elif type_ == Q6_K:
        raw[..., 208:210] = f16(0)[..., None].view(np.uint8).reshape(N, nb, 2)
    return raw.reshape(N, nb * B)


# ------------------------------------------- f16 prefill path (kq_mmf), stated tolerance
def mmf_operands(w, type_, K, x):
    """The operands kq_mmf feeds the f16 matrix core, as float64 of their f16 values, and
    the per-element magnitude A used by the tolerance bound.

    Returns (W16 (N, K), X16 (M, K), G16w (N, nb*16), G16x (M, nb*16), A (N, K), Xhat (M, K)):
    y ~= W16 @ X16.T + G16w @ G16x.T (main + per-group terms, csrc/kq_mmf.hip header)."""
    nb = K // QK_K
    q, sc, mn, f = weights_int(w, type_, K)
    N = q.shape[0]
    f16 = np.float16
    q8 = quantize_q8_K(x)
    d = q8["d"].astype(F32)                                # (M, nb)
    qs = q8["qs"].astype(F32)                              # (M, nb, 256)
    X16 = (d[..., None] * qs).astype(F32).astype(f16).astype(F64).reshape(-1, K)
    Xhat = (d[..., None].astype(F64) * qs.astype(F64)).reshape(-1, K)
    bs16 = q8["bsums"].astype(F32)                         # (M, nb, 16)
    G16x = (d[..., None] * bs16).astype(F32).astype(f16).astype(F64).reshape(-1, nb * 16)
    if type_ in (Q4_K, Q5_K):
        dd = fp16_to_f32(f["d"])[..., None]                # (N, nb, 1)
        dm = fp16_to_f32(f["dmin"])[..., None]
        dsc = (dd * sc.astype(F32)).astype(f16)            # (N, nb, 8) one rounding
        W16 = (np.repeat(dsc.astype(F64), 32, -1) * q).astype(f16).astype(F64).reshape(N, K)
        mneg = -(dm * mn.astype(F32)).astype(f16).astype(F64)  # (N, nb, 8)
        G16w = np.repeat(mneg, 2, -1).reshape(N, nb * 16)
        A = (np.repeat(np.abs(dsc.astype(F64)), 32, -1) * q + np.repeat(np.abs(mneg), 32, -1)).reshape(N, K)
    else:
        dd = fp16_to_f32(f["d"])[..., None]
        dsc = (dd * sc.astype(F32)).astype(f16)            # (N, nb, 16)
        W16 = (np.repeat(dsc.astype(F64), 16, -1) * q).astype(f16).astype(F64).reshape(N, K)
        G16w = (-32.0 * dsc.astype(F64)).reshape(N, nb * 16)
        A = (np.repeat(np.abs(dsc.astype(F64)), 16, -1) * (q + 32)).reshape(N, K)
    return W16, X16, G16w, G16x, A, Xhat


def mmf_emulate(w, type_, K, x):
    """kq_mmf's value up to the f32 accumulation order: (M, N) float64."""
    W16, X16, G16w, G16x, _, _ = mmf_operands(w, type_, K, x)
    return X16 @ W16.T + G16x @ G16w.T


MMF_REL_TOL = 2.0 ** -8


def mmf_bound(w, type_, K, x):
    """Stated tolerance of the f16 prefill path against the bit-exact reference (M, N):
    2^-8 * sum_k A_k |x^_k| + 2^-24 * K * max A * max |x^|, with A_k = |f16(d sc)| q_k +
    |f16(dmin m)| (Q4_K/Q5_K) or |f16(d sc)| (q_k + 32) (Q6_K) and x^ = y.d * q8."""
    _, _, _, _, A, Xhat = mmf_operands(w, type_, K, x)
    S = np.abs(Xhat) @ A.T
    return MMF_REL_TOL * S + 2.0 ** -24 * K * float(A.max(initial=0.0)) * float(np.abs(Xhat).max(initial=0.0))
