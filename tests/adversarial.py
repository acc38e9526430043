"""Inputs built to separate summation orders (test data, not a checker).

rms_norm: ggml sums (double)(x*x) sequentially (ggml_compute_forward_rms_norm_f32);
the GPU's fast path sums in a tree order (kq_ops_device.h). `order_split_rows` builds
rows whose float mean differs between the two orders, so a GPU result equal to the
oracle's proves the exactness guard (rms_mean_ambiguous -> sequential re-sum) ran.

Construction for n = 256 * nb: S_big = n + n * 2^-24 made of exact float squares
(x = 32-multiples and 2^-7-like values), so mean_seq = 1 + 2^-24 exactly: a float
rounding tie that goes to 1.0f (even). Sixteen tiny squares tau = ulp(S_big) / 8 sit
in one 16-element group: each is rounded away by the sequential adds, but the tree adds
the group first (16 tau, exact) and that survives, so mean_tree = 1 + 2^-24 + 16tau/n
rounds UP to 1 + 2^-23. Rows are scaled by powers of two (squares scale exactly).
"""
from __future__ import annotations

import numpy as np


def _tree_sumsq(x):
    """The GPU's fast order (kq_ops_device.h): per 16 a sequential double sum, a
    xor-1/2/4/8 tree over the 16 groups of a superblock, superblocks in order."""
    x = np.asarray(x, np.float32)
    tot = 0.0
    for b in range(x.size // 256):
        g = []
        for k in range(16):
            s = 0.0
            for v in x[256 * b + 16 * k: 256 * b + 16 * k + 16]:
                s += float(np.float32(v) * np.float32(v))
            g.append(s)
        for step in (1, 2, 4, 8):
            g = [g[i] + g[i ^ step] for i in range(16)]
        tot += g[0]
    return tot


def _seq_sumsq(x):
    tot = 0.0
    for v in np.asarray(x, np.float32):
        tot += float(np.float32(v) * np.float32(v))
    return tot


def order_split_rows(n, count=6, seed=0):
    """Rows of n floats (n a power of two >= 1024) whose rms_norm float mean differs
    between the sequential and the tree order. Returns (rows, means_seq, means_tree)."""
    assert n >= 1024 and n & (n - 1) == 0
    L = n.bit_length() - 1
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(count):
        x = np.zeros(n, np.float32)
        # two distinct 16-element groups, the tiny one later (sequentially it meets the big sum)
        gbig, gtiny = sorted(int(v) for v in rng.permutation(n // 16)[:2])
        terms = [32.0] * (n // 1024)                 # squares 1024 each: sum n
        e = L - 25                                   # n * 2^-24 = 2 * 2^e
        terms += [2.0 ** (e // 2)] * 2 if e % 2 == 0 else [2.0 ** ((e - 1) // 2)] * 4
        x[16 * gbig: 16 * gbig + len(terms)] = terms
        et = L - 55 - ((L - 55) % 2)                 # tau = (2^(et/2))^2 <= ulp(n) / 8
        x[16 * gtiny: 16 * gtiny + 16] = 2.0 ** (et // 2)
        rows.append(x * np.float32(2.0 ** int(rng.integers(-6, 7))))
    rows = np.stack(rows).astype(np.float32)
    ms = np.array([np.float32(_seq_sumsq(r) / n) for r in rows], np.float32)
    mt = np.array([np.float32(_tree_sumsq(r) / n) for r in rows], np.float32)
    return rows, ms, mt
