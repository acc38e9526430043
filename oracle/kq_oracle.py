"""ctypes binding of the C oracle (oracle/_build/libkq_oracle.so).

TEST INFRASTRUCTURE ONLY — the checker used by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg. The product package never imports this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libkq_oracle.so")
Q4_K, Q5_K, Q6_K, Q8_K = 12, 13, 14, 15
BLOCK_BYTES = {Q4_K: 144, Q5_K: 176, Q6_K: 210, Q8_K: 292}

_lib = None
VARIANTS = {"neon": 0, "generic": 1, "simd": 2}  # simd: AVX2 integer parts, bit-identical to neon


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i64, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int
        L.kqo_quantize_row_q8_K.argtypes = [vp, vp, i64, i32]
        for name in ("kqo_vec_dot_q4_K_q8_K_neon", "kqo_vec_dot_q4_K_q8_K_generic", "kqo_vec_dot_q5_K_q8_K_neon",
                     "kqo_vec_dot_q6_K_q8_K_neon", "kqo_vec_dot_q6_K_q8_K_generic", "kqo_vec_dot_q4_K_q8_K_simd",
                     "kqo_vec_dot_q5_K_q8_K_simd", "kqo_vec_dot_q6_K_q8_K_simd"):
            getattr(L, name).argtypes = [i32, vp, sz, vp, sz, vp, sz, i32]
        L.kqo_block_partials.argtypes = [i32, i32, vp, vp, vp]
        L.kqo_mul_mat.argtypes = [i32, vp, i64, i64, sz, vp, i64, sz, vp, i32, i32]
        L.kqo_mul_mat.restype = i32
        L.kqo_mul_mat_q8.argtypes = [i32, vp, i64, i64, sz, vp, i64, vp, i32, i32]
        L.kqo_mul_mat_q8.restype = i32
        L.kqo_fp16_to_fp32.argtypes = [ctypes.c_uint16]
        L.kqo_fp16_to_fp32.restype = ctypes.c_float
        L.kqo_fp32_to_fp16.argtypes = [ctypes.c_float]
        L.kqo_fp32_to_fp16.restype = ctypes.c_uint16
        L.kqo_dequantize_row_q4_K.argtypes = [vp, vp, i64]
        L.kqo_dequantize_row_q5_K.argtypes = [vp, vp, i64]
        L.kqo_dequantize_row_q6_K.argtypes = [vp, vp, i64]
        L.kqo_set_contraction_variant.argtypes = [i32, i32]
        _lib = L
    return _lib


class contraction_variant:
    """with contraction_variant(which, v): the Q5_K (which 0) or Q6_K (which 1) fp32 update
    as one of the [U] alternatives of kq_oracle.c (0 = the restatement's gcc choice); tests
    only."""

    def __init__(self, which, v):
        self.which, self.v = which, v

    def __enter__(self):
        lib().kqo_set_contraction_variant(self.which, self.v)
        return self

    def __exit__(self, *exc):
        lib().kqo_set_contraction_variant(self.which, 0)
        return False


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def quantize_q8_K(x, fused=True):
    """x: (M, K) float32 -> (M, K/256*292) uint8 Q8_K rows."""
    x = np.ascontiguousarray(x, np.float32)
    if x.ndim == 1:
        x = x[None]
    M, K = x.shape
    out = np.zeros((M, K // 256 * 292), np.uint8)
    for i in range(M):
        lib().kqo_quantize_row_q8_K(_p(x[i]), _p(out[i]), K, 1 if fused else 0)
    return out


def vec_dot(type_, w_row, q8_row, K, variant="neon"):
    w_row = np.ascontiguousarray(w_row, np.uint8)
    q8_row = np.ascontiguousarray(q8_row, np.uint8)
    s = np.zeros(1, np.float32)
    name = {(Q4_K, "neon"): "kqo_vec_dot_q4_K_q8_K_neon", (Q4_K, "generic"): "kqo_vec_dot_q4_K_q8_K_generic",
            (Q5_K, "neon"): "kqo_vec_dot_q5_K_q8_K_neon", (Q6_K, "neon"): "kqo_vec_dot_q6_K_q8_K_neon",
            (Q6_K, "generic"): "kqo_vec_dot_q6_K_q8_K_generic", (Q4_K, "simd"): "kqo_vec_dot_q4_K_q8_K_simd",
            (Q5_K, "simd"): "kqo_vec_dot_q5_K_q8_K_simd", (Q6_K, "simd"): "kqo_vec_dot_q6_K_q8_K_simd"}[(type_, variant)]
    getattr(lib(), name)(K, _p(s), 0, _p(w_row), 0, _p(q8_row), 0, 1)
    return s[0]


def block_partials(type_, w, q8, K):
    """w: (N, rowbytes), q8: (rowbytes_q8,) one column -> (N, nb, 2) int32."""
    w = np.ascontiguousarray(w, np.uint8)
    q8 = np.ascontiguousarray(q8, np.uint8)
    N = w.shape[0]
    nb = K // 256
    out = np.zeros((N, nb, 2), np.int32)
    for r in range(N):
        lib().kqo_block_partials(type_, K, _p(w[r]), _p(q8), _p(out[r]))
    return out


def mul_mat(type_, w, x, n_threads=1, variant="neon"):
    """Restated ggml_compute_forward_mul_mat: w (N, rowbytes) uint8, x (M, K) f32 -> (M, N) f32."""
    w = np.ascontiguousarray(w, np.uint8)
    x = np.ascontiguousarray(x, np.float32)
    if x.ndim == 1:
        x = x[None]
    M, K = x.shape
    N = w.shape[0]
    out = np.zeros((M, N), np.float32)
    rc = lib().kqo_mul_mat(type_, _p(w), K, N, w.shape[1] if N else 0, _p(x), M, K * 4, _p(out), n_threads,
                           VARIANTS[variant])
    assert rc == 0
    return out


def mul_mat_q8(type_, w, q8, K, n_threads=1, variant="neon"):
    w = np.ascontiguousarray(w, np.uint8)
    q8 = np.ascontiguousarray(q8, np.uint8)
    if q8.ndim == 1:
        q8 = q8[None]
    M = q8.shape[0]
    N = w.shape[0]
    out = np.zeros((M, N), np.float32)
    rc = lib().kqo_mul_mat_q8(type_, _p(w), K, N, w.shape[1] if N else 0, _p(q8), M, _p(out), n_threads,
                              VARIANTS[variant])
    assert rc == 0
    return out


def dequantize(type_, w, K):
    w = np.ascontiguousarray(w, np.uint8)
    N = w.shape[0]
    out = np.zeros((N, K), np.float32)
    fn = {Q4_K: lib().kqo_dequantize_row_q4_K, Q5_K: lib().kqo_dequantize_row_q5_K,
          Q6_K: lib().kqo_dequantize_row_q6_K}[type_]
    for r in range(N):
        fn(_p(w[r]), _p(out[r]), K)
    return out
