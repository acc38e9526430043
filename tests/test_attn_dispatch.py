"""The decode attention dispatch policy (mi355x_attn_path: no launch, no device access), on the CPU.

DESIGN.md §4 "KQ split over cells" and profiles/r06_ctx_ab.txt measured where each kernel pays:
one workgroup per head (register path) up to 256 cells; each head split by output over 4 / 8
workgroups past them; the two-launch split over cells for caches of more than 1024 cells where
the output split would need 8 slices or does not fit. The GPU tests run every path; this pins
which one a shape takes."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]


@pytest.fixture(scope="module")
def g():
    import ggml_mi355x as g
    if not os.path.exists(g.LIB_PATH):
        pytest.skip("library not built")
    return g


TINY = (32, 4, 64)   # TinyLlama: n_head, n_head_kv, head_dim
L3_8B = (32, 8, 128)  # Llama-3-8B


@pytest.mark.parametrize("shape,n_ctx,path", [
    (TINY, 32, "HEAD"), (TINY, 256, "HEAD"), (TINY, 512, "SPLIT4"), (TINY, 1024, "SPLIT4"),
    (TINY, 2048, "SPLIT4"), (TINY, 3072, "CELLS"), (TINY, 4096, "CELLS"), (TINY, 6144, "CELLS"),
    (L3_8B, 256, "HEAD"), (L3_8B, 1024, "SPLIT4"), (L3_8B, 2048, "CELLS"), (L3_8B, 4096, "CELLS"),
    (L3_8B, 6144, "CELLS"),
])
def test_attn_dispatch_default(g, shape, n_ctx, path):
    nh, nkv, hd = shape
    assert g.attn_path(n_ctx, nh, nkv, hd) == getattr(g, "ATTN_PATH_" + path)


def test_attn_dispatch_alignment_and_limits(g):
    # the staged rope row of the decode graph sits 8 B into its tensor: the split still runs
    # (its f32 vectors need 4-B alignment; the caches 16 B, which attn_decode requires anyway)
    assert g.attn_path(2048, 32, 4, 64, f32_offset=8) == g.ATTN_PATH_SPLIT4
    assert g.attn_path(4096, 32, 4, 64, f32_offset=8) == g.ATTN_PATH_CELLS
    # f32 vectors not 4-B aligned: no output split (it stages them by LDS-DMA); the split over
    # cells reads them with plain loads and takes the cache (measured equal at 2048 cells)
    assert g.attn_path(2048, 32, 4, 64, f32_offset=2) == g.ATTN_PATH_CELLS
    assert g.attn_path(1024, 32, 4, 64, f32_offset=2) == g.ATTN_PATH_HEAD_BATCH  # (<= 1024 cells: per head)
    assert g.attn_path(2048, 32, 4, 64, cache_offset=8) == g.E_INVAL  # caches must be 16-B aligned
    assert g.attn_path(8192, 32, 4, 64) == g.E_UNSUPPORTED  # past the per-head kernel's LDS
    assert g.attn_path(100, 32, 4, 64) == g.E_UNSUPPORTED   # n_ctx % 32
    assert g.attn_path(1024, 32, 4, 96) == g.E_UNSUPPORTED  # head_dim


def test_attn_dispatch_selectors(g):
    prev = g.attn_impl(g.ATTN_HEAD)
    try:
        assert g.attn_path(128, 32, 4, 64) == g.ATTN_PATH_HEAD
        assert g.attn_path(4096, 32, 4, 64) == g.ATTN_PATH_HEAD_BATCH  # every size on one workgroup per head
    finally:
        g.attn_impl(prev)
    assert g.attn_path(4096, 32, 4, 64) == g.ATTN_PATH_CELLS
