"""GPU parity of the non-matmul decode ops and of the full llama decode token
 against the CPU oracle (oracle/kq_ops_oracle.c), through
the C-ABI.

Bar: bit-exact (every op restates ggml-cpu's arithmetic op for op). One stated
exception by construction: RMS_NORM's double sum of squares runs in a fixed tree
order on the GPU vs ggml's sequential order (kq_ops_device.h); the float results
are compared bit-exactly here and a difference would be reported as the ≤ 1-ulp
case of that note (none has been seen).
"""
import numpy as np
import pytest

from tests.test_gpu_parity import bits_equal, first_mismatch, t

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def O():
    from oracle import kq_ops_oracle
    kq_ops_oracle.lib()
    return kq_ops_oracle


# ---------------------------------------------------------------- elementwise
@pytest.mark.parametrize("type_", [0, 12, 13, 14])
def test_get_rows(dev, O, npo, type_):
    import torch
    import ggml_mi355x as g
    rng = np.random.default_rng(type_)
    K, R = 2048, 50
    if type_ == 0:
        table = rng.standard_normal((R, K)).astype(np.float32)
    else:
        table = npo.random_blocks(rng, type_, R, K)
    ids = np.array([0, 7, 49, 7, 13], np.int32)
    got = g.get_rows(type_, t(table, dev), K, t(ids, dev)).cpu().numpy()
    ref = O.get_rows(type_, table, K, ids)
    assert bits_equal(got, ref), first_mismatch(got, ref)
    torch.cuda.synchronize()


@pytest.mark.parametrize("n", [256, 2048, 5632, 8192])
def test_rms_norm(dev, O, n):
    import ggml_mi355x as g
    rng = np.random.default_rng(n)
    x = (rng.standard_normal((6, n)) * rng.uniform(1e-3, 1e3, (6, 1))).astype(np.float32)
    x[1, : n // 2] *= 1e-5  # wide dynamic range inside one row
    w = rng.uniform(0.5, 1.5, n).astype(np.float32)
    for eps in (1e-5, 1e-6):
        got = g.rms_norm(t(x, dev), eps).cpu().numpy()
        ref = O.rms_norm(x, eps)
        assert bits_equal(got, ref), first_mismatch(got, ref)
        got = g.rms_norm(t(x, dev), eps, w=t(w, dev)).cpu().numpy()
        ref = np.stack([O.mul(O.rms_norm(r, eps), w) for r in x])
        assert bits_equal(got, ref), first_mismatch(got, ref)


def test_add_mul_swiglu(dev, O):
    import ggml_mi355x as g
    rng = np.random.default_rng(5)
    n = 5632
    a = (rng.standard_normal(n) * 4).astype(np.float32)
    b = rng.standard_normal(n).astype(np.float32)
    a[:8] = [0.0, -0.0, 1e-30, -1e-30, 88.0, -88.0, 100.0, -100.0]
    a[8:16] = [-130.0, -150.0, -190.0, -200.0, 1e4, -1e4, 3.0e-39, -3.0e-39]  # v_expf slow path, denormals
    assert bits_equal(g.add(t(a, dev), t(b, dev)).cpu().numpy(), O.add(a, b))
    assert bits_equal(g.mul(t(a, dev), t(b, dev)).cpu().numpy(), O.mul(a, b))
    got = g.swiglu(t(a, dev), t(b, dev)).cpu().numpy()
    ref = O.swiglu(a, b)
    assert bits_equal(got, ref), first_mismatch(got, ref)


def test_v_expf_lanes(dev, O):
    """The soft_max/silu exponential lane for lane over its whole range (fast and slow paths)."""
    import ggml_mi355x as g
    x = np.concatenate([np.linspace(-200, 90, 20001), -np.logspace(-30, 2.3, 3000)]).astype(np.float32)
    # swiglu(x, 1) = x / (1 + v_expf(-x)): exercises v_expf at -x
    got = g.swiglu(t(x, dev), t(np.ones_like(x), dev)).cpu().numpy()
    ref = O.swiglu(x, np.ones_like(x))
    assert bits_equal(got, ref), first_mismatch(got, ref)


# ---------------------------------------------------------------- rope
@pytest.mark.parametrize("hd,nh,base", [(64, 36, 10000.0), (128, 40, 500000.0)])
def test_rope(dev, O, hd, nh, base):
    import ggml_mi355x as g
    import torch
    n_ctx = 512
    tab = g.rope_table(n_ctx, hd, base, 1.0, device=dev)
    tref = O.rope_table(n_ctx, hd, base)
    assert bits_equal(tab.cpu().numpy(), tref)  # the host C library builds both
    rng = np.random.default_rng(hd)
    x = rng.standard_normal(nh * hd).astype(np.float32) * 3
    for p in (0, 1, 37, 511):
        pos = torch.tensor([p], dtype=torch.int32, device=dev)
        got = g.rope(t(x, dev), hd, hd, pos, tab).cpu().numpy()
        ref = O.rope(x, hd, hd, p, tref)
        assert bits_equal(got, ref), (p, first_mismatch(got, ref))


# ---------------------------------------------------------------- attention
@pytest.fixture(params=[0, 1, 2], ids=["group", "head", "split"])
def attn_impl(request):
    """Runs an attention test on every kernel: one workgroup per kv group (the per-head
    kernel where the group's slice does not fit in LDS), one per query head, and (past 256
    cache cells) each head split over 4 or 8 workgroups by output."""
    import ggml_mi355x as g
    prev = g.attn_impl(request.param)
    yield request.param
    g.attn_impl(prev)


@pytest.mark.parametrize("hd,nh,nkv,n_ctx", [(64, 32, 4, 256), (128, 32, 8, 128), (64, 8, 8, 64), (64, 8, 2, 512),
                                             (128, 8, 4, 512), (64, 4, 2, 4096), (128, 64, 8, 96)])
@pytest.mark.parametrize("rope_row", [False, True])
def test_attn_decode_sequence(dev, O, attn_impl, hd, nh, nkv, n_ctx, rope_row):
    """A growing KV cache: every position's output and both caches bit-exact (positions
    past the kernel's prefetched cells — 256 K rows, 256/128 V cells — included); the
    rope table whole (row *pos read on device) or only the position's row (rope_row)."""
    import torch
    import ggml_mi355x as g
    rng = np.random.default_rng(hd + nh)
    kvw = nkv * hd
    tab = g.rope_table(n_ctx, hd, 10000.0, 1.0, device=dev)
    tref = O.rope_table(n_ctx, hd, 10000.0)
    kc = torch.zeros((n_ctx, kvw), dtype=torch.int16, device=dev)
    vc = torch.zeros((kvw, n_ctx), dtype=torch.int16, device=dev)
    kc_ref = np.zeros((n_ctx, kvw), np.uint16)
    vc_ref = np.zeros((kvw, n_ctx), np.uint16)
    scale = float(np.float32(1.0) / np.sqrt(np.float32(hd)))
    positions = list(range(0, 40)) + ([63, 64, 65, 100] if n_ctx > 100 else []) + \
        ([127, 128, 255, 256, 300] if n_ctx > 256 else []) + [n_ctx - 1]
    for p in positions:
        q = (rng.standard_normal(nh * hd) * 2).astype(np.float32)
        k = (rng.standard_normal(kvw) * 2).astype(np.float32)
        v = rng.standard_normal(kvw).astype(np.float32)
        pos = torch.tensor([p], dtype=torch.int32, device=dev)
        got = g.attn_decode(t(q, dev), t(k, dev), t(v, dev), pos, tab[p].contiguous() if rope_row else tab, kc, vc,
                            nh, nkv, hd, scale, rope_row=rope_row).cpu().numpy()
        ref = O.attn_decode(O.rope(q, hd, hd, p, tref), O.rope(k, hd, hd, p, tref), v, kc_ref, vc_ref, p, nh, nkv,
                            hd, scale)
        assert bits_equal(got, ref), (p, first_mismatch(got, ref))
    assert (kc.cpu().numpy().view(np.uint16) == kc_ref).all()
    assert (vc.cpu().numpy().view(np.uint16) == vc_ref).all()


@pytest.mark.parametrize("hd,nh,nkv,n_ctx", [(64, 32, 4, 1024), (128, 16, 4, 512), (64, 8, 2, 256), (64, 8, 2, 288),
                                             (128, 8, 2, 2048), (128, 8, 2, 288), (128, 8, 2, 1312), (64, 8, 2, 2400)])
def test_attn_decode_long_random_cache(dev, O, attn_impl, hd, nh, nkv, n_ctx):
    """Every cell of both caches random (not only the cells this test wrote), then positions
    across the whole cache: the batched loads of kq_attn_decode<HD, true> (caches past 256
    cells: two K rows per round at head_dim 64, eight V chunks per batch) and the boundary
    cache sizes on either side of that choice, bit-exact with the oracle. The split kernel
    (past 256 cells) at both head sizes, with 4 slices and with 8 (1312 / 2400 cells: sizes
    that are not whole 64-cell chunks, so the split over cells does not take them; at 2048
    cells head_dim 128 now takes the split over cells, mi355x_attn_path)."""
    import torch
    import ggml_mi355x as g
    rng = np.random.default_rng(n_ctx + hd)
    kvw = nkv * hd
    tab = g.rope_table(n_ctx, hd, 10000.0, 1.0, device=dev)
    tref = O.rope_table(n_ctx, hd, 10000.0)
    kc_ref = rng.standard_normal((n_ctx, kvw)).astype(np.float16).view(np.uint16)
    vc_ref = rng.standard_normal((kvw, n_ctx)).astype(np.float16).view(np.uint16)
    kc = torch.from_numpy(kc_ref.view(np.int16).copy()).to(dev)
    vc = torch.from_numpy(vc_ref.view(np.int16).copy()).to(dev)
    scale = float(np.float32(1.0) / np.sqrt(np.float32(hd)))
    for p in sorted(x for x in {0, 31, 32, 255, 256, 257, n_ctx // 2 + 7, n_ctx - 9, n_ctx - 1} if x < n_ctx):
        q = (rng.standard_normal(nh * hd) * 2).astype(np.float32)
        k = (rng.standard_normal(kvw) * 2).astype(np.float32)
        v = rng.standard_normal(kvw).astype(np.float32)
        pos = torch.tensor([p], dtype=torch.int32, device=dev)
        got = g.attn_decode(t(q, dev), t(k, dev), t(v, dev), pos, tab[p].contiguous(), kc, vc, nh, nkv, hd, scale,
                            rope_row=True).cpu().numpy()
        ref = O.attn_decode(O.rope(q, hd, hd, p, tref), O.rope(k, hd, hd, p, tref), v, kc_ref, vc_ref, p, nh, nkv,
                            hd, scale)
        assert bits_equal(got, ref), (p, first_mismatch(got, ref))
    assert (kc.cpu().numpy().view(np.uint16) == kc_ref).all()
    assert (vc.cpu().numpy().view(np.uint16) == vc_ref).all()


@pytest.mark.parametrize("hd,nh,nkv,n_ctx,qs", [(64, 32, 4, 4096, 2.0), (128, 32, 8, 4096, 2.0), (64, 8, 2, 6144, 2.0),
                                                 (128, 16, 2, 3072, 2.0), (64, 32, 4, 4096, 40.0), (128, 32, 8, 4096, 40.0),
                                                 (128, 8, 2, 6144, 2.0)])
def test_attn_decode_cells_split(dev, O, hd, nh, nkv, n_ctx, qs):
    """Caches past what the output split's LDS holds (round 6): the head's KQ split over cells in
    two launches (kq_attn_cells scores 64-cell chunks of a kv group for all its heads into a
    workspace and stores the new cell; kq_attn_cells_kqv runs soft_max and KQV per output
    slice). Every cell random, positions across the whole cache: bit-exact with the oracle,
    both caches too, and the launch names show the two kernels ran. q scaled by 2 (group sums
    on both sides of the exact-tree bound) and by 40 (very peaked: soft_max's in-order sum,
    seq_sum_wave, with many binade changes and exact zeros)."""
    import torch
    import ggml_mi355x as g
    prev = g.attn_impl(2)  # split (the default)
    try:
        rng = np.random.default_rng(n_ctx + 3 * hd)
        kvw = nkv * hd
        tab = g.rope_table(n_ctx, hd, 10000.0, 1.0, device=dev)
        tref = O.rope_table(n_ctx, hd, 10000.0)
        kc_ref = rng.standard_normal((n_ctx, kvw)).astype(np.float16).view(np.uint16)
        vc_ref = rng.standard_normal((kvw, n_ctx)).astype(np.float16).view(np.uint16)
        kc = torch.from_numpy(kc_ref.view(np.int16).copy()).to(dev)
        vc = torch.from_numpy(vc_ref.view(np.int16).copy()).to(dev)
        scale = float(np.float32(1.0) / np.sqrt(np.float32(hd)))
        positions = [0, 1, 31, 32, 63, 64, 65, 1000, n_ctx // 2 + 7, n_ctx - 65, n_ctx - 64, n_ctx - 9, n_ctx - 1]
        for i, p in enumerate(positions):
            q = (rng.standard_normal(nh * hd) * qs).astype(np.float32)
            k = (rng.standard_normal(kvw) * 2).astype(np.float32)
            v = rng.standard_normal(kvw).astype(np.float32)
            pos = torch.tensor([p], dtype=torch.int32, device=dev)
            if i == 0:
                g.timing_enable(True)
            got = g.attn_decode(t(q, dev), t(k, dev), t(v, dev), pos, tab[p].contiguous(), kc, vc, nh, nkv, hd, scale,
                                rope_row=True).cpu().numpy()
            if i == 0:
                names = [r[0] for r in g.timing_read()]
                g.timing_enable(False)
                assert any("kq_attn_cells<" in n for n in names) and any("kq_attn_cells_kqv" in n for n in names), names
            ref = O.attn_decode(O.rope(q, hd, hd, p, tref), O.rope(k, hd, hd, p, tref), v, kc_ref, vc_ref, p, nh, nkv,
                                hd, scale)
            assert bits_equal(got, ref), (p, first_mismatch(got, ref))
        assert (kc.cpu().numpy().view(np.uint16) == kc_ref).all()
        assert (vc.cpu().numpy().view(np.uint16) == vc_ref).all()
        # a position outside the cache: NaN, caches untouched
        x = torch.ones(nh * hd, device=dev)
        out = g.attn_decode(x, x[:kvw], x[:kvw], torch.tensor([n_ctx], dtype=torch.int32, device=dev), tab, kc, vc,
                            nh, nkv, hd, scale)
        assert torch.isnan(out).all()
        assert (kc.cpu().numpy().view(np.uint16) == kc_ref).all()
        assert (vc.cpu().numpy().view(np.uint16) == vc_ref).all()
    finally:
        g.attn_impl(prev)


@pytest.mark.parametrize("hd", [64, 128])
def test_decode_graph_cells_equals_per_head(dev, hd):
    """The split over cells inside the decode graph (the backend reserves its workspace before
    capture; eager steps and graph replays interleaved) over every position of a 4096-cell
    cache: each token's logits equal those of the per-head kernel (MI355X_ATTN_HEAD, bit-exact
    with the oracle at every cache size), TinyLlama's and Llama-3-8B's head shapes, one layer."""
    import ggml_mi355x as g
    from tests import llama_model as LM
    from ggml_mi355x.llama import LlamaDecoder, hparams
    hp = hparams(32 * hd, 1, 32, 4 if hd == 64 else 8, 1024, 512)
    n_ctx = 4096
    assert g.attn_path(n_ctx, 32, hp["n_head_kv"], hd) == g.ATTN_PATH_CELLS
    wdev = LM.to_device(LM.build(hp, 21 + hd), dev)
    tokens = np.random.default_rng(hd).integers(0, hp["n_vocab"], size=n_ctx).tolist()
    keep = set(range(0, n_ctx, 61)) | set(range(n_ctx - 40, n_ctx))

    def run(impl):
        prev = g.attn_impl(impl)
        b = g.Backend()
        try:
            dec = LlamaDecoder(b, hp, wdev, n_ctx, fuse=True)
            out = {}
            for p, tok in enumerate(tokens):
                dec.step(tok, p, use_graph=(p % 11 != 5))
                if p in keep:
                    b.synchronize()
                    out[p] = dec.logits.cpu().numpy().copy()
            b.synchronize()
            g.timing_enable(True)  # the last token again, eager: which attention kernels ran
            dec.step(tokens[-1], n_ctx - 1, use_graph=False)
            b.synchronize()
            names = [r[0] for r in g.timing_read()]
            g.timing_enable(False)
            assert any("kq_attn_cells_kqv" in n for n in names) == (impl == g.ATTN_SPLIT), names
            return out
        finally:
            b.close()
            g.attn_impl(prev)

    cells = run(g.ATTN_SPLIT)
    head = run(g.ATTN_HEAD)
    for p in sorted(keep):
        assert bits_equal(cells[p], head[p]), (p, first_mismatch(cells[p], head[p]))


def test_attn_decode_cells_two_streams(dev, O):
    """The split over cells keeps its score workspace per (device, stream): two decoders'
    long-cache attentions enqueued on two streams at once, interleaved and unsynchronized,
    each bit-exact with the oracle (one shared workspace would mix their scores)."""
    import torch
    import ggml_mi355x as g
    prev = g.attn_impl(2)
    try:
        hd, nh, nkv, n_ctx = 64, 32, 4, 4096
        kvw = nkv * hd
        tab = g.rope_table(n_ctx, hd, 10000.0, 1.0, device=dev)
        tref = O.rope_table(n_ctx, hd, 10000.0)
        scale = float(np.float32(1.0) / np.sqrt(np.float32(hd)))
        streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
        state = []
        for si in range(2):
            rng = np.random.default_rng(77 + si)
            kc_ref = rng.standard_normal((n_ctx, kvw)).astype(np.float16).view(np.uint16)
            vc_ref = rng.standard_normal((kvw, n_ctx)).astype(np.float16).view(np.uint16)
            state.append(dict(rng=rng, kc_ref=kc_ref, vc_ref=vc_ref,
                              kc=torch.from_numpy(kc_ref.view(np.int16).copy()).to(dev),
                              vc=torch.from_numpy(vc_ref.view(np.int16).copy()).to(dev), outs=[]))
        torch.cuda.synchronize()
        positions = [4095, 2000, 3000, 17, 4094, 1500]
        for p in positions:
            for si, st in enumerate(state):
                q = (st["rng"].standard_normal(nh * hd) * 2).astype(np.float32)
                k = (st["rng"].standard_normal(kvw) * 2).astype(np.float32)
                v = st["rng"].standard_normal(kvw).astype(np.float32)
                with torch.cuda.stream(streams[si]):
                    pos = torch.tensor([p], dtype=torch.int32, device=dev)
                    got = g.attn_decode(t(q, dev), t(k, dev), t(v, dev), pos, tab[p].contiguous(), st["kc"], st["vc"], nh,
                                        nkv, hd, scale, rope_row=True, stream=streams[si].cuda_stream)
                st["outs"].append((p, q, k, v, got))
        torch.cuda.synchronize()
        for st in state:
            for p, q, k, v, got in st["outs"]:
                ref = O.attn_decode(O.rope(q, hd, hd, p, tref), O.rope(k, hd, hd, p, tref), v, st["kc_ref"], st["vc_ref"],
                                    p, nh, nkv, hd, scale)
                gn = got.cpu().numpy()
                assert bits_equal(gn, ref), (p, first_mismatch(gn, ref))
            assert (st["kc"].cpu().numpy().view(np.uint16) == st["kc_ref"]).all()
            assert (st["vc"].cpu().numpy().view(np.uint16) == st["vc_ref"]).all()
    finally:
        g.attn_impl(prev)


@pytest.mark.parametrize("qscale", [0.05, 2.0, 40.0], ids=["flat", "normal", "peaked"])
def test_attn_softmax_sum_tree_and_fallback(dev, O, attn_impl, qscale):
    """soft_max's double sum runs as a wave tree where every partial sum is exact (then it
    equals ggml's in-order sum bit for bit) and in order otherwise: flat scores (every
    group sum ~4, the tree), N(0, 2) scores, and very peaked ones (group sums far below
    2^-22: the in-order path). Positions up to 511 (n_kv 512, the > 256-cell path too)."""
    import torch
    import ggml_mi355x as g
    hd, nh, nkv, n_ctx = 64, 8, 2, 512
    rng = np.random.default_rng(int(qscale * 100))
    kvw = nkv * hd
    tab = g.rope_table(n_ctx, hd, 10000.0, 1.0, device=dev)
    tref = O.rope_table(n_ctx, hd, 10000.0)
    kc = torch.zeros((n_ctx, kvw), dtype=torch.int16, device=dev)
    vc = torch.zeros((kvw, n_ctx), dtype=torch.int16, device=dev)
    kc_ref = np.zeros((n_ctx, kvw), np.uint16)
    vc_ref = np.zeros((kvw, n_ctx), np.uint16)
    scale = float(np.float32(1.0) / np.sqrt(np.float32(hd)))
    for p in list(range(0, 300)) + [383, 384, 511]:
        q = (rng.standard_normal(nh * hd) * qscale).astype(np.float32)
        k = rng.standard_normal(kvw).astype(np.float32)
        v = rng.standard_normal(kvw).astype(np.float32)
        pos = torch.tensor([p], dtype=torch.int32, device=dev)
        got = g.attn_decode(t(q, dev), t(k, dev), t(v, dev), pos, tab, kc, vc, nh, nkv, hd, scale).cpu().numpy()
        ref = O.attn_decode(O.rope(q, hd, hd, p, tref), O.rope(k, hd, hd, p, tref), v, kc_ref, vc_ref, p, nh, nkv,
                            hd, scale)
        assert bits_equal(got, ref), (p, first_mismatch(got, ref))


def test_attn_decode_rejects_bad_position(dev, attn_impl):
    """A position outside the cache never computes silently: NaN output, caches untouched."""
    import torch
    import ggml_mi355x as g
    hd, nh, nkv, n_ctx = 64, 4, 2, 64
    tab = g.rope_table(n_ctx, hd, device=dev)
    kc = torch.zeros((n_ctx, nkv * hd), dtype=torch.int16, device=dev)
    vc = torch.zeros((nkv * hd, n_ctx), dtype=torch.int16, device=dev)
    x = torch.ones(nh * hd, device=dev)
    out = g.attn_decode(x, x[: nkv * hd], x[: nkv * hd], torch.tensor([n_ctx], dtype=torch.int32, device=dev), tab,
                        kc, vc, nh, nkv, hd, 0.125)
    assert torch.isnan(out).all()
    assert int(kc.abs().sum()) == 0 and int(vc.abs().sum()) == 0


# ---------------------------------------------------------------- fused GEMV prologue / epilogue
@pytest.mark.parametrize("pro", ["norm", "swiglu"])
def test_gemv_fused_ext(dev, O, oracle, npo, impl, pro):
    """RMS_NORM -> MUL -> MUL_MAT(s) -> ADD and SWIGLU -> MUL_MAT -> ADD in one launch
    (kq_rows) or staged (kq_gemv): equal to the separate ops, bit for bit."""
    import torch
    import ggml_mi355x as g
    rng = np.random.default_rng(11)
    K = 2048 if pro == "norm" else 5632
    mats = [(12, 384), (14, 128)] if pro == "norm" else [(14, 2048)]
    x = (rng.standard_normal(K) * 3).astype(np.float32)
    x2 = rng.uniform(0.5, 1.5, K).astype(np.float32) if pro == "norm" else rng.standard_normal(K).astype(np.float32)
    ws = [npo.random_blocks(rng, ty, n, K) for ty, n in mats]
    res = [rng.standard_normal(n).astype(np.float32) for _, n in mats]
    ys = [torch.empty(n, device=dev) for _, n in mats]
    g.gemv_fused_ext([(ty, t(w, dev), y) for (ty, _), w, y in zip(mats, ws, ys)], t(x, dev),
                     prologue=g.PRO_RMS_NORM if pro == "norm" else g.PRO_SWIGLU, x2=t(x2, dev), eps=1e-5,
                     residual=[t(r, dev) for r in res])
    torch.cuda.synchronize()
    xin = O.mul(O.rms_norm(x, 1e-5), x2) if pro == "norm" else O.swiglu(x, x2)
    for (ty, _), w, r, y in zip(mats, ws, res, ys):
        ref = O.add(oracle.mul_mat(ty, w, xin)[0], r)
        got = y.cpu().numpy()
        assert bits_equal(got, ref), first_mismatch(got, ref)


@pytest.mark.parametrize("n", [5632, 1000, 24])
def test_gemv_swiglu_epilogue(dev, O, oracle, npo, impl, n):
    """RMS_NORM -> MUL -> MUL_MAT(gate), MUL_MAT(up) -> SWIGLU in one launch: the gate
    and up outputs and the SWIGLU output bit-exact with the separate ops (paired waves
    in kq_rows at the real shape; the staged fallback where the waves cannot pair)."""
    import torch
    import ggml_mi355x as g
    rng = np.random.default_rng(n)
    K = 2048
    x = (rng.standard_normal(K) * 3).astype(np.float32)
    nw = rng.uniform(0.5, 1.5, K).astype(np.float32)
    ws = [npo.random_blocks(rng, 12, n, K) for _ in range(2)]
    ys = [torch.empty(n, device=dev) for _ in range(2)]
    h = torch.empty(n, device=dev)
    g.gemv_fused_ext([(12, t(w, dev), y) for w, y in zip(ws, ys)], t(x, dev), prologue=g.PRO_RMS_NORM,
                     x2=t(nw, dev), eps=1e-5, epi_y=h)
    torch.cuda.synchronize()
    xin = O.mul(O.rms_norm(x, 1e-5), nw)
    refs = [oracle.mul_mat(12, w, xin)[0] for w in ws]
    for y, ref in zip(ys, refs):
        assert bits_equal(y.cpu().numpy(), ref)
    got, ref = h.cpu().numpy(), O.swiglu(refs[0], refs[1])
    assert bits_equal(got, ref), first_mismatch(got, ref)


# ---------------------------------------------------------------- the whole token
def _decoder(dev, hp, seed, n_ctx, fuse=True, mix="q4_k_m"):
    from tests import llama_model as LM
    import ggml_mi355x as g
    from ggml_mi355x.llama import LlamaDecoder
    w = LM.build(hp, seed, mix=mix)
    b = g.Backend()
    dec = LlamaDecoder(b, hp, LM.to_device(w, dev), n_ctx, fuse=fuse)
    return w, b, dec


@pytest.mark.parametrize("fuse", [True, False], ids=["fused", "unfused"])
@pytest.mark.parametrize("mix", ["q4_k_m", "q5_k_m"])
def test_llama_decode_tokens(dev, O, fuse, mix):
    """Two TinyLlama-width layers (Q4_K_M mix, and the Q5_K_M mix of BASELINE config 5:
    Q5_K matrices and token_embd beside Q6_K attn_v / ffn_down / output) + a 4096-token
    vocabulary: the logits and every layer's residual stream of 5 consecutive tokens
    (hipGraph replay across tokens) bit-exact with the oracle's llm_build_llama restatement."""
    import torch
    from tests import llama_model as LM
    from ggml_mi355x.llama import hparams
    hp = hparams(2048, 2, 32, 4, 5632, 4096)
    n_ctx = 64
    w, b, dec = _decoder(dev, hp, 3, n_ctx, fuse, mix=mix)
    model, cache = LM.oracle_model(hp, w, n_ctx)
    tokens = [1, 4095, 17, 17, 300]
    for p, tok in enumerate(tokens):
        dec.step(tok, p)
        b.synchronize()
        got = dec.logits.cpu().numpy()
        ref, trace = O.decode_token(model, tok, p, cache)
        hid = dec.last_hidden.cpu().numpy()
        assert bits_equal(hid, trace[-1]), (p, "hidden", first_mismatch(hid, trace[-1]))
        assert bits_equal(got, ref), (p, first_mismatch(got, ref))
    torch.cuda.synchronize()
    b.close()


def test_llama_fused_launch_count(dev):
    """Fusion leaves 5 launches per layer (q/k/v, attention, o-proj + residual, gate/up,
    down) + get_rows + the output GEMV; with the opt-in attention/o-proj fusion 4 per layer."""
    import ggml_mi355x as g
    from ggml_mi355x.llama import hparams
    hp = hparams(2048, 3, 32, 4, 5632, 1024)
    _, b, dec = _decoder(dev, hp, 4, 64, True)
    dec.step(5, 0, use_graph=False)
    b.synchronize()
    g.timing_enable(True)
    dec.step(6, 1, use_graph=False)
    rows = g.timing_read()
    g.timing_enable(False)
    assert len(rows) == 5 * hp["n_layer"] + 2, [r[0] for r in rows]
    assert b.set_attn_oproj(True) == 0
    g.timing_enable(True)
    dec.step(7, 2, use_graph=False)
    rows = g.timing_read()
    g.timing_enable(False)
    assert len(rows) == 4 * hp["n_layer"] + 2, [r[0] for r in rows]
    b.close()


# ---------------------------------------------------------------- review fixes (r2)
@pytest.mark.parametrize("n", [2048, 4096, 8192])
def test_rms_norm_order_split_rows(dev, O, oracle, npo, n):
    """Rows whose float mean differs between ggml's sequential double sum and the GPU's
    fast tree order (tests/adversarial.py): kq_rms_norm and the kq_rows norm prologue
    both detect the ambiguity and re-sum in ggml's order, so the bits are the oracle's."""
    import torch
    import ggml_mi355x as g
    from tests.adversarial import order_split_rows
    rows, ms, mt = order_split_rows(n, count=4, seed=n)
    assert (ms != mt).all()
    w = np.random.default_rng(n).uniform(0.5, 1.5, n).astype(np.float32)
    got = g.rms_norm(t(rows, dev), 1e-5).cpu().numpy()
    ref = O.rms_norm(rows, 1e-5)
    assert bits_equal(got, ref), first_mismatch(got, ref)
    got = g.rms_norm(t(rows, dev), 1e-5, w=t(w, dev)).cpu().numpy()
    ref = np.stack([O.mul(O.rms_norm(r, 1e-5), w) for r in rows])
    assert bits_equal(got, ref), first_mismatch(got, ref)
    # the fused prologue: the normalized row goes straight into the Q8_K quantizer
    rng = np.random.default_rng(n + 1)
    wq = npo.random_blocks(rng, 12, 512, n)
    for r in rows:
        y = torch.empty(512, device=dev)
        g.gemv_fused_ext([(12, t(wq, dev), y)], t(r, dev), prologue=g.PRO_RMS_NORM, x2=t(w, dev), eps=1e-5)
        torch.cuda.synchronize()
        refy = oracle.mul_mat(12, wq, O.mul(O.rms_norm(r, 1e-5), w))[0]
        assert bits_equal(y.cpu().numpy(), refy), first_mismatch(y.cpu().numpy(), refy)


def test_get_rows_out_of_range_id(dev, npo):
    """An id outside [0, n_rows) reads nothing and yields a NaN row (ggml asserts)."""
    import ggml_mi355x as g
    rng = np.random.default_rng(1)
    K, R = 512, 10
    table = npo.random_blocks(rng, 12, R, K)
    ids = np.array([0, R, -1, 3, 1 << 30], np.int32)
    got = g.get_rows(12, t(table, dev), K, t(ids, dev)).cpu().numpy()
    assert np.isfinite(got[[0, 3]]).all()
    assert np.isnan(got[[1, 2, 4]]).all()


def _gemv_graph(be, K, N, rng, npo):
    """Helper: device buffers for a 1-column MUL_MAT graph."""
    import ggml_mi355x as g
    w = npo.random_blocks(rng, 12, N, K)
    p = be.alloc(w.nbytes)
    be.set_tensor(p, w)
    return w, g.make_tensor(12, K, N, p)


@pytest.mark.parametrize("view_offset", [0, 64])
def test_fusion_respects_reused_buffers_and_views(dev, O, oracle, npo, view_offset):
    """ggml-alloc reuses a dead node's buffer: node 2's MUL_MAT output lands in the buffer
    node 0 wrote, and node 4 reads it through a separate view (at offset 0 or 64 floats).
    The MUL_MAT -> ADD epilogue fusion may not elide the MUL_MAT output then
    (readers are credited to the LATEST overlapping writer)."""
    import ggml_mi355x as g
    K, N = 1024, 512
    rng = np.random.default_rng(view_offset)
    be = g.Backend()
    w, wt = _gemv_graph(be, K, N, rng, npo)
    x = rng.standard_normal(K).astype(np.float32)
    w0 = rng.uniform(0.5, 1.5, K).astype(np.float32)
    res = rng.standard_normal(N).astype(np.float32)
    res2 = rng.standard_normal(N).astype(np.float32)
    keep = []

    def buf(a=None, n=None):
        n = a.size if a is not None else n
        p = be.alloc(n * 4)
        if a is not None:
            be.set_tensor(p, a)
        return p

    P = buf(n=max(K, N))  # shared by node 0 (dead after node 1) and node 2
    xt = g.make_tensor(g.TYPE_F32, K, 1, buf(x))
    w0t = g.make_tensor(g.TYPE_F32, K, 1, buf(w0))
    n0 = g.make_tensor(g.TYPE_F32, K, 1, P, op=g.OP_MUL, src0=xt, src1=w0t)
    n1 = g.make_tensor(g.TYPE_F32, K, 1, buf(n=K), op=g.OP_ADD, src0=n0, src1=xt)
    n2 = g.make_tensor(g.TYPE_F32, N, 1, P, op=g.OP_MUL_MAT, src0=wt, src1=n1)
    rt = g.make_tensor(g.TYPE_F32, N, 1, buf(res))
    n3 = g.make_tensor(g.TYPE_F32, N, 1, buf(n=N), op=g.OP_ADD, src0=n2, src1=rt)
    nv = N - view_offset
    view = g.make_tensor(g.TYPE_F32, nv, 1, P + 4 * view_offset)  # a view of n2's output (op NONE)
    r2t = g.make_tensor(g.TYPE_F32, nv, 1, buf(res2[view_offset:].copy()))
    n4 = g.make_tensor(g.TYPE_F32, nv, 1, buf(n=nv), op=g.OP_ADD, src0=view, src1=r2t)
    keep += [xt, w0t, view, rt, r2t, wt]
    nodes = [n0, n1, n2, n3, n4]
    for use_graph in (0, 1):
        assert be.graph_compute(nodes, use_graph=use_graph) == 0
        be.synchronize()
        mm = oracle.mul_mat(12, w, O.add(O.mul(x, w0), x))[0]
        h3 = np.zeros(N, np.float32)
        h4 = np.zeros(nv, np.float32)
        be.get_tensor(h3, n3.data)
        be.get_tensor(h4, n4.data)
        be.synchronize()
        assert bits_equal(h3, O.add(mm, res))
        assert bits_equal(h4, O.add(mm[view_offset:], res2[view_offset:])), first_mismatch(
            h4, O.add(mm[view_offset:], res2[view_offset:]))
    be.close()


# ---------------------------------------------------------------- prompt processing (batched)
@pytest.fixture(params=[0, 1], ids=["pgroup", "phead"])
def prompt_impl(request):
    """Runs a prompt test on both prompt-attention kernels (per kv group and token, the
    default; per query head and token)."""
    import ggml_mi355x as g
    prev = g.attn_prompt_impl(request.param)
    yield request.param
    g.attn_prompt_impl(prev)


@pytest.fixture(params=[0, 2, 3, 5], ids=["mmq_auto", "mmq_tile128", "mmq_tile128w", "mmq_tile128x"])
def prompt_mmq(request):
    """The prompt's GEMMs on the default choice and on the 128-row tiles (the streamed
    Q4_K kernel was removed in round 3)."""
    import ggml_mi355x as g
    prev = g.mmq_impl(request.param)
    yield request.param
    g.mmq_impl(prev)


def test_llama_prompt_q5km(dev, O):
    """BASELINE config 5's mix (Q5_K matrices, Q6_K attn_v / ffn_down / output) through the
    prompt graph: the int8-MFMA GEMMs on Q5_K (balanced-byte operands) and Q6_K give the
    oracle's logits for the last token of a 37-token prompt and the KV caches of decoding
    the tokens one by one, bit for bit."""
    from tests import llama_model as LM
    from ggml_mi355x.llama import hparams
    hp = hparams(2048, 2, 32, 4, 5632, 4096)
    n_ctx = 64
    w, b, dec = _decoder(dev, hp, 6, n_ctx, True, mix="q5_k_m")
    model, cache = LM.oracle_model(hp, w, n_ctx)
    tokens = np.random.default_rng(12).integers(0, hp["n_vocab"], size=37).tolist()
    lg = dec.prompt(tokens, 0)
    b.synchronize()
    got = lg.cpu().numpy().copy()
    kc = [c.clone() for c in dec.k_cache]
    vc = [c.clone() for c in dec.v_cache]
    for p, tok in enumerate(tokens):
        ref, _ = O.decode_token(model, tok, p, cache)
    assert bits_equal(got, ref), first_mismatch(got, ref)
    dec.reset()
    for p, tok in enumerate(tokens):
        dec.step(tok, p)
    b.synchronize()
    for i in range(hp["n_layer"]):
        assert (dec.k_cache[i].cpu().numpy() == kc[i].cpu().numpy()).all(), i
        assert (dec.v_cache[i].cpu().numpy() == vc[i].cpu().numpy()).all(), i
    b.close()


@pytest.mark.parametrize("hd", [64, 128])
def test_llama_prompt_equals_tokens(dev, O, hd, prompt_impl, prompt_mmq):
    """A prompt batch through one graph (MUL_MAT at ne11 = T on the int8-MFMA GEMMs,
    batched norms, the prompt attention: all cells, then every query causally) gives the
    logits of its last token and the KV caches of decoding the tokens one by one, bit for
    bit, and equal to the oracle's sequential llm_build_llama; a second batch continues
    from the cache (start_pos > 0); decode steps after it (the cached hipGraphs alternate)."""
    import torch
    from tests import llama_model as LM
    from ggml_mi355x.llama import hparams
    hp = hparams(2048, 2, 2048 // hd, 4 if hd == 64 else 8, 5632, 4096)
    n_ctx = 128
    w, b, dec = _decoder(dev, hp, 5, n_ctx, True)
    model, cache = LM.oracle_model(hp, w, n_ctx)
    rng = np.random.default_rng(11)
    tokens = rng.integers(0, hp["n_vocab"], size=53).tolist()
    first, second = tokens[:37], tokens[37:50]
    lg = dec.prompt(first, 0)
    b.synchronize()
    got1 = lg.cpu().numpy().copy()
    kc1 = [c.clone() for c in dec.k_cache]
    vc1 = [c.clone() for c in dec.v_cache]
    for p, tok in enumerate(first):
        ref, _ = O.decode_token(model, tok, p, cache)
    assert bits_equal(got1, ref), first_mismatch(got1, ref)
    lg = dec.prompt(second, len(first))
    b.synchronize()
    got2 = lg.cpu().numpy().copy()
    for p, tok in enumerate(second, start=len(first)):
        ref, _ = O.decode_token(model, tok, p, cache)
    assert bits_equal(got2, ref), first_mismatch(got2, ref)
    # decode continues from the prompt's cache; then the same tokens decoded one by one
    # from an empty cache reproduce the prompt's caches exactly
    for p, tok in enumerate(tokens[50:], start=50):
        dec.step(tok, p)
        b.synchronize()
        ref, _ = O.decode_token(model, tok, p, cache)
        assert bits_equal(dec.logits.cpu().numpy(), ref), p
    dec.reset()
    for p, tok in enumerate(first):
        dec.step(tok, p)
    b.synchronize()
    for i in range(hp["n_layer"]):
        assert torch.equal(dec.k_cache[i], kc1[i]) and torch.equal(dec.v_cache[i], vc1[i]), i
    torch.cuda.synchronize()
    b.close()


def test_attn_prompt_rejects_bad_position(dev, prompt_impl):
    """A position outside the cache: that token's row is NaN, no cell is written."""
    import torch
    import ggml_mi355x as g
    hd, nh, nkv, n_ctx, T = 64, 8, 2, 64, 5
    table = g.rope_table(n_ctx, hd, 10000.0, 1.0, device=dev)
    q = torch.randn(T, nh * hd, device=dev)
    k = torch.randn(T, nkv * hd, device=dev)
    v = torch.randn(T, nkv * hd, device=dev)
    kc = torch.zeros((n_ctx, nkv * hd), dtype=torch.int16, device=dev)
    vc = torch.zeros((nkv * hd, n_ctx), dtype=torch.int16, device=dev)
    pos = torch.tensor([0, 1, n_ctx + 3, 3, -1], dtype=torch.int32, device=dev)
    out = g.attn_prompt(q, k, v, pos, table, kc, vc, nh, nkv, hd, 0.125)
    torch.cuda.synchronize()
    o = out.cpu()
    assert torch.isnan(o[2]).all() and torch.isnan(o[4]).all()
    assert torch.isfinite(o[[0, 1, 3]]).all()
    assert (kc[2] == 0).all() and (kc[4:] == 0).all()
    assert (kc[[0, 1, 3]] != 0).any(dim=1).all()
