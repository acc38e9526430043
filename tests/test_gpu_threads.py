"""The threading contract and the trait-table surface (a10, b).

ggml-cpu runs one MUL_MAT node on nth threads at once: every thread quantizes its
slice of src1 with type_traits_cpu[Q8_K].from_float, then walks 64-row chunks calling
type_traits_cpu[Q4_K].vec_dot(n, &tmp[i], 0, src0_row, 0, wdata_col, 0, 1) with HOST
pointers (ggml_compute_forward_mul_mat / _one_chunk, README.md:121-137; signature
README.md:449). The exported mi355x_vec_dot_* / mi355x_quantize_row_q8_K take exactly
those calls — host or device pointers, any thread — on a per-thread stream. Here:
 * host-pointer calls, bit-exact with the oracle;
 * 8 host threads running a restated mul_mat chunk loop through the trait entries;
 * 8 threads each launching mi355x_mul_mat on their own stream, concurrently;
 * two backends in two threads decoding tokens concurrently.
"""
import ctypes
import threading

import numpy as np
import pytest

from tests.test_gpu_parity import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

VEC_DOT = {12: "mi355x_vec_dot_q4_K_q8_K", 13: "mi355x_vec_dot_q5_K_q8_K", 14: "mi355x_vec_dot_q6_K_q8_K"}


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


@pytest.mark.parametrize("type_", [12, 13, 14])
def test_vec_dot_host_pointers(dev, oracle, npo, type_):
    """One vec_dot per row with host src0 row, host Q8_K column and host output, and the
    device / host mixes: the same bits as the oracle's NEON-order vec_dot."""
    import torch
    import ggml_mi355x as g
    L = g.lib()
    rng = np.random.default_rng(40 + type_)
    K, N = 4096, 12
    w = npo.random_blocks(rng, type_, N, K)
    x = rng.standard_normal((1, K)).astype(np.float32)
    q8 = np.zeros(K // 256 * 292, np.uint8)
    L.mi355x_quantize_row_q8_K(_ptr(x[0]), _ptr(q8), K)  # from_float with host pointers
    assert (q8 == oracle.quantize_q8_K(x)[0]).all()
    fn = getattr(L, VEC_DOT[type_])
    ref = oracle.mul_mat(type_, w, x)[0]
    s = np.zeros(1, np.float32)
    for r in range(N):
        fn(K, _ptr(s), 0, _ptr(w[r]), 0, _ptr(q8), 0, 1)
        assert s.view(np.uint32)[0] == ref[r:r + 1].view(np.uint32)[0], r
    wd = torch.from_numpy(w).to(dev)
    qd = torch.from_numpy(q8).to(dev)
    sd = torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    fn(K, _ptr(s), 0, ctypes.c_void_p(wd[3].data_ptr()), 0, _ptr(q8), 0, 1)  # device row, host column
    assert s.view(np.uint32)[0] == ref[3:4].view(np.uint32)[0]
    fn(K, ctypes.c_void_p(sd.data_ptr()), 0, _ptr(w[5]), 0, ctypes.c_void_p(qd.data_ptr()), 0, 1)
    assert bits_equal(sd.cpu().numpy(), ref[5:6])


@pytest.mark.parametrize("type_", [12, 14])
def test_trait_table_mul_mat_from_threads(dev, oracle, npo, type_):
    """ggml-cpu's mul_mat restated over the exported trait entries: 8 host threads
    quantize their src1 slices (from_float) into a shared host wdata, meet at a
    barrier, then take 64-row chunks from a shared counter and call vec_dot per row
    with host pointers — every output bit-exact with the oracle's mul_mat."""
    import ggml_mi355x as g
    L = g.lib()
    rng = np.random.default_rng(50 + type_)
    K, N, nth = 2048, 300, 8
    w = npo.random_blocks(rng, type_, N, K)
    x = rng.standard_normal(K).astype(np.float32)
    nb = K // 256
    wdata = np.zeros(nb * 292, np.uint8)
    dst = np.zeros(N, np.float32)
    fn = getattr(L, VEC_DOT[type_])
    bar = threading.Barrier(nth)
    lock = threading.Lock()
    nxt = [0]
    errors = []

    def worker(ith):
        try:
            b0, b1 = ith * nb // nth, (ith + 1) * nb // nth
            if b1 > b0:  # the thread's block slice of the activation row
                L.mi355x_quantize_row_q8_K(_ptr(x[b0 * 256:]), ctypes.c_void_p(wdata.ctypes.data + b0 * 292),
                                           (b1 - b0) * 256)
            bar.wait()
            tmp = np.zeros(1, np.float32)
            while True:
                with lock:
                    c = nxt[0]
                    nxt[0] += 1
                if c * 64 >= N:
                    break
                for r in range(c * 64, min(N, c * 64 + 64)):
                    fn(K, _ptr(tmp), 0, _ptr(w[r]), 0, _ptr(wdata), 0, 1)
                    dst[r] = tmp[0]
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(nth)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errors, errors
    ref = oracle.mul_mat(type_, w, x[None])[0]
    assert bits_equal(dst, ref), first_mismatch(dst, ref)


def test_concurrent_streams_mul_mat(dev, oracle, npo):
    """8 host threads, each with its own HIP stream and its own weights, launching the
    GEMV and the prefill GEMM 20 times concurrently: every result bit-exact."""
    import torch
    import ggml_mi355x as g
    rng = np.random.default_rng(60)
    K, N, nth = 2048, 520, 8
    cases = []
    for i in range(nth):
        typ = (12, 14, 13)[i % 3]
        w = npo.random_blocks(rng, typ, N, K)
        x = rng.standard_normal((1 + 16 * (i % 2), K)).astype(np.float32)
        cases.append((typ, w, x, oracle.mul_mat(typ, w, x)))
    outs = [None] * nth
    errors = []

    def worker(i):
        try:
            typ, w, x, _ = cases[i]
            st = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(st):
                wd = torch.from_numpy(w).to(dev, non_blocking=False)
                xd = torch.from_numpy(x).to(dev)
                y = torch.empty((x.shape[0], N), device=dev)
                st.synchronize()
                for _ in range(20):
                    g.mul_mat(typ, wd, K, xd, out=y, stream=st.cuda_stream)
                st.synchronize()
                outs[i] = y.cpu().numpy()
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(nth)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errors, errors
    for i in range(nth):
        assert bits_equal(outs[i], cases[i][3]), (i, first_mismatch(outs[i], cases[i][3]))


def test_two_backends_decode_concurrently(dev, O):
    """Two backends (own streams, own hipGraphs) decoding different models from two host
    threads at once: each token's logits bit-exact with the oracle."""
    import torch
    import ggml_mi355x as g
    from ggml_mi355x.llama import LlamaDecoder, hparams
    from tests import llama_model as LM
    hp = hparams(512, 2, 8, 2, 768, 1024)
    n_ctx = 32
    toks = [3, 900, 17, 44]
    runs = []
    for seed in (21, 22):
        w = LM.build(hp, seed)
        model, cache = LM.oracle_model(hp, w, n_ctx)
        ref = [O.decode_token(model, t, p, cache, n_threads=2)[0] for p, t in enumerate(toks)]
        b = g.Backend()
        dec = LlamaDecoder(b, hp, LM.to_device(w, dev), n_ctx)
        runs.append((b, dec, ref))
    got = [[], []]
    errors = []

    def worker(i):
        try:
            b, dec, _ = runs[i]
            for p, t in enumerate(toks):
                dec.step(t, p)
                b.synchronize()
                got[i].append(dec.logits.cpu().numpy())
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errors, errors
    for i in range(2):
        for p in range(len(toks)):
            assert bits_equal(got[i][p], runs[i][2][p]), (i, p)
    torch.cuda.synchronize()
    for b, _, _ in runs:
        b.close()


@pytest.fixture(scope="module")
def O():
    from oracle import kq_ops_oracle
    kq_ops_oracle.lib()
    return kq_ops_oracle
