"""Multi-process (gloo, CPU) tests of the row-split decode token: the TokenSplit plan
(ggml_mi355x/rowsplit.py) executed rank by rank with the oracle's ops and gloo
collectives standing in for the backend's ALL_GATHER / ALL_REDUCE nodes (RCCL on GPUs):
gather mode bit-identical to the single-process oracle token at world 2, 4 and 8;
reduce mode (K-split + all-reduce) bit-identical to its one-process restatement with a
rank-ordered sum and within the fp32 re-association bound of the unsplit token."""
import os
import socket

import numpy as np
import pytest


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ------------------------------------------------ the dependent row-split decode token
SPLIT_HP = dict(n_embd=512, n_layer=2, n_head=8, n_head_kv=2, head_dim=64, n_ff=768, n_vocab=1024, eps=1e-5,
                freq_base=10000.0)
SPLIT_CTX, SPLIT_TOKENS = 32, (5, 77, 1000)


def _split_token_worker(rank, world, port, results):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ggml_mi355x.rowsplit import TokenSplit
        from tests import llama_model as LM
        from tests.split_token import local_cache, local_model, split_decode_token
        hp = SPLIT_HP
        w = LM.build(hp, seed=4)
        model, _ = LM.oracle_model(hp, w, SPLIT_CTX)
        split = TokenSplit(hp, world, rank)
        lm = local_model(model, split)
        cache = local_cache(hp, split, SPLIT_CTX)

        def gather(local):  # the ALL_GATHER node: rank-ordered concatenation
            t = torch.from_numpy(np.ascontiguousarray(local, np.float32))
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            return torch.cat(parts).numpy()

        out = []
        for pos, tok in enumerate(SPLIT_TOKENS):
            tr = []
            logits = split_decode_token(lm, split, tok, pos, cache, gather, full_trace=tr)
            out.append((logits.view(np.uint32).copy(), [{k: v.view(np.uint32).copy() for k, v in d.items()} for d in tr]))
        results[rank] = out
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rowsplit_decode_token_gloo_bit_exact(world):
    """Every rank of a row-split decode token (TokenSplit: q/k/v rows by head, attention
    on the rank's KV heads, row slices of o / gate / up / down / output, ALL_GATHER after
    each stage), run over gloo with the oracle's ops, reproduces the single-process
    oracle token bit for bit: the logits and every gathered vector, at 3 dependent
    positions of one KV cache. world 8 > n_head_kv 2: 4 ranks share each KV head."""
    import torch.multiprocessing as mp
    from oracle import kq_ops_oracle as OO
    from tests import llama_model as LM
    hp = SPLIT_HP
    w = LM.build(hp, seed=4)
    model, cache = LM.oracle_model(hp, w, SPLIT_CTX)
    ref = []
    for pos, tok in enumerate(SPLIT_TOKENS):
        tr = []
        logits, _ = OO.decode_token(model, tok, pos, cache, n_threads=2, full_trace=tr)
        ref.append((logits.view(np.uint32), tr))
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    results = mgr.dict()
    port = free_port()
    procs = [ctx.Process(target=_split_token_worker, args=(r, world, port, results)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert sorted(results.keys()) == list(range(world))
    for r in range(world):
        for (lg, tr), (rlg, rtr) in zip(results[r], ref):
            assert (lg == rlg).all()
            for d, rd in zip(tr, rtr):
                for k in ("att", "ffn_inp", "glu", "x"):
                    assert (d[k] == rd[k].view(np.uint32)).all(), (r, k)


def test_token_split_plan():
    """TokenSplit row ranges: disjoint and covering for the row-split matrices, the KV
    heads of the rank's query heads, and rejection of splits the plan cannot express."""
    from ggml_mi355x.rowsplit import TokenSplit
    for hp in (SPLIT_HP, dict(SPLIT_HP, n_embd=2048, n_head=32, n_head_kv=4, n_ff=5632, n_vocab=32000),
               dict(SPLIT_HP, n_embd=8192, n_head=64, n_head_kv=8, n_ff=28672, n_vocab=128256, head_dim=128)):
        group = hp["n_head"] // hp["n_head_kv"]
        for world in (1, 2, 4, 8):
            sp = [TokenSplit(hp, world, r) for r in range(world)]
            for name, n in (("attn_q", hp["n_head"] * hp["head_dim"]), ("attn_output", hp["n_embd"]),
                            ("ffn_gate", hp["n_ff"]), ("ffn_down", hp["n_embd"]), ("output", hp["n_vocab"])):
                cov = [i for s in sp for i in range(*s.rows[name])]
                assert cov == list(range(n)), (name, world)
            for s in sp:
                assert s.n_head == hp["n_head"] // world
                assert s.kv0 == s.q0 // group and s.kv1 == (s.q1 - 1) // group + 1
                assert s.rows["attn_k"] == (s.kv0 * hp["head_dim"], s.kv1 * hp["head_dim"])
    with pytest.raises(ValueError):
        TokenSplit(dict(SPLIT_HP, n_head=6), 4, 0)
    with pytest.raises(ValueError):
        TokenSplit(dict(SPLIT_HP, n_head_kv=3, n_head=24), 2, 0)


# ------------------------------------------------ reduce mode: K-split + all-reduce
# n_embd 1024 / 16 heads of 64: 4 heads = one superblock of attn_output's K at world 4;
# n_ff 1536 = 6 superblocks: an uneven ffn_down K split at world 4 (1, 2, 1, 2)
KSPLIT_HP = dict(n_embd=1024, n_layer=2, n_head=16, n_head_kv=4, head_dim=64, n_ff=1536, n_vocab=1024, eps=1e-5,
                 freq_base=10000.0)


def _ksplit_worker(rank, world, port, results, native):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ggml_mi355x.rowsplit import TokenSplit
        from tests import llama_model as LM
        from tests.split_token import ksplit_decode_token, local_cache, local_model, rank_ordered_sum
        hp = KSPLIT_HP
        w = LM.build(hp, seed=6)
        model, _ = LM.oracle_model(hp, w, SPLIT_CTX)
        split = TokenSplit(hp, world, rank, mode="reduce")
        lm = local_model(model, split)
        cache = local_cache(hp, split, SPLIT_CTX)

        def gather_parts(local):
            t = torch.from_numpy(np.ascontiguousarray(local, np.float32))
            sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(sizes, torch.tensor([t.numel()]))
            parts = [torch.empty(int(s.item())) for s in sizes]
            if len({p.numel() for p in parts}) == 1:
                dist.all_gather(parts, t)
            else:  # (uneven slices: gloo's all_gather wants equal sizes)
                m = max(p.numel() for p in parts)
                pad = torch.zeros(m)
                pad[:t.numel()] = t
                full = [torch.empty(m) for _ in range(world)]
                dist.all_gather(full, pad)
                parts = [f[:p.numel()] for f, p in zip(full, parts)]
            return [p.numpy() for p in parts]

        def gather(local):
            return np.concatenate(gather_parts(local)).astype(np.float32)

        def allreduce(local):
            if native:  # gloo's own all_reduce(SUM): its summation order
                t = torch.from_numpy(np.ascontiguousarray(local, np.float32)).clone()
                dist.all_reduce(t)
                return t.numpy()
            return rank_ordered_sum(gather_parts(local))

        out = []
        for pos, tok in enumerate(SPLIT_TOKENS):
            logits = ksplit_decode_token(lm, split, tok, pos, cache, allreduce, gather)
            out.append(logits.copy())
        results[rank] = out
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("native", [False, True], ids=["ordered_sum", "gloo_allreduce"])
def test_ksplit_decode_token_gloo(world, native):
    """Reduce mode (the north_star's all-reduce: q/k/v and gate/up by output rows,
    attn_output and ffn_down split along K at superblock boundaries, one all-reduce(sum)
    of the partials after each, 2 per layer) over gloo with the oracle's ops: with a
    rank-ordered f32 sum every rank's logits equal the one-process restatement
    (split_token.ksplit_reference) bit for bit; with gloo's own all_reduce order and
    against the unsplit oracle token the logits agree within the fp32 re-association
    bound (the K-split changes only the summation order of each row's chain)."""
    import torch.multiprocessing as mp
    from oracle import kq_ops_oracle as OO
    from tests import llama_model as LM
    from tests.split_token import ksplit_reference
    hp = KSPLIT_HP
    w = LM.build(hp, seed=6)
    model, cache = LM.oracle_model(hp, w, SPLIT_CTX)
    seq = [OO.decode_token(model, tok, pos, cache, n_threads=2)[0] for pos, tok in enumerate(SPLIT_TOKENS)]
    model2, _ = LM.oracle_model(hp, w, SPLIT_CTX)
    kref = ksplit_reference(model2, hp, world, SPLIT_TOKENS, SPLIT_CTX)
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    results = mgr.dict()
    port = free_port()
    procs = [ctx.Process(target=_ksplit_worker, args=(r, world, port, results, native)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert sorted(results.keys()) == list(range(world))
    for r in range(world):
        for lg, (klg, _), slg in zip(results[r], kref, seq):
            if not native:
                assert (lg.view(np.uint32) == klg.view(np.uint32)).all(), r
            # fp32 re-association of 2 * n_layer K-split chains, through the norms,
            # attention and swiglu of 2 layers: relative to the logits' scale
            scale = float(np.max(np.abs(slg)))
            assert np.max(np.abs(lg - slg)) <= 2e-4 * scale, (r, np.max(np.abs(lg - slg)), scale)
            assert np.argmax(lg) == np.argmax(slg)


def test_ksplit_gemv_within_fp32_bound():
    """One K-split GEMV: each rank's partial is the reference's fp32 chain
    over its superblocks (the oracle vec_dot on the column slice, integer parts exact by
    construction); their rank-ordered sum differs from the full row's chain by at most
    1e-5 * sum_i(|d_i sumi_i| + |dmin_i summins_i|) (+1e-30), for Q4_K / Q5_K / Q6_K,
    uneven superblock splits, worlds 2 .. 8."""
    from oracle import kq_oracle as KO
    from oracle import kq_oracle_np as N
    from tests.split_token import rank_ordered_sum
    rng = np.random.default_rng(0x5EED)
    for typ in (N.Q4_K, N.Q5_K, N.Q6_K):
        for K, world in ((2048, 2), (5632, 4), (5632, 8), (8192, 8)):
            nb, B, Nr = K // 256, N.BLOCK_BYTES[typ], 24
            w = N.random_blocks(rng, typ, Nr, K)
            x = rng.standard_normal(K).astype(np.float32)
            full = KO.mul_mat(typ, w, x)[0]
            parts = []
            for r in range(world):
                c0, c1 = r * nb // world, (r + 1) * nb // world
                parts.append(KO.mul_mat(typ, np.ascontiguousarray(w[:, c0 * B:c1 * B]), x[c0 * 256:c1 * 256])[0])
            got = rank_ordered_sum(parts)
            q8 = N.quantize_q8_K(x[None])
            sumi, summins = N.block_partials(w, typ, K, q8)  # (Nr, 1, nb)
            f = N.split_blocks(w, typ, K)
            yd = q8["d"][0].astype(np.float64)
            d = N.fp16_to_f32(f["d"]).astype(np.float64) * yd
            terms = np.abs(d * sumi[:, 0]).sum(-1)
            if typ != N.Q6_K:
                terms += np.abs(N.fp16_to_f32(f["dmin"]).astype(np.float64) * yd * summins[:, 0]).sum(-1)
            bound = 1e-5 * terms + 1e-30
            err = np.abs(got.astype(np.float64) - full.astype(np.float64))
            assert (err <= bound).all(), (typ, K, world, float((err / bound).max()))


def test_token_split_plan_reduce():
    """Reduce-mode plan: attn_output / ffn_down keep every row and split their K into
    disjoint superblock ranges covering the row (the rank's heads / ffn rows), gate/up
    rows follow the ffn_down columns; splits the superblock grid cannot express raise."""
    from ggml_mi355x.rowsplit import TokenSplit
    for hp in (KSPLIT_HP, dict(KSPLIT_HP, n_embd=2048, n_head=32, n_head_kv=4, n_ff=5632, n_vocab=32000),
               dict(KSPLIT_HP, n_embd=8192, n_head=64, n_head_kv=8, n_ff=28672, n_vocab=128256, head_dim=128)):
        E, F, hd = hp["n_embd"], hp["n_ff"], hp["head_dim"]
        worlds = [wd for wd in (1, 2, 4, 8) if (hp["n_head"] // wd) * hd % 256 == 0]
        for world in worlds:
            sp = [TokenSplit(hp, world, r, mode="reduce") for r in range(world)]
            assert [c for s in sp for c in range(*s.cols["attn_output"])] == list(range(E // 256))
            assert [c for s in sp for c in range(*s.cols["ffn_down"])] == list(range(F // 256))
            for s in sp:
                assert s.rows["attn_output"] == (0, E) and s.rows["ffn_down"] == (0, E)
                f0, f1 = s.cols["ffn_down"]
                assert s.rows["ffn_gate"] == s.rows["ffn_up"] == (256 * f0, 256 * f1)
                q0, q1 = s.rows["attn_q"]
                assert s.cols["attn_output"] == (q0 // 256, q1 // 256)
                assert s.collectives_per_token() == 2 * hp["n_layer"] + 1
    assert 8 in [wd for wd in (1, 2, 4, 8) if (32 // wd) * 64 % 256 == 0]
    with pytest.raises(ValueError):
        TokenSplit(KSPLIT_HP, 8, 0, mode="reduce")  # 2 heads x 64 = half a superblock
    with pytest.raises(ValueError):
        TokenSplit(KSPLIT_HP, 2, 0, mode="bogus")


# ------------------------------------------------ bench.py's N > 1 control plane
def _bench_connect_worker(rank, world, port, fail_rank, results):
    import types
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench

        class FakeBackend:  # the GPU backend's communicator entry point, failing on one rank
            def __init__(self):
                self.calls = []

            def set_comm(self, r, n, uid):
                self.calls.append((r, n, len(uid)))
                if r == fail_rank:
                    raise RuntimeError("ncclCommInitRank failed (test)")

        bench.g = types.SimpleNamespace(lib=lambda: types.SimpleNamespace(mi355x_comm_id_size=lambda: 128),
                                        comm_unique_id=lambda: bytes(range(128)))
        be = FakeBackend()
        err = bench.connect(be, world, rank)
        # what main() does with the agreed error: every rank falls back to replicas
        mode = bench.resolve_mode("auto", world)
        rowsplit = mode != "replicas" and err is None
        head = bench.headline_fields(mode if rowsplit else "replicas", world)
        results[rank] = (err, be.calls, mode, head)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [None, 1])
def test_bench_connect_failure_falls_back_to_replicas(fail_rank):
    """bench.py at N = 2 (gloo control plane, as the driver's scaling run):
    the headline is the reduce row split; the RCCL id goes from rank 0 to every rank; when
    the communicator fails on ANY rank, every rank agrees on the failure (so none waits in a
    collective the others never enter) and the line falls back to replicas with the replicas
    fields (weak scaling, N tokens per step)."""
    import torch.multiprocessing as mp
    world = 2
    results = mp.Manager().dict()
    mp.spawn(_bench_connect_worker, args=(world, free_port(), fail_rank, results), nprocs=world, join=True)
    for r in range(world):
        err, calls, mode, head = results[r]
        assert mode == "rowsplit-reduce"
        assert calls == [(r, world, 128)]
        if fail_rank is None:
            assert err is None
            assert head == {"scaling": "strong", "parallelism": "rowsplit-reduce2", "tokens_per_step": 1}
        else:
            assert err is not None
            assert ("ncclCommInitRank" in err) if r == fail_rank else err == "communicator setup failed on another rank"
            assert head == {"scaling": "weak", "parallelism": "replicas x2", "tokens_per_step": 2}
