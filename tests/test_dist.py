"""Multi-process (gloo, CPU) tests of the row-split decode token: the TokenSplit plan
(ggml_mi355x/rowsplit.py) executed rank by rank with the oracle's ops and a gloo
all_gather standing in for the backend's ALL_GATHER node (RCCL on GPUs), bit-identical
to the single-process oracle token at world 2, 4 and 8."""
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
