"""Multi-process (world_size 2, gloo, CPU) tests of the row-split path: shard layout,
the packed per-stage gather / all-reduce, and that the reassembled outputs are
bit-identical to the single-process result. The per-rank compute here is the
oracle (CPU); on GPUs the same StageGather runs over RCCL with the HIP GEMV."""
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


def test_shard_rows_cover_and_align():
    from ggml_mi355x.rowsplit import shard_rows
    for n in (0, 1, 7, 8, 255, 256, 2048, 5632, 32000, 128256):
        for world in (1, 2, 3, 4, 8):
            got = [shard_rows(n, world, r) for r in range(world)]
            covered = []
            for r0, r1, per in got:
                assert per % 8 == 0 and r1 - r0 <= per
                assert r0 % 8 == 0 or r0 == r1
                covered.extend(range(r0, r1))
            assert covered == list(range(n))


def _worker(rank, world, port, collective, results):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ggml_mi355x.rowsplit import StageGather
        from oracle import kq_oracle as O
        from oracle import kq_oracle_np as N
        rng = np.random.default_rng(123)
        K = 2048
        specs = [(12, 2048), (12, 256), (14, 256)]  # q, k, v(Q6_K) of a TinyLlama layer
        ws = [N.random_blocks(rng, t, n, K) for t, n in specs]
        x = rng.standard_normal((1, K)).astype(np.float32)
        sg = StageGather([n for _, n in specs], world, rank, torch.device("cpu"), collective=collective)
        for i, ((t, n), w) in enumerate(zip(specs, ws)):
            r0, r1, _ = sg.shards[i]
            part = O.mul_mat(t, w[r0:r1], x)[0] if r1 > r0 else np.zeros(0, np.float32)
            sg.local_view(i).copy_(torch.from_numpy(part))
        sg.exchange()
        ok = True
        for i, ((t, n), w) in enumerate(zip(specs, ws)):
            full = O.mul_mat(t, w, x)[0]
            got = sg.output(i).numpy()
            ok &= bool((got.view(np.uint32) == full.view(np.uint32)).all())
        results[rank] = ok
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("collective", ["all_gather", "all_reduce"])
def test_rowsplit_gloo_world2_bit_exact(collective):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    results = mgr.dict()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, collective, results)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert dict(results) == {0: True, 1: True}
