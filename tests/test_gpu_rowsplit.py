"""GPU tests of the row-split decode token (SURVEY.md §8e, rows e / f4): the
ALL_GATHER node over a real RCCL communicator (world 1 on this one-GPU box), and
every rank of worlds 2 / 4 / 8 emulated on one GPU (mi355x_backend_set_comm_loopback:
the rank's ALL_GATHER writes only its own slice; the other ranks' slices are
pre-filled with the oracle's values) — each rank's q/k/v head rows, local attention
on its KV-cache slice, and row slices of o / gate / up / down / output reproduce the
oracle's gathered vectors bit for bit. The multi-rank exchange itself is covered by
tests/test_dist.py (gloo) and runs over RCCL in bench.py --gpus N."""
import numpy as np
import pytest

from tests.test_gpu_parity import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

TOKENS = (1, 4095, 17, 300)


@pytest.fixture(scope="module")
def O():
    from oracle import kq_ops_oracle
    kq_ops_oracle.lib()
    return kq_ops_oracle


def _hp():
    from ggml_mi355x.llama import hparams
    return hparams(2048, 2, 32, 4, 5632, 4096)  # TinyLlama width, 2 layers, 4096-token vocab


def _reference(O, hp, w, n_ctx):
    from tests import llama_model as LM
    model, cache = LM.oracle_model(hp, w, n_ctx)
    out = []
    for p, tok in enumerate(TOKENS):
        tr = []
        logits, _ = O.decode_token(model, tok, p, cache, full_trace=tr)
        out.append((logits, tr))
    return out


@pytest.mark.parametrize("use_graph", [True, False], ids=["graph", "eager"])
def test_rowsplit_token_world1_rccl(dev, O, use_graph):
    """A world-1 row split through a real RCCL communicator: the ALL_GATHER nodes
    (ncclAllGather on the backend stream, captured in the hipGraph) around every stage;
    logits and gathered vectors bit-exact with the oracle token."""
    import torch
    import ggml_mi355x as g
    from ggml_mi355x.llama import LlamaDecoder
    from ggml_mi355x.rowsplit import TokenSplit
    from tests import llama_model as LM
    hp, n_ctx = _hp(), 64
    w = LM.build(hp, 11)
    ref = _reference(O, hp, w, n_ctx)
    b = g.Backend()
    b.set_comm(0, 1, g.comm_unique_id())
    assert b.comm_world == 1
    split = TokenSplit(hp, 1, 0)
    dec = LlamaDecoder(b, hp, LM.to_device(split.slice_weights(w), dev), n_ctx, split=split)
    assert len(dec.gathers) == 4 * hp["n_layer"] + 1
    for p, tok in enumerate(TOKENS):
        dec.step(tok, p, use_graph=use_graph)
        b.synchronize()
        logits, tr = ref[p]
        got = dec.logits.cpu().numpy()
        assert bits_equal(got, logits), (p, first_mismatch(got, logits))
        for li in range(hp["n_layer"]):
            for j, k in enumerate(("att", "ffn_inp", "glu", "x")):
                gv = dec.gathers[4 * li + j].cpu().numpy()
                assert bits_equal(gv, tr[li][k]), (p, li, k)
    torch.cuda.synchronize()
    b.close()


@pytest.mark.parametrize("world,rank", [(2, 0), (2, 1), (4, 1), (4, 3), (8, 0), (8, 5), (8, 7)])
def test_rowsplit_token_rank_emulated(dev, O, world, rank):
    """Rank `rank` of a `world`-GPU row split on this GPU: its local GEMVs, attention
    (world 8 > n_head_kv 4: two ranks per KV head) and epilogues, bit-exact with the
    oracle's gathered vectors at 4 dependent positions (hipGraph replay)."""
    import torch
    import ggml_mi355x as g
    from ggml_mi355x.llama import LlamaDecoder
    from ggml_mi355x.rowsplit import TokenSplit
    from tests import llama_model as LM
    hp, n_ctx = _hp(), 64
    w = LM.build(hp, 12)
    ref = _reference(O, hp, w, n_ctx)
    b = g.Backend()
    b.set_comm_loopback(rank, world)
    split = TokenSplit(hp, world, rank)
    dec = LlamaDecoder(b, hp, LM.to_device(split.slice_weights(w), dev), n_ctx, split=split)
    keys = ("att", "ffn_inp", "glu", "x")
    for p, tok in enumerate(TOKENS):
        logits, tr = ref[p]
        full = [tr[li][k] for li in range(hp["n_layer"]) for k in keys] + [logits]
        for buf, v in zip(dec.gathers, full):  # the other ranks' slices, as RCCL would deliver them
            buf.copy_(torch.from_numpy(np.ascontiguousarray(v, np.float32)))
        torch.cuda.synchronize()
        dec.step(tok, p)
        b.synchronize()
        for i, (buf, v) in enumerate(zip(dec.gathers, full)):
            got = buf.cpu().numpy()
            assert bits_equal(got, v), (p, i, first_mismatch(got, v))
    torch.cuda.synchronize()
    b.close()
