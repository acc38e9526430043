"""End to end through the drop-in adapter path: llm_build_llama's ggml decode graph
(tests/ggml_graph.py, ggml-alloc-style output buffers on the device) lowered by
mi355x_lower_ggml_graph and run by mi355x_backend_graph_compute (fusion + hipGraph),
token after token on one KV cache — the logits bit-exact with the oracle's token."""
import numpy as np
import pytest

from tests.test_gpu_parity import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu


def test_lowered_llama_graph_decodes_bit_exact(dev):
    import torch
    import ggml_mi355x as g
    from ggml_mi355x.llama import LlamaDecoder, hparams
    from oracle import kq_ops_oracle as O
    from tests import ggml_graph as GG
    from tests import llama_model as LM
    from tests.test_lower import _leaves
    hp = hparams(2048, 2, 32, 4, 5632, 4096)
    n_ctx = 64
    w = LM.build(hp, 31)
    b = g.Backend()
    wd = LM.to_device(w, dev)
    dec = LlamaDecoder(b, hp, wd, n_ctx, rope_src="table")  # device leaves: weights, caches, inputs, table
    bufs = []

    def alloc(nbytes):
        t = torch.zeros((nbytes + 3) // 4, dtype=torch.float32, device=dev)
        bufs.append(t)
        return t.data_ptr()

    G = GG.llama_decode_graph(hp, _leaves(hp, wd, dec), n_ctx, alloc=alloc)
    rc, nodes, keep = g.lower_ggml_graph(G.nodes, dec.table.data_ptr(), n_ctx, hp["freq_base"])
    assert rc == 0
    logits_ptr = G.nodes[-1].data
    out = next(x for x in bufs if x.data_ptr() == logits_ptr)
    model, cache = LM.oracle_model(hp, w, n_ctx)
    torch.cuda.synchronize()
    for p, tok in enumerate((7, 4000, 7, 123)):
        host = np.array([tok, p], np.int32)
        b.set_tensor(dec.inp.data_ptr(), host)  # inp_tokens, inp_pos
        assert b.graph_compute(nodes, use_graph=True) == 0
        b.synchronize()
        got = out[:hp["n_vocab"]].cpu().numpy()
        ref, _ = O.decode_token(model, tok, p, cache)
        assert bits_equal(got, ref), (p, first_mismatch(got, ref))
    b.close()
