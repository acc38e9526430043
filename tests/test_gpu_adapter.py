"""GPU: the ggml-backend registration (adapter/ggml-mi355x.cpp) driven the way llama.cpp's
registry and scheduler drive a backend — ggml_backend_mi355x_reg() -> device (props,
supports_op, supports_buft) -> init_backend -> buffer type -> alloc_buffer -> set_tensor of
the weights (GGUF block bytes unchanged) -> per token the graph inputs (set_tensor, and the
backend's async set) -> graph_compute(cgraph) -> get_tensor of the logits — on
llm_build_llama's decode graph (tests/ggml_graph.py) at TinyLlama width. The logits of
every token are bit-exact with the oracle's sequential token (oracle/kq_ops_oracle.py), and a
KQ mask that hides a cell inside [0, pos] (another sequence's cell) is refused
(GGML_STATUS_FAILED), never computed wrongly. The harness (tests/adapter/glue_test.cpp) is
prebuilt by __graft_entry__.build()."""
import os
import subprocess

import numpy as np
import pytest

from tests.test_gpu_parity import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLUE = os.path.join(ROOT, "tests", "adapter", "bin", "glue_test")


def test_glue_registry_on_device(dev):
    assert os.path.exists(GLUE), "tests/adapter/bin/glue_test missing: run __graft_entry__.build()"
    r = subprocess.run([GLUE, "reg"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    assert int(r.stdout.split()[1]) >= 1


@pytest.mark.parametrize("n_layer", [2])
def test_glue_decodes_llama_graph_bit_exact(dev, tmp_path, n_layer):
    from oracle import kq_ops_oracle as O
    from tests import llama_model as LM
    from tests.test_adapter import glue_inputs
    from ggml_mi355x.llama import hparams
    assert os.path.exists(GLUE), "tests/adapter/bin/glue_test missing: run __graft_entry__.build()"
    O.lib()
    hp = hparams(2048, n_layer, 32, 4, 5632, 4096)
    n_ctx = 64
    tokens = [7, 4000, 7, 123, 1]
    argv, w = glue_inputs(tmp_path, hp, n_ctx, 41, tokens)
    r = subprocess.run([GLUE, "decode"] + argv, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-3000:] + r.stderr[-3000:]
    assert "unsupported 0" in r.stdout  # the scheduler would place every node of the graph here
    assert "refused -1" in r.stdout
    got = np.fromfile(argv[3], np.float32).reshape(len(tokens), hp["n_vocab"])
    model, cache = LM.oracle_model(hp, w, n_ctx)
    for p, tok in enumerate(tokens):
        ref, _ = O.decode_token(model, tok, p, cache)
        assert bits_equal(got[p], ref), (p, first_mismatch(got[p], ref))
