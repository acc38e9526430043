"""The ggml-backend adapter, compiled and run (host only, no device).

adapter/mi355x_ggml_mirror.hpp is the part of the ggml backend that
sits between `iface.graph_compute(backend, cgraph)` (ggml-backend.cpp:1553, README.md:163)
and this library: the ggml_tensor -> mi355x_gtensor mirror, the GGML_OP_* name map, the
cells == positions check and the mi355x_lower_ggml_graph call. These tests compile it with
g++ against include/ggml_mi355x.h (tests/adapter/adapter_test.cpp: a `struct ggml_tensor`
with upstream ggml.h's field names and sizes [U]), feed it llm_build_llama's decode and
prompt graphs (tests/ggml_graph.py) as ggml tensors, and check that the node list it
produces is LlamaDecoder's — so a change to the C-ABI that the adapter does not follow
breaks the build or this comparison."""
import ctypes
import os
import subprocess

import pytest

import ggml_mi355x as g
from ggml_mi355x.llama import hparams
from tests import ggml_graph as GG
from tests.test_lower import _describe, _leaves, canon

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ggml_op_name() strings of the lowering's op numbering (enum mi355x_gop order)
GGML_OP_NAMES = ["NONE", "GET_ROWS", "RMS_NORM", "MUL", "ADD", "MUL_MAT", "ROPE", "SET_ROWS", "SOFT_MAX", "GLU",
                 "RESHAPE", "VIEW", "PERMUTE", "TRANSPOSE", "CONT", "CPY"]
GGML_TENSOR_FLAG_OUTPUT = 2  # ggml.h [U]


@pytest.fixture(scope="module")
def adapter_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("adapter") / "adapter_test")
    lib_dir = os.path.dirname(g.LIB_PATH)
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "ggml-neon-opt_amd", "adapter"),
           os.path.join(ROOT, "tests", "adapter", "adapter_test.cpp"), "-o", out,
           "-L", lib_dir, "-lggml_mi355x", f"-Wl,-rpath,{lib_dir}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


def serialize(nodes, op_name=None):
    """The graph as adapter_test.cpp reads it: every tensor reachable from the nodes."""
    ids, order = {}, []

    def visit(t):
        a = ctypes.addressof(t)
        if a in ids:
            return
        ids[a] = len(ids)
        order.append(t)
        for s in range(10):
            if t.src[s]:
                visit(t.src[s].contents)
        if t.view_src:
            visit(t.view_src.contents)

    for n in nodes:
        visit(n)

    def ref(p):
        return str(ids[ctypes.addressof(p.contents)]) if p else "-1"

    lines = []
    for t in order:
        name = (op_name or {}).get(ctypes.addressof(t)) or \
            (GGML_OP_NAMES[t.op] if 0 <= t.op < len(GGML_OP_NAMES) else "FLASH_ATTN_EXT")
        flags = GGML_TENSOR_FLAG_OUTPUT if t.flags & g.FLAG_OUTPUT else 0
        f = [str(ids[ctypes.addressof(t)]), str(t.type), name] + [str(v) for v in t.ne] + [str(v) for v in t.nb]
        f += [str(v) for v in t.op_params] + [str(flags)] + [ref(t.src[s]) for s in range(10)] + [ref(t.view_src)]
        f += [str(t.view_offs), str(t.data or 0), t.name.decode() or "-"]
        lines.append("T " + " ".join(f))
    lines.append("N %d %s" % (len(nodes), " ".join(str(ids[ctypes.addressof(n)]) for n in nodes)))
    return "\n".join(lines) + "\n"


def run_adapter(binary, tmp_path, nodes, table, n_pos, freq_base, cells_eq_pos=True):
    path = tmp_path / "graph.txt"
    path.write_text(serialize(nodes))
    r = subprocess.run([binary, str(path), "1" if cells_eq_pos else "0", str(table), str(n_pos), repr(freq_base)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    _, rc, n = lines[0].split()
    out = []
    for ln in lines[1:]:
        head, _, srcs = ln.partition(";")
        v = [int(x) for x in head.split()]
        ss = []
        for s in srcs.split():
            if s[0] == "n":
                ss.append(("node", int(s[1:])))
            else:
                ty, ne0, ne1, nb1, data = (int(x) for x in s[1:].split(","))
                ss.append(("leaf", ty, ne0, ne1, nb1, data or None))
        out.append((v[0], tuple(v[1:5]), tuple(v[5:13]), v[13], tuple(ss)))
    assert len(out) == int(n)
    return int(rc), out


@pytest.mark.parametrize("hp", [hparams(512, 2, 8, 2, 768, 1024), hparams(2048, 2, 32, 4, 5632, 4096)],
                         ids=["small-gqa4", "tinyllama-width"])
def test_adapter_lowers_llama_decode_graph(adapter_bin, tmp_path, hp):
    n_ctx = 64
    wt, dec = _describe(hp, n_ctx)
    G = GG.llama_decode_graph(hp, _leaves(hp, wt, dec), n_ctx)
    rc, got = run_adapter(adapter_bin, tmp_path, G.nodes, dec.table.data_ptr(), n_ctx, hp["freq_base"])
    assert rc == 0
    want = canon(dec.nodes)
    assert len(got) == len(want) == 2 + 15 * hp["n_layer"] + 2
    for i, (a, b) in enumerate(zip(got, want)):
        assert a == b, (i, a, b)


def test_adapter_lowers_llama_prompt_graph(adapter_bin, tmp_path):
    hp = hparams(512, 2, 8, 2, 768, 1024)
    n_ctx, n_tok = 64, 7
    wt, dec = _describe(hp, n_ctx)
    pg = dec._prompt_graph(n_tok)
    L = _leaves(hp, wt, dec)
    L["inp_tokens"] = pg["inp"][:n_tok].data_ptr()
    L["inp_pos"] = pg["inp"][n_tok:2 * n_tok].data_ptr()
    L["inp_out_ids"] = pg["inp"][2 * n_tok:].data_ptr()
    G = GG.llama_decode_graph(hp, L, n_ctx, n_tokens=n_tok)
    rc, got = run_adapter(adapter_bin, tmp_path, G.nodes, dec.table.data_ptr(), n_ctx, hp["freq_base"])
    assert rc == 0
    assert got == canon(pg["nodes"])


def test_adapter_leaves_what_it_cannot_run(adapter_bin, tmp_path):
    """No cells == positions promise, an op outside the name map (FLASH_ATTN_EXT) or a
    rope table that does not match: the lowering refuses, the scheduler keeps the graph."""
    hp = hparams(512, 1, 8, 2, 768, 1024)
    wt, dec = _describe(hp, 32)
    L = _leaves(hp, wt, dec)
    tab = dec.table.data_ptr()
    G = GG.llama_decode_graph(hp, L, 32)
    assert run_adapter(adapter_bin, tmp_path, G.nodes, tab, 32, hp["freq_base"])[0] == 0
    assert run_adapter(adapter_bin, tmp_path, G.nodes, tab, 32, hp["freq_base"],
                       cells_eq_pos=False)[0] == g.E_UNSUPPORTED
    assert run_adapter(adapter_bin, tmp_path, G.nodes, tab, 32, 500000.0)[0] == g.E_UNSUPPORTED
    next(t for t in G.nodes if t.op == g.GOP_SOFT_MAX).op = 99  # -> "FLASH_ATTN_EXT"
    assert run_adapter(adapter_bin, tmp_path, G.nodes, tab, 32, hp["freq_base"])[0] == g.E_UNSUPPORTED


# ---------------------------------------------------------------- the registration glue
BASE = 1 << 44  # glue_test.cpp: tensor data at BASE + offset lives in the backend's buffer


@pytest.fixture(scope="module")
def glue_bin(tmp_path_factory):
    """adapter/ggml-mi355x.cpp (the whole ggml-backend registration: reg, device, buffer
    type, buffer, backend iface, GGML_BACKEND_DL_IMPL) + tests/adapter/glue_test.cpp,
    compiled with -Werror against the restated ggml-backend-impl.h subset."""
    out = tmp_path_factory.mktemp("glue")
    r = subprocess.run(["make", "-B", "-C", os.path.join(ROOT, "tests", "adapter"), f"BIN={out}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return str(out / "glue_test")


def test_glue_compiles_and_registers(glue_bin):
    """reg -> device count (= the library's gfx950 devices: 0 on this host) -> the DL
    entry points (ggml_backend_init returns the same registry, ggml_backend_score 0 without a
    device) -> init on a missing device is NULL, not a crash."""
    r = subprocess.run([glue_bin, "reg"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    n = int(r.stdout.split()[1])
    assert n == g.lib().mi355x_device_count()


def glue_inputs(tmp_path, hp, n_ctx, seed, tokens):
    """The files glue_test decode reads: llm_build_llama's decode graph with every tensor in
    ONE backend buffer (weights, norms, KV caches, inputs, node outputs at BASE + offset),
    the weight / norm bytes to upload, the tokens. Returns (argv tail, host weights)."""
    import numpy as np
    from tests import llama_model as LM
    w = LM.build(hp, seed)
    off, blob = [0], []

    def place(nbytes, data=None):
        o = (off[0] + 255) // 256 * 256
        off[0] = o + max(int(nbytes), 1)
        if data is not None:
            blob.append((o, np.ascontiguousarray(data).tobytes()))
        return BASE + o

    L = {}
    for k, v in w.items():
        if isinstance(v, tuple):
            t, a = v
            L[k] = (t, a.shape[1] // g.BLOCK_BYTES[t] * 256, a.shape[0], place(a.nbytes, a), a.shape[1])
        else:
            L[k] = place(v.nbytes, v)
    kvw = hp["n_head_kv"] * hp["head_dim"]
    for i in range(hp["n_layer"]):
        L[f"k_cache.{i}"] = place(n_ctx * kvw * 2)
        L[f"v_cache.{i}"] = place(n_ctx * kvw * 2)
    L["inp_tokens"], L["inp_pos"] = place(4), place(4)
    L["kq_mask"], L["k_idxs"], L["v_idxs"] = place(n_ctx * 2), place(8), place(kvw * 8)
    G = GG.llama_decode_graph(hp, L, n_ctx, alloc=lambda nb: place(nb))
    (tmp_path / "graph.txt").write_text(serialize(G.nodes))
    with open(tmp_path / "blob.bin", "wb") as f:
        for o, b in blob:
            f.write(np.array([o, len(b)], np.uint64).tobytes())
            f.write(b)
    (tmp_path / "tokens.txt").write_text(" ".join(str(t) for t in tokens))
    total = (off[0] + 4095) // 4096 * 4096
    argv = [str(tmp_path / "graph.txt"), str(tmp_path / "blob.bin"), str(tmp_path / "tokens.txt"),
            str(tmp_path / "logits.bin"), str(total), str(hp["n_vocab"])]
    return argv, w


def test_glue_inputs_address_one_buffer(tmp_path):
    """The decode files describe one buffer: every tensor's data is BASE + offset inside it
    (so the harness's single alloc_buffer holds the whole graph), and the graph carries
    the inputs the glue's cells == positions check reads (k_idxs, inp_pos, the f16 mask)."""
    hp = hparams(512, 1, 8, 2, 768, 1024)
    argv, _ = glue_inputs(tmp_path, hp, 32, 0, [1, 2])
    total = int(argv[4])
    names = set()
    for ln in open(argv[0]):
        f = ln.split()
        if f[0] != "T":
            continue
        data = int(f[-2])
        assert BASE <= data < BASE + total, ln[:80]
        names.add(f[-1])
    assert {"inp_tokens", "inp_pos", "kq_mask", "k_idxs", "v_idxs", "result_output"} <= names
