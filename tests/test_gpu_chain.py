"""GPU parity of the persistent decode chain (kq_chain): a backend graph of decode
MUL_MAT stages runs as ONE launch whose stages hand activations over through
tagged write-through buffers. Every output must be bit-identical to the oracle
evaluated stage by stage (the reference's node loop, ggml-cpu.cpp:186 /
ggml_compute_forward_mul_mat ggml-cpu.c:1389), and to the per-stage kq_rows
launches (GEMV_ROWS), across repeated launches with changing inputs.
"""
import numpy as np
import pytest

from test_gpu_parity import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu


class Graph:
    """Nodes of a decode graph on a Backend: stages of (type, N) matrices sharing one
    K; `src` = index of the producing node (its output is the stage's activation) or
    None (a host-written activation)."""

    def __init__(self, g, be, rng, npo, spec, K0, d_lo=2.0 ** -14, d_hi=2.0 ** -6):
        self.g, self.be = g, be
        self.bufs, self.nodes, self.w, self.meta = [], [], [], []
        self.x_ext = {}
        for si, (src, mats) in enumerate(spec):
            K = K0 if src is None else mats_N(spec, src)
            if src is None:
                x = rng.standard_normal((1, K)).astype(np.float32)
                xp = self.up(x)
                xt = g.make_tensor(g.TYPE_F32, K, 1, xp)
                self.x_ext[si] = (x, xp)
            else:
                prod = self.nodes[src]
                xt = g.make_tensor(g.TYPE_F32, K, 1, prod.data)
            for ty, N in mats:
                w = npo.random_blocks(rng, ty, N, K, d_lo=d_lo, d_hi=d_hi)
                wt = g.make_tensor(ty, K, N, self.up(w))
                out = g.make_tensor(g.TYPE_F32, N, 1, self.alloc(N * 4), op=g.OP_MUL_MAT, src0=wt, src1=xt)
                self.nodes.append(out)
                self.w.append((ty, w))
                self.meta.append((si, src, K, N))

    def up(self, a):
        p = self.be.alloc(a.nbytes)
        self.be.set_tensor(p, a)
        self.bufs.append(p)
        return p

    def alloc(self, n):
        p = self.be.alloc(n)
        self.bufs.append(p)
        return p

    def set_x(self, si, x):
        self.x_ext[si] = (x, self.x_ext[si][1])
        self.be.set_tensor(self.x_ext[si][1], x)

    def outputs(self):
        res = []
        for (si, src, K, N), o in zip(self.meta, self.nodes):
            h = np.zeros(N, np.float32)
            self.be.get_tensor(h, o.data)
            res.append(h)
        self.be.synchronize()
        return res

    def oracle(self, oracle):
        res = []
        for (si, src, K, N), (ty, w) in zip(self.meta, self.w):
            x = self.x_ext[si][0] if src is None else res[src][:K][None]
            res.append(oracle.mul_mat(ty, w, x)[0])
        return res

    def close(self):
        for p in self.bufs:
            self.be.free_buffer(p)
        self.be.close()


def mats_N(spec, node):
    """N of the node-th matrix (flattened over stages)."""
    i = 0
    for _, mats in spec:
        for _, N in mats:
            if i == node:
                return N
            i += 1
    raise IndexError(node)


# A small decoder-shaped chain: E=512, KV=256, FF=1024; nodes are numbered in order
# q=0 k=1 v=2 | o=3 | gate=4 up=5 | down=6 | q'=7 k'=8 | out=9
SMALL = [
    (None, [(12, 512), (12, 256), (14, 256)]),
    (0, [(12, 512)]),
    (3, [(12, 1024), (12, 1024)]),
    (4, [(14, 512)]),
    (6, [(13, 512), (12, 256)]),
    (7, [(14, 1000)]),
]


def run(be, nodes, use_graph):
    assert be.graph_compute(nodes, use_graph=use_graph) == 0
    be.synchronize()  # raises on MI355X_E_TIMEOUT (a hand-off that never completed)


def test_chain_dependent_bit_exact(dev, oracle, npo):
    """Dependent chain (every stage reads an earlier node's output), three launches
    with a new host activation each time: bit-exact with the oracle every time (no
    stale hand-off data), and with the per-stage kq_rows launches."""
    import ggml_mi355x as g
    rng = np.random.default_rng(5)
    be = g.Backend(0)
    G = Graph(g, be, rng, npo, SMALL, 512)
    prev = g.gemv_impl(g.GEMV_CHAIN)
    try:
        for it in range(3):
            if it:
                G.set_x(0, rng.standard_normal((1, 512)).astype(np.float32))
            run(be, G.nodes, use_graph=it % 2)
            got = G.outputs()
            want = G.oracle(oracle)
            for i, (a, b) in enumerate(zip(got, want)):
                assert bits_equal(a, b), (it, i, first_mismatch(a, b))
        g.gemv_impl(g.GEMV_ROWS)
        run(be, G.nodes, use_graph=0)
        rows = G.outputs()
        for i, (a, b) in enumerate(zip(rows, want)):
            assert bits_equal(a, b), (i, first_mismatch(a, b))
    finally:
        g.gemv_impl(prev)
        G.close()


def test_chain_independent_stages(dev, oracle, npo):
    """Stages whose activations are all host-written (no hand-off): one chain launch."""
    import ggml_mi355x as g
    rng = np.random.default_rng(6)
    be = g.Backend(0)
    spec = [(None, [(12, 300)]), (None, [(14, 77), (12, 64)]), (None, [(13, 129)])]
    G = Graph(g, be, rng, npo, spec, 768)
    prev = g.gemv_impl(g.GEMV_CHAIN)
    try:
        for it in range(2):
            run(be, G.nodes, use_graph=0)
            for i, (a, b) in enumerate(zip(G.outputs(), G.oracle(oracle))):
                assert bits_equal(a, b), (it, i, first_mismatch(a, b))
    finally:
        g.gemv_impl(prev)
        G.close()


def test_chain_tinyllama_layers_equal_rows(dev, npo):
    """Two TinyLlama-1.1B layers (real shapes, Q4_K_M mix) + the Q6_K output head as
    one dependent chain: bit-identical to the per-stage kq_rows launches (which the
    oracle pins in test_gpu_parity), over repeated launches."""
    import ggml_mi355x as g
    E, KV, FF, V = 2048, 256, 5632, 32000
    spec = []
    node = 0
    src = None
    for layer in range(2):
        spec.append((src, [(12, E), (12, KV), (14 if layer == 0 else 12, KV)]))
        q = node
        node += 3
        spec.append((q, [(12, E)]))
        o = node
        node += 1
        spec.append((o, [(12, FF), (12, FF)]))
        gate = node
        node += 2
        spec.append((gate, [(14 if layer == 0 else 12, E)]))
        src = node
        node += 1
    spec.append((src, [(14, V)]))
    rng = np.random.default_rng(8)
    be = g.Backend(0)
    # d in [2^-20, 2^-14]: activations stay O(1) down the chain
    G = Graph(g, be, rng, npo, spec, E, d_lo=2.0 ** -20, d_hi=2.0 ** -14)
    prev = g.gemv_impl(g.GEMV_ROWS)
    try:
        run(be, G.nodes, use_graph=0)
        want = G.outputs()
        assert all(np.isfinite(w).all() for w in want)
        g.gemv_impl(g.GEMV_CHAIN)
        for it in range(3):
            run(be, G.nodes, use_graph=0)
            for i, (a, b) in enumerate(zip(G.outputs(), want)):
                assert bits_equal(a, b), (it, i, first_mismatch(a, b))
    finally:
        g.gemv_impl(prev)
        G.close()
