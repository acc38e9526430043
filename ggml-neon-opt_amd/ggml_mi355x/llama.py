"""The llama decode graph (llm_build_llama, one token, non-flash attention) as
ggml-mirror nodes on the MI355X backend.

The reference builds this graph in llama.cpp (llama_model::build_graph ->
llm_build_llama, artifacts/perf/out.folded:249-251) and ggml-cpu computes it node by
node (ggml_graph_compute_thread -> ggml_compute_forward, out.folded:91-234). Here the
same nodes go to mi355x_backend_graph_compute, which fuses RMS_NORM -> MUL -> MUL_MAT,
SWIGLU -> MUL_MAT and MUL_MAT -> ADD into the GEMV launches, and replays the token's
launches from a hipGraph (the node list is identical for every token; the token id
and position are device inputs written before each step, as ggml's inp_tokens /
inp_pos are).

Per layer:
  rms_norm(x)*attn_norm -> q, k, v (MUL_MAT) -> ATTN_DECODE (rope, f16 KV cache,
  KQ, soft_max, KQV) -> attn_output (MUL_MAT) -> +x -> rms_norm*ffn_norm ->
  gate, up (MUL_MAT) -> swiglu -> down (MUL_MAT) -> +ffn_inp
then rms_norm*output_norm -> output (MUL_MAT) -> logits.
"""
from __future__ import annotations

import ctypes

from . import (FLAG_OUTPUT, OP_ADD, OP_ALL_GATHER, OP_ALL_REDUCE, OP_ATTN_DECODE, OP_GET_ROWS, OP_MUL, OP_MUL_MAT,
               OP_RMS_NORM,
               OP_SWIGLU, TYPE_F16, TYPE_F32, TYPE_I32, Backend, Mi355xError, f32_bits, make_tensor, rope_table)

def torch_tensor(values):
    import torch
    return torch.tensor(list(values), dtype=torch.int32)


LAYER_MATS = ("attn_q", "attn_k", "attn_v", "attn_output", "ffn_gate", "ffn_up", "ffn_down")


def hparams(n_embd, n_layer, n_head, n_head_kv, n_ff, n_vocab, eps=1e-5, freq_base=10000.0):
    return dict(n_embd=n_embd, n_layer=n_layer, n_head=n_head, n_head_kv=n_head_kv, head_dim=n_embd // n_head,
                n_ff=n_ff, n_vocab=n_vocab, eps=eps, freq_base=freq_base)


TINYLLAMA = hparams(2048, 22, 32, 4, 5632, 32000)
LLAMA3_8B = hparams(4096, 32, 32, 8, 14336, 128256, eps=1e-5, freq_base=500000.0)


class LlamaDecoder:
    """Device state and node list of one decode token.

    weights: dict with "token_embd", "output", "output_norm" and per layer i
    "blk.{i}.<name>" for name in LAYER_MATS + ("attn_norm", "ffn_norm"); a K-quant
    matrix is (type, uint8 cuda tensor [rows, rowbytes]), a norm is an f32 cuda tensor.

    split: a rowsplit.TokenSplit — this process is one rank of a row split; the
    matrices in `weights` are then the rank's row slices (TokenSplit.slice_weights),
    the KV caches hold the rank's KV heads, and every stage's slice is ALL_GATHERed
    (RCCL, the backend's communicator) before the next stage reads it. The logits
    (and every gathered vector) are bit-identical to the single-GPU token.
    """

    HOST_SLOTS = 1024

    def __init__(self, backend: Backend, hp: dict, weights: dict, n_ctx: int, fuse: bool = True, split=None,
                 rope_src: str = "row"):
        """backend None: describe only (host tensors, no device work) — the node list
        the ggml lowering must reproduce (tests/test_lower.py). rope_src "row": the
        attention reads the position's rope row staged with the inputs (the default);
        "table": the whole table (what mi355x_lower_ggml_graph passes)."""
        import torch
        self.b, self.hp, self.w, self.n_ctx, self.split = backend, hp, weights, n_ctx, split
        dev = weights["output_norm"].device
        E, F, V = hp["n_embd"], hp["n_ff"], hp["n_vocab"]
        hd, nh, nkv = hp["head_dim"], hp["n_head"], hp["n_head_kv"]
        world = split.world if split is not None else 1
        if split is not None:
            nh, nkv = split.n_head, split.n_head_kv  # this rank's heads
        kvw = nkv * hd
        self.gathers = []  # (node output buffer) of every ALL_GATHER, in graph order
        self.reduces = []  # (input partial, output) buffers of every ALL_REDUCE (split mode "reduce")
        reduce_mode = split is not None and split.mode == "reduce"
        f32 = torch.float32

        def buf(n, dtype=f32):
            return torch.zeros(n, dtype=dtype, device=dev)

        # inp_tokens, inp_pos and the rope row of that position side by side: one
        # set_tensor of 8 + 4*head_dim bytes per token. The attention reads its cos/sin
        # with q/k/v instead of after the position (one dependent round trip less);
        # the row is the table's row, so the values are those of the device table.
        self.inp = buf(2 + hd, torch.int32)
        self.token, self.pos = self.inp[0:1], self.inp[1:2]
        if backend is not None:
            self.table = rope_table(n_ctx, hd, hp["freq_base"], 1.0, device=dev, stream=backend.stream)
            self._table_host = self.table.cpu().reshape(n_ctx, hd).view(torch.int32)
        else:
            self.table = torch.zeros(n_ctx * hd, dtype=f32, device=dev)
        self.k_cache = [torch.zeros((n_ctx, kvw), dtype=torch.int16, device=dev) for _ in range(hp["n_layer"])]
        self.v_cache = [torch.zeros((kvw, n_ctx), dtype=torch.int16, device=dev) for _ in range(hp["n_layer"])]
        self._bufs = []
        self.nodes = []
        T = []  # keeps every Tensor alive

        def leaf(t, type_, ne0, ne1=1, row_stride=None):
            x = make_tensor(type_, ne0, ne1, t.data_ptr(), row_stride=row_stride)
            T.append(x)
            return x

        def node(op, n, srcs, params=None, flags=0, ne1=1):
            b = buf(n)
            self._bufs.append(b)
            x = make_tensor(TYPE_F32, n, ne1, b.data_ptr(), op=op, srcs=srcs, op_params=params, flags=flags)
            T.append(x)
            self.nodes.append(x)
            return x, b

        def mat(name):
            t, w = weights[name]
            return leaf(w, t, w.shape[1] * 256 // {12: 144, 13: 176, 14: 210}[t], w.shape[0], row_stride=w.stride(0))

        def mm(name, x):
            wt = mat(name)
            return node(OP_MUL_MAT, wt.ne[1], [wt, x])[0]

        def gather(part, n_local, flags=0):
            """ALL_GATHER of a row-split stage's slice (emitted for every split, a
            world-1 split included: one RCCL copy; none without a split)."""
            if split is None:
                return part, None
            full, b = node(OP_ALL_GATHER, n_local * world, [part], flags=flags)
            self.gathers.append(b)
            return full, b

        def allreduce(part, part_buf):
            """ALL_REDUCE(sum) of a K-split stage's partial (reduce mode)."""
            full, b = node(OP_ALL_REDUCE, part.ne[0], [part])
            self.reduces.append((part_buf, b))
            return full, b

        def rows_view(t_buf, lo, n):
            """The rows [lo, lo+n) of a full f32 vector (the residual of a local slice)."""
            return leaf(t_buf[lo:lo + n], TYPE_F32, n)

        El = E // world
        r_e0 = split.rows["attn_output"][0] if split is not None else 0

        eps_bits = [f32_bits(hp["eps"])]
        tok = leaf(self.token, TYPE_I32, 1)
        pos = leaf(self.pos, TYPE_I32, 1)
        if rope_src == "row":
            tab = leaf(self.inp[2:], TYPE_F32, hd, 1)  # the position's rope row (ne1 = 1)
        else:
            tab = leaf(self.table, TYPE_F32, hd, n_ctx)
        et, ew = weights["token_embd"]
        emb_t = leaf(ew, et, E, ew.shape[0], row_stride=ew.stride(0) * ew.element_size())
        x, xb = node(OP_GET_ROWS, E, [emb_t, tok])
        scale = f32_bits(float(torch.tensor(1.0) / torch.sqrt(torch.tensor(float(hd)))))
        for i in range(hp["n_layer"]):
            p = f"blk.{i}."
            n1, _ = node(OP_RMS_NORM, E, [x], eps_bits)
            m1, _ = node(OP_MUL, E, [n1, leaf(weights[p + "attn_norm"], TYPE_F32, E)])
            q = mm(p + "attn_q", m1)
            k = mm(p + "attn_k", m1)
            v = mm(p + "attn_v", m1)
            kc = leaf(self.k_cache[i], TYPE_F16, kvw, n_ctx)
            vc = leaf(self.v_cache[i], TYPE_F16, n_ctx, kvw)
            att, _ = node(OP_ATTN_DECODE, nh * hd, [q, k, v, pos, kc, vc, tab], [nh, nkv, hd, scale])
            if reduce_mode:
                # K-split attn_output over the rank's heads; the residual rides on rank 0's
                # partial, so the ALL_REDUCE delivers mul_mat + x
                o = mm(p + "attn_output", att)
                if split.rank == 0:
                    o, ob = node(OP_ADD, E, [o, x])
                else:
                    ob = self._bufs[-1]
                ffn_inp, fb = allreduce(o, ob)
            else:
                att, _ = gather(att, nh * hd)
                o = mm(p + "attn_output", att)
                res = x if split is None else rows_view(xb, r_e0, El)
                ffn_inp, fb = node(OP_ADD, El, [o, res])
                ffn_inp, fbg = gather(ffn_inp, El)
                fb = fbg if fbg is not None else fb
            n2, _ = node(OP_RMS_NORM, E, [ffn_inp], eps_bits)
            m2, _ = node(OP_MUL, E, [n2, leaf(weights[p + "ffn_norm"], TYPE_F32, E)])
            gt = mm(p + "ffn_gate", m2)
            up = mm(p + "ffn_up", m2)
            glu, _ = node(OP_SWIGLU, gt.ne[0], [gt, up])
            if reduce_mode:  # the rank's ffn rows are its K slice of ffn_down
                dn = mm(p + "ffn_down", glu)
                if split.rank == 0:
                    dn, db = node(OP_ADD, E, [dn, ffn_inp])
                else:
                    db = self._bufs[-1]
                x, xb = allreduce(dn, db)
            else:
                glu, _ = gather(glu, F // world)
                dn = mm(p + "ffn_down", glu)
                res = ffn_inp if split is None else rows_view(fb, r_e0, El)
                x, xb = node(OP_ADD, El, [dn, res])
                x, xbg = gather(x, El)
                xb = xbg if xbg is not None else xb
            self.last_hidden = xb
        n3, _ = node(OP_RMS_NORM, E, [x], eps_bits)
        m3, _ = node(OP_MUL, E, [n3, leaf(weights["output_norm"], TYPE_F32, E)])
        wt = mat("output")
        if split is None:
            _, self.logits = node(OP_MUL_MAT, V, [wt, m3], flags=FLAG_OUTPUT)
        else:
            lg, _ = node(OP_MUL_MAT, wt.ne[1], [wt, m3])
            _, self.logits = gather(lg, V // world, flags=FLAG_OUTPUT)
        self._tensors = T
        self._arr = (ctypes.POINTER(type(T[0])) * len(self.nodes))(*[ctypes.pointer(n) for n in self.nodes])
        if backend is None:
            return
        # pinned staging slots for (token, pos): a slot is reused only after the stream
        # has been synchronized (the H2D copies are asynchronous)
        self._host = torch.zeros((self.HOST_SLOTS, 2 + hd), dtype=torch.int32).pin_memory()
        self._slot = 0
        backend.set_fusion(fuse)
        torch.cuda.synchronize()  # weights / zeroed caches (torch's stream) before the backend stream runs

    def reset(self):
        for c in self.k_cache + self.v_cache:
            c.zero_()

    # ------------------------------------------------------------ prompt processing
    def _prompt_graph(self, n_tok: int):
        """Node list of a prompt batch of n_tok tokens (llm_build_llama over a ubatch,
        ggml's batched non-flash attention; llama-bench pp): the same weights, caches and
        rope table as the decode token. MUL_MATs take ne11 = n_tok columns (the int8-MFMA
        GEMMs), RMS_NORM/MUL/ADD/SWIGLU run on [n, n_tok], the attention node writes the
        batch's cells then runs every query causally, and only the last token's row goes
        through the output norm and head (llama.cpp computes the logits of the last token
        of a prompt)."""
        import torch
        cached = getattr(self, "_prompts", {}).get(n_tok)
        if cached is not None:
            return cached
        if self.split is not None:
            raise Mi355xError("prompt processing runs on one GPU (no row split)")
        hp, weights, n_ctx = self.hp, self.w, self.n_ctx
        dev = weights["output_norm"].device
        E, V = hp["n_embd"], hp["n_vocab"]
        hd, nh, nkv = hp["head_dim"], hp["n_head"], hp["n_head_kv"]
        kvw = nkv * hd
        T, bufs, nodes = [], [], []
        inp = torch.zeros(2 * n_tok + 1, dtype=torch.int32, device=dev)  # token ids | positions | out id

        def leaf(t, type_, ne0, ne1=1, row_stride=None):
            x = make_tensor(type_, ne0, ne1, t.data_ptr(), row_stride=row_stride)
            T.append(x)
            return x

        def node(op, n, srcs, params=None, flags=0, ne1=1):
            b = torch.zeros(n * ne1, dtype=torch.float32, device=dev)
            bufs.append(b)
            x = make_tensor(TYPE_F32, n, ne1, b.data_ptr(), op=op, srcs=srcs, op_params=params, flags=flags)
            T.append(x)
            nodes.append(x)
            return x, b

        def mm(name, x):
            t, w = weights[name]
            wt = leaf(w, t, w.shape[1] * 256 // {12: 144, 13: 176, 14: 210}[t], w.shape[0], row_stride=w.stride(0))
            return node(OP_MUL_MAT, wt.ne[1], [wt, x], ne1=x.ne[1])[0]

        eps_bits = [f32_bits(hp["eps"])]
        tok = leaf(inp[:n_tok], TYPE_I32, n_tok)
        pos = leaf(inp[n_tok:2 * n_tok], TYPE_I32, n_tok)
        out_ids = leaf(inp[2 * n_tok:], TYPE_I32, 1)  # inp_out_ids: the last token's row
        tab = leaf(self.table, TYPE_F32, hd, n_ctx)
        et, ew = weights["token_embd"]
        emb_t = leaf(ew, et, E, ew.shape[0], row_stride=ew.stride(0) * ew.element_size())
        x, xb = node(OP_GET_ROWS, E, [emb_t, tok], ne1=n_tok)
        scale = f32_bits(float(torch.tensor(1.0) / torch.sqrt(torch.tensor(float(hd)))))
        for i in range(hp["n_layer"]):
            p = f"blk.{i}."
            n1, _ = node(OP_RMS_NORM, E, [x], eps_bits, ne1=n_tok)
            m1, _ = node(OP_MUL, E, [n1, leaf(weights[p + "attn_norm"], TYPE_F32, E)], ne1=n_tok)
            q, k, v = mm(p + "attn_q", m1), mm(p + "attn_k", m1), mm(p + "attn_v", m1)
            kc = leaf(self.k_cache[i], TYPE_F16, kvw, n_ctx)
            vc = leaf(self.v_cache[i], TYPE_F16, n_ctx, kvw)
            att, _ = node(OP_ATTN_DECODE, nh * hd, [q, k, v, pos, kc, vc, tab], [nh, nkv, hd, scale], ne1=n_tok)
            o = mm(p + "attn_output", att)
            rows = n_tok
            if i == hp["n_layer"] - 1 and n_tok > 1:
                # llm_build_llama's inp_out_ids: after the last attention only the rows whose
                # logits are wanted (the last token's) go on: GET_ROWS of attn_out and inpSA
                o, _ = node(OP_GET_ROWS, E, [o, out_ids])
                x, _ = node(OP_GET_ROWS, E, [x, out_ids])
                rows = 1
            ffn_inp, _ = node(OP_ADD, E, [o, x], ne1=rows)
            n2, _ = node(OP_RMS_NORM, E, [ffn_inp], eps_bits, ne1=rows)
            m2, _ = node(OP_MUL, E, [n2, leaf(weights[p + "ffn_norm"], TYPE_F32, E)], ne1=rows)
            gt, up = mm(p + "ffn_gate", m2), mm(p + "ffn_up", m2)
            glu, _ = node(OP_SWIGLU, gt.ne[0], [gt, up], ne1=rows)
            dn = mm(p + "ffn_down", glu)
            x, xb = node(OP_ADD, E, [dn, ffn_inp], ne1=rows)
        n3, _ = node(OP_RMS_NORM, E, [x], eps_bits)
        m3, _ = node(OP_MUL, E, [n3, leaf(weights["output_norm"], TYPE_F32, E)])
        t_out, w_out = weights["output"]
        wt = leaf(w_out, t_out, w_out.shape[1] * 256 // {12: 144, 13: 176, 14: 210}[t_out], w_out.shape[0],
                  row_stride=w_out.stride(0))
        _, logits = node(OP_MUL_MAT, V, [wt, m3], flags=FLAG_OUTPUT)
        g = dict(inp=inp, nodes=nodes, tensors=T, bufs=bufs, logits=logits, hidden=xb, pos=pos,
                 arr=(ctypes.POINTER(type(T[0])) * len(nodes))(*[ctypes.pointer(n) for n in nodes]),
                 host=torch.zeros(2 * n_tok + 1, dtype=torch.int32).pin_memory() if self.b is not None else None)
        if not hasattr(self, "_prompts"):
            self._prompts = {}
        self._prompts[n_tok] = g
        if self.b is not None:
            torch.cuda.synchronize()  # zeroed buffers (torch's stream) before the backend stream runs
        return g

    def prompt(self, tokens, start_pos: int = 0, use_graph: bool = True):
        """Enqueue a prompt batch (positions start_pos ..): writes its KV cells and returns
        the device logits of its last token (no synchronization). The logits and the cache
        equal those of decoding the tokens one by one with step(), bit for bit."""
        n_tok = len(tokens)
        if n_tok < 1 or start_pos < 0 or start_pos + n_tok > self.n_ctx:
            raise Mi355xError(f"prompt of {n_tok} tokens at {start_pos} outside the KV cache (n_ctx {self.n_ctx})")
        if any(not 0 <= t < self.hp["n_vocab"] for t in tokens):
            raise Mi355xError("prompt token outside the vocabulary")
        from . import lib
        g = self._prompt_graph(n_tok)
        self.b.synchronize()  # the pinned staging row is reused: the previous prompt's copy is done
        host = g["host"]
        host[:n_tok] = torch_tensor(tokens)
        host[n_tok:2 * n_tok] = torch_tensor(range(start_pos, start_pos + n_tok))
        host[2 * n_tok] = n_tok - 1
        L = lib()
        rc = L.mi355x_backend_set_tensor(self.b.h, g["inp"].data_ptr(), host.data_ptr(), 4 * host.numel())
        if rc:
            raise Mi355xError(f"set_tensor failed ({rc})")
        rc = L.mi355x_backend_graph_compute(self.b.h, g["arr"], len(g["nodes"]), 1 if use_graph else 0)
        if rc:
            raise Mi355xError(f"graph_compute failed ({rc})")
        self.prompt_hidden = g["hidden"]
        return g["logits"]

    def step(self, token: int, pos: int, use_graph: bool = True):
        """Enqueue one token (no synchronization); returns the device logits tensor."""
        if not 0 <= pos < self.n_ctx:
            raise Mi355xError(f"position {pos} outside the KV cache (n_ctx {self.n_ctx})")
        if not 0 <= token < self.hp["n_vocab"]:
            raise Mi355xError(f"token {token} outside the vocabulary (n_vocab {self.hp['n_vocab']})")
        from . import lib
        if self._slot == self.HOST_SLOTS:
            self.b.synchronize()
            self._slot = 0
        row = self._host[self._slot]
        row[0] = token
        row[1] = pos
        row[2:] = self._table_host[pos]
        L = lib()
        hp = row.data_ptr()
        self._slot += 1
        rc = L.mi355x_backend_set_tensor(self.b.h, self.inp.data_ptr(), hp, 4 * row.numel())
        if rc:
            raise Mi355xError(f"set_tensor failed ({rc})")
        rc = L.mi355x_backend_graph_compute(self.b.h, self._arr, len(self.nodes), 1 if use_graph else 0)
        if rc:
            raise Mi355xError(f"graph_compute failed ({rc})")
        return self.logits
