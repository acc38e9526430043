#!/usr/bin/env python3
"""bench.py — tg128 tokens/s of TinyLlama-1.1B Q4_K_M on MI355X (the full decode graph),
plus the Q4_K x Q8_K GEMV's achieved HBM bandwidth against the roofline.

Default workload ("token"): llama-bench's tg128 — token i decoded at position i of
a fresh KV cache, i = 0 .. steps-1, each step the whole llm_build_llama graph
(get_rows, per layer rms_norm -> q/k/v -> rope + f16 KV cache + attention -> o ->
add -> rms_norm -> gate/up -> swiglu -> down -> add, then rms_norm -> output)
through ggml_mi355x.llama.LlamaDecoder and mi355x_backend_graph_compute (node
fusion: 5 launches per layer + 2, replayed from a hipGraph). The token id and
position are written to the device before each step as ggml's inputs are. The
per-token MUL_MAT chain alone ("chain" workload, described below) is reported
beside it in "matmul_chain".

Metric (BASELINE.json): "tg128 tok/s + Q4_K GEMV achieved-HBM-GB/s, TinyLlama-1.1B
Q4_K_M @1 GPU". One step = one decoded token of the whole graph; its matmuls carry
629.8 MB of K-quant weights in the Q4_K_M type mix of llama-quant.cpp [U]
(attn_v/ffn_down Q6_K in the 10 use_more_bits layers, output Q6_K, token_embd
Q4_K), each GEMV including its bit-exact Q8_K activation quantization. Weights are
synthetic random blocks of the real shapes (no network for the GGUF), their fp16
scales sized so the residual stream keeps an O(1) RMS; norms f32 in [0.8, 1.2].

"chain" workload (--workload chain; the GGUF-file and kernel A/B modes): the
per-token MUL_MAT chain only, every stage reading the previous stage's output
(attn_q -> attn_output -> ffn_gate -> ffn_down -> next layer's q/k/v ... -> output);
q/k/v and gate/up fuse into one launch each, 89 launches per token from one hipGraph.

"roofline": the dominant kernel's algorithmic bytes per launch over its event-timed
launch duration; "traffic": its HBM read per launch from the committed rocprofv3
PMC pass (profiles/). "gemv_large": single decode GEMVs of the Llama-3 configs, each
beside the single-launch streaming ceiling of its byte count ("stream_us": LDS-DMA of
a once-read buffer, no arithmetic; "of_stream_ceiling" = stream_us / us_median).
"prefill_pp512": every matmul of the token at ne11 = 512 (int8 MFMA, bit-exact);
"prefill_pp512_f16" / "pp512_f16" the same on the stated-tolerance f16 path (kq_mmf,
mi355x_prefill_precision), with an f16-peak roofline. "cpu_baseline":
the oracle's restated ggml-cpu token on this host's cores, a bounded sample.

Multi-GPU (--gpus N under torch.distributed.run): the headline is the north_star's
row-split path, ONE TinyLlama token stream split over the N GPUs in the reduce schedule
(q/k/v by heads and gate/up by ffn rows, attn_output / ffn_down split along K at
superblock boundaries, one RCCL all-reduce per K-split stage: 2 per layer; "scaling":
"strong", value = tokens/s of that one stream, max-over-ranks time). Beside it the line
carries "replicas" (every rank decodes its own stream with its own weights: the
data-parallel serving figure, weak scaling), the gather schedule ("rowsplit.gather":
every matrix by rows + one RCCL all-gather per stage), Llama-3-70B (config 4) in both
schedules with its per-GPU token_hbm_frac, and "collectives_us", the per-collective
cost on the job's ranks. `--mode replicas|rowsplit|rowsplit-reduce` picks the headline
explicitly. DESIGN.md §6 has the budget of when a split pays.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402

MODELS = {
    "tinyllama-1.1b": dict(E=2048, L=22, KV=256, FF=5632, V=32000),
    "llama-3-8b": dict(E=4096, L=32, KV=1024, FF=14336, V=128256),
    "llama-3-70b": dict(E=8192, L=80, KV=1024, FF=28672, V=128256),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
I8_PEAK_TOPS = 5000.0  # dense int8 MFMA peak (2x the 2.5 PFLOP/s dense bf16; no sparsity)


def use_more_bits(i, n):
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def q4km_chain(model, mix="q4_k_m"):
    """Per-token GEMV chain: list of stages; a stage is a list of (name, type, K, N)
    sharing one input vector (fused into one launch). mix: llama-quant.cpp's Q4_K_M
    (default) or Q5_K_M [U] (every matrix Q5_K except attn_v / ffn_down of the
    use_more_bits layers and the output, Q6_K: BASELINE config 5)."""
    m = MODELS[model]
    E, L, KV, FF, V = m["E"], m["L"], m["KV"], m["FF"], m["V"]
    big = model == "llama-3-70b"
    base = g.TYPE_Q5_K if mix == "q5_k_m" else g.TYPE_Q4_K
    stages = []
    for i in range(L):
        mb = use_more_bits(i, L)
        v_type = g.TYPE_Q6_K if mb else (g.TYPE_Q5_K if big or mix == "q5_k_m" else g.TYPE_Q4_K)
        stages.append([(f"blk.{i}.attn_q", base, E, E), (f"blk.{i}.attn_k", base, E, KV),
                       (f"blk.{i}.attn_v", v_type, E, KV)])
        stages.append([(f"blk.{i}.attn_output", base, E, E)])
        stages.append([(f"blk.{i}.ffn_gate", base, E, FF), (f"blk.{i}.ffn_up", base, E, FF)])
        stages.append([(f"blk.{i}.ffn_down", g.TYPE_Q6_K if mb else base, FF, E)])
    stages.append([("output", g.TYPE_Q6_K, E, V)])
    return stages


def gguf_chain(f):
    """The same per-token chain read from a llama-architecture GGUF file (types and
    shapes as stored; output.weight, or the tied token_embd.weight)."""
    L = int(f.kv["llama.block_count"])
    stages = []

    def mat(name, tensor=None):
        info = f.tensors[(tensor or name) + ".weight"]
        assert len(info["ne"]) == 2 and info["type"] in (g.TYPE_Q4_K, g.TYPE_Q5_K, g.TYPE_Q6_K), name
        return (name, info["type"], info["ne"][0], info["ne"][1])

    for i in range(L):
        b = f"blk.{i}."
        stages.append([mat(b + "attn_q"), mat(b + "attn_k"), mat(b + "attn_v")])
        stages.append([mat(b + "attn_output")])
        stages.append([mat(b + "ffn_gate"), mat(b + "ffn_up")])
        stages.append([mat(b + "ffn_down")])
    stages.append([mat("output", "output" if "output.weight" in f.tensors else "token_embd")])
    return stages


# E[w^2] / d^2 of a random block (6-bit scales/mins uniform, quants uniform, dmin =
# d * mean quant so a sub-block averages ~0): sum_j w_ij x_j keeps the RMS of x when
# d = 1 / sqrt(K * W2).
W2 = {12: 66727.0, 13: 277630.0, 14: 1.865e6}


def random_kquant(type_, N, K, gen, dev, rms_keep=False):
    """Random valid K-quant rows generated on the device (every qs/scales byte is
    legal; d/dmin fp16, never NaN/Inf). Default d, dmin in [2^-14, 2^-6]; rms_keep:
    d ~ U[0.75, 1.25] / sqrt(1.0208 K W2) and dmin = d * mean quant, so a chain of
    GEMVs neither blows up nor vanishes."""
    nb = K // 256
    B = g.BLOCK_BYTES[type_]
    w = torch.randint(0, 256, (N, nb, B), dtype=torch.uint8, device=dev, generator=gen)

    def f16(r):
        return r.to(torch.float16).view(torch.uint8).view(N, nb, 2)

    if rms_keep:
        d = (torch.rand((N, nb), device=dev, generator=gen) * 0.5 + 0.75) / float(np.sqrt(1.0208 * K * W2[type_]))
        dmin = d * (7.5 if type_ == g.TYPE_Q4_K else 15.5)
    else:
        d = torch.rand((N, nb), device=dev, generator=gen) * (2.0 ** -6 - 2.0 ** -14) + 2.0 ** -14
        dmin = torch.rand((N, nb), device=dev, generator=gen) * (2.0 ** -6 - 2.0 ** -14) + 2.0 ** -14
    if type_ in (g.TYPE_Q4_K, g.TYPE_Q5_K):
        w[..., 0:2] = f16(d)
        w[..., 2:4] = f16(dmin)
    else:
        w[..., 208:210] = f16(d)
    return w.view(N, nb * B)


class Chain:
    """Weights, inputs and ggml-style MUL_MAT nodes for one rank's token chain."""

    def __init__(self, model, dev, seed, gguf=None):
        self.model = model
        self.gguf = gguf
        if gguf is not None:  # real weights: a GGUFFile (ggml_mi355x.gguf)
            self.stages = gguf_chain(gguf)
            self.model = gguf.kv.get("general.name", os.path.basename(gguf.path))
        else:
            self.stages = q4km_chain(model)
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        self.w, self.x, self.y, self.nodes, self.keep = [], [], [], [], []
        self.bytes_per_token = 0
        # one decode stream: stage s+1 reads stage s's first output
        self.dependent = True
        for si, stage in enumerate(self.stages):
            K = stage[0][2]
            if self.dependent and si > 0:
                x = self.y[si - 1][0][:K]
                assert self.stages[si - 1][0][3] >= K
            else:
                x = torch.randn(K, device=dev, generator=gen)
            xt = g.make_tensor(g.TYPE_F32, K, 1, x.data_ptr())
            self.x.append(x)
            self.keep.append(xt)
            ws, ys = [], []
            for name, typ, K_, N in stage:
                r0, r1 = 0, N
                if gguf is not None:
                    tname = name + ".weight" if name + ".weight" in gguf.tensors else "token_embd.weight"
                    w = gguf.to_device(tname, dev)[r0:r1].contiguous()
                else:
                    w = random_kquant(typ, r1 - r0, K_, gen, dev, rms_keep=self.dependent)
                y = torch.empty(r1 - r0, device=dev)
                wt = g.make_tensor(typ, K_, r1 - r0, w.data_ptr())
                node = g.make_tensor(g.TYPE_F32, r1 - r0, 1, y.data_ptr(), op=g.OP_MUL_MAT, src0=wt, src1=xt)
                self.keep.append(wt)
                self.nodes.append(node)
                ws.append((typ, w))
                ys.append(y)
                self.bytes_per_token += w.numel()
            self.w.append(ws)
            self.y.append(ys)
        torch.cuda.synchronize()

    def launches(self):
        return len(self.stages)


HPARAMS = {"tinyllama-1.1b": dict(n_head=32, n_head_kv=4, freq_base=10000.0),
           "llama-3-8b": dict(n_head=32, n_head_kv=8, freq_base=500000.0),
           "llama-3-70b": dict(n_head=64, n_head_kv=8, freq_base=500000.0)}


class Token:
    """The full llama decode graph of one token (ggml_mi355x.llama.LlamaDecoder:
    get_rows, 22 x [rms_norm, q/k/v, rope + KV cache + attention, o, add, rms_norm,
    gate/up, swiglu, down, add], rms_norm, output) on synthetic Q4_K_M weights of the
    real shapes (the chain's weights and type mix, plus token_embd Q4_K and f32 norms)."""

    def __init__(self, model, dev, seed, be, n_ctx, split=None, mix="q4_k_m"):
        from ggml_mi355x.llama import LlamaDecoder, hparams
        from ggml_mi355x.rowsplit import TokenSplit
        m = MODELS[model]
        h = HPARAMS[model]
        self.hp = hparams(m["E"], m["L"], h["n_head"], h["n_head_kv"], m["FF"], m["V"], freq_base=h["freq_base"])
        self.model = model
        self.split = TokenSplit(self.hp, *split) if split is not None else None  # (world, rank[, mode])
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        self.mix = mix
        self.stages = q4km_chain(model, mix)
        w = {}
        self.bytes_per_token = 0  # this GPU's matmul weight bytes per token (its row slices)
        for stage in self.stages:
            for name, typ, K, N in stage:
                r0, r1 = self.split.rows_of(name) if self.split is not None else (0, N)
                base = name.split(".")[-1]
                if self.split is not None and base in self.split.cols:  # reduce mode: the rank's K slice
                    c0, c1 = self.split.cols[base]
                    K = 256 * (c1 - c0)
                w[name] = (typ, random_kquant(typ, r1 - r0, K, gen, dev, rms_keep=True))
                self.bytes_per_token += w[name][1].numel()
        et = g.TYPE_Q5_K if mix == "q5_k_m" else g.TYPE_Q4_K  # token_embd: the mix's base type [U]
        w["token_embd"] = (et, random_kquant(et, m["V"], m["E"], gen, dev))
        w["output_norm"] = torch.rand(m["E"], device=dev, generator=gen) * 0.4 + 0.8
        for i in range(m["L"]):
            for nm in ("attn_norm", "ffn_norm"):
                w[f"blk.{i}.{nm}"] = torch.rand(m["E"], device=dev, generator=gen) * 0.4 + 0.8
        self.w = w
        self.wl = [[w[name] for name, _, _, _ in stage] for stage in self.stages]  # per stage, as Chain.w
        self.n_ctx = n_ctx
        self.dec = LlamaDecoder(be, self.hp, w, n_ctx, split=self.split)
        self.n_launch = None
        rng = np.random.default_rng(0x51A7)  # the same token stream on every rank
        self.tokens = rng.integers(0, m["V"], size=n_ctx).tolist()

    def launches(self):
        """Kernel launches (+ collectives) per token, counted on one eager token at position 0
        (the backend's fusions decide: 4 per layer with attention + o-proj in one launch, 5
        without). Collective under a row split: every rank calls it."""
        if self.n_launch is None:
            g.timing_enable(True)
            self.dec.step(self.tokens[0], 0, use_graph=False)
            rows = g.timing_read()
            g.timing_enable(False)
            self.dec.reset()
            self.n_launch = len(rows) + (self.split.collectives_per_token() if self.split is not None else 0)
        return self.n_launch


def timed_kernel_stats(be, chain, tokens):
    """Per-launch kernel timing (hipExtLaunchKernelGGL events) over `tokens` eager chains."""
    g.timing_enable(True)
    for i in range(tokens):
        if isinstance(chain, Token):
            chain.dec.step(chain.tokens[i], i, use_graph=False)
            continue
        rc = be.graph_compute(chain.nodes, use_graph=False)
        assert rc == 0, rc
    rows = g.timing_read()
    g.timing_enable(False)
    if isinstance(chain, Token) and tokens > 0:  # launches per token, measured (every rank runs this)
        chain.n_launch = len(rows) // tokens + (chain.split.collectives_per_token() if chain.split is not None else 0)
    if os.environ.get("BENCH_KINDS_OUT") and tokens > 0:  # launch kinds of one token, in order (profiles)
        n = len(rows) // tokens
        with open(os.environ["BENCH_KINDS_OUT"], "w") as f:
            json.dump([f"{name} @ {nbytes / 1e6:.3f} MB" for name, nbytes, _ in rows[:n]], f)
    per, kinds = {}, {}
    for name, nbytes, ms in rows:
        # by kernel name, and by launch kind (name + algorithmic bytes: the q/k/v and the
        # gate/up launches of one kernel instantiation differ 4.4x in size)
        for key, tab in ((name, per), (f"{name} @ {nbytes / 1e6:.3f} MB", kinds)):
            d = tab.setdefault(key, {"launches": 0, "bytes": 0.0, "ms": 0.0, "kernel": name})
            d["launches"] += 1
            d["bytes"] += nbytes
            d["ms"] += ms
    return per, kinds


def large_gemv(dev, reps=20):
    """Decode GEMVs of the Llama-3 configs (BASELINE.json configs 3-4), one launch each,
    weight buffers rotated over > 600 MB so the 256 MB Infinity Cache cannot serve them:
    the 8B ffn_up, the 70B ffn_down, the 70B ffn_gate + ffn_up pair as the decode graph
    fuses it (one launch, shared activation) and the 8B Q6_K output head."""
    out = {}
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    shapes = (("llama3-8b ffn_up 4096x14336", g.TYPE_Q4_K, 4096, (14336,)),
              ("llama3-70b ffn_down 28672x8192", g.TYPE_Q4_K, 28672, (8192,)),
              ("llama3-70b ffn_gate+ffn_up 8192x2x28672", g.TYPE_Q4_K, 8192, (28672, 28672)),
              ("llama3-8b output q6_K 4096x128256", g.TYPE_Q6_K, 4096, (128256,)))
    for label, typ, K, Ns in shapes:
        nbytes = sum(N * (K // 256) * g.BLOCK_BYTES[typ] for N in Ns)
        nbuf = max(2, int(np.ceil(600e6 / nbytes)))
        ws = [[random_kquant(typ, N, K, gen, dev) for N in Ns] for _ in range(nbuf)]
        x = torch.randn(1, K, device=dev, generator=gen)
        ys = [torch.empty(1, N, device=dev) for N in Ns]

        def call(i):
            if len(Ns) == 1:
                g.mul_mat(typ, ws[i % nbuf][0], K, x, out=ys[0])
            else:
                g.gemv_fused([(typ, w, y[0]) for w, y in zip(ws[i % nbuf], ys)], x[0])

        for i in range(nbuf):
            call(i)
        g.timing_enable(True)
        for r in range(reps):
            call(r)
        rows = g.timing_read()
        g.timing_enable(False)
        per_call = len(rows) // reps  # K > 8192: Q8_K quantize launch + GEMV launch
        ms = [sum(r[2] for r in rows[i * per_call:(i + 1) * per_call]) for i in range(reps)]
        b = nbytes + K * 4 + sum(Ns) * 4
        del ws
        # the single-launch streaming ceiling of the same byte count (mi355x_debug_stream:
        # LDS-DMA of a once-read buffer, no arithmetic), buffers rotated the same way
        pool = torch.empty(nbuf * ((nbytes + 4095) // 4096 * 4096), dtype=torch.uint8, device=dev)
        sink = torch.zeros(16, dtype=torch.int32, device=dev)
        step = pool.numel() // nbuf
        st = torch.cuda.current_stream().cuda_stream
        for i in range(nbuf):
            g.lib().mi355x_debug_stream(pool.data_ptr() + i * step, nbytes, sink.data_ptr(), st)
        g.timing_enable(True)
        for r in range(reps):
            assert g.lib().mi355x_debug_stream(pool.data_ptr() + (r % nbuf) * step, nbytes, sink.data_ptr(), st) == 0
        srows = g.timing_read()
        g.timing_enable(False)
        sus = float(np.median([r[2] for r in srows])) * 1e3
        out[label] = {"bytes": b, "launches_per_call": per_call, "kernel": rows[per_call - 1][0],
                      "us_median": round(float(np.median(ms) * 1e3), 2),
                      "GBps_median": round(b / (np.median(ms) * 1e-3) / 1e9, 1),
                      "frac_median": round(b / (np.median(ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "stream_us": round(sus, 2),
                      "stream_frac": round(nbytes / (sus * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                      "of_stream_ceiling": round(sus / float(np.median(ms) * 1e3), 3)}
        del pool
        torch.cuda.empty_cache()
    return out


F16_PEAK_TFLOPS = 2500.0  # dense f16 MFMA peak (MI355X_MICROARCH.md)


def on_f16(fn, *a, **kw):
    """fn on the stated-tolerance f16 prefill path (mi355x_prefill_precision F16, kq_mmf),
    the bit-exact kq_mmq restored after."""
    prev = g.prefill_precision(g.PREFILL_F16)
    try:
        out = fn(*a, **kw)
    finally:
        g.prefill_precision(prev)
    if out is not None:
        out["precision"] = "f16 MFMA (kq_mmf), stated tolerance: csrc/kq_mmf.hip, tests/test_gpu_mmf.py"
        out["note"] = out["note"].replace("kq_mmq", "kq_mmf").replace("int8-MFMA", "f16-MFMA")
        if "int_TOPS" in out:
            out["f16_TFLOPS"] = out.pop("int_TOPS")
            out["roofline"] = {"bound": "mfma", "achieved": out["f16_TFLOPS"], "peak": F16_PEAK_TFLOPS,
                               "unit": "TFLOP/s (f16 dense)", "frac": round(out["f16_TFLOPS"] / F16_PEAK_TFLOPS, 4)}
    return out


def prefill_chain(chain, dev, M=512, reps=3):
    """pp512-style prefill of the same weights: every matrix of the chain times an
    M-column activation block (ne11 = M: Q8_K quantization + the int8-MFMA kq_mmq
    GEMM, bit-exact with the per-column vec_dot chain). Eager launches, one CUDA
    event pair around the whole chain; non-matmul ops excluded as in the tg chain."""
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    xs, ys = {}, {}
    for stage in chain.stages:
        for _, _, K, N in stage:
            if K not in xs:
                xs[K] = torch.randn(M, K, device=dev, generator=gen)
            if N not in ys:
                ys[N] = torch.empty(M, N, device=dev)
    ws_need = max(g.lib().mi355x_mul_mat_workspace_size(12, K, 1, M) for K in xs)
    ws = torch.empty(ws_need, dtype=torch.uint8, device=dev)

    def run():
        for si, stage in enumerate(chain.stages):
            for (name, typ, K, N), (_, w) in zip(stage, getattr(chain, "wl", chain.w)[si]):
                g.mul_mat(typ, w, K, xs[K], out=ys[N], workspace=ws)

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    macs = sum(N * K for stage in chain.stages for _, _, K, N in stage) * M
    return {"M": M, "ms_per_batch": round(ms, 3), "tok_s": round(M / (ms * 1e-3), 1),
            "int_TOPS": round(2 * macs / (ms * 1e-3) / 1e12, 1),
            "note": "all chain matmuls at ne11=M (quantize + kq_mmq per matmul, eager)"}


def prompt_side(tk, be, n_tok=512, reps=3):
    """llama-bench's pp512 through the graph: one 512-token prompt batch of the same model
    (LlamaDecoder.prompt: every MUL_MAT at ne11 = 512 on the int8-MFMA GEMMs, batched
    norms and adds, the prompt attention over the batch's causal cells, the head on the
    last token), hipGraph replay, on a decoder of n_ctx = n_tok sharing tk's weights."""
    from ggml_mi355x.llama import LlamaDecoder
    dec = LlamaDecoder(be, tk.hp, tk.w, n_tok)
    rng = np.random.default_rng(0x5EED)
    toks = rng.integers(0, tk.hp["n_vocab"], size=n_tok).tolist()
    dec.prompt(toks, 0)  # capture
    be.synchronize()
    st = torch.cuda.ExternalStream(be.stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        dec.prompt(toks, 0)
    e1.record(st)
    be.synchronize()
    ms = e0.elapsed_time(e1) / reps
    out = {"tokens": n_tok, "ms_per_batch": round(ms, 3), "tok_s": round(n_tok / (ms * 1e-3), 1),
           "nodes": len(dec._prompt_graph(n_tok)["nodes"]),
           "note": "whole prompt through the graph (MUL_MAT ne11=512 on kq_mmq, batched norms, prompt attention, "
                   "head on the last token), hipGraph replay"}
    del dec
    torch.cuda.empty_cache()
    return out


def chain_side(model, dev, be, steps=64, warmup=8):
    """The per-token MUL_MAT chain alone (no norm/rope/attention/swiglu), hipGraph replay:
    the figure earlier rounds reported as the headline."""
    chain = Chain(model, dev, seed=0x51A7)
    for _ in range(warmup):
        assert be.graph_compute(chain.nodes) == 0
    be.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = torch.cuda.ExternalStream(be.stream)
    e0.record(st)
    for _ in range(steps):
        assert be.graph_compute(chain.nodes) == 0
    e1.record(st)
    be.synchronize()
    ms = e0.elapsed_time(e1) / steps
    out = {"tok_s": round(1e3 / ms, 1), "ms_per_token": round(ms, 4), "stages_per_token": chain.launches(),
           "weights_MB_per_token": round(chain.bytes_per_token / 1e6, 1)}
    del chain
    torch.cuda.empty_cache()
    return out


def model_side(model, dev, steps=64, warmup=8, mix="q4_k_m"):
    """Another BASELINE config on the same executor: the full decode token of `model`
    (tg<steps> from an empty KV cache, hipGraph replay) and its pp512 (every matmul
    of the token at ne11 = 512, kq_mmq). Llama-3-8B covers configs 3 (pp512 + tg,
    Q4_K_M) and 5 (mix "q5_k_m": Q5_K matrices beside the Q6_K output / attn_v /
    ffn_down, one kernel template)."""
    be = g.Backend(torch.cuda.current_device())
    n_ctx = max(128, (steps + 31) // 32 * 32)
    tk = Token(model, dev, 0x51A7, be, n_ctx, mix=mix)
    for i in range(warmup):
        tk.dec.step(tk.tokens[i], i)
    be.synchronize()
    tk.dec.reset()
    torch.cuda.synchronize()
    st = torch.cuda.ExternalStream(be.stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for i in range(steps):
        tk.dec.step(tk.tokens[i], i)
    e1.record(st)
    be.synchronize()
    ms = e0.elapsed_time(e1) / steps
    out = {"tg_tok_s": round(1e3 / ms, 1), "ms_per_token": round(ms, 4), "tg_steps": steps,
           "weights_MB_per_token": round(tk.bytes_per_token / 1e6, 1),
           "effective_GBps": round(tk.bytes_per_token / (ms * 1e-3) / 1e9, 1),
           "launches_per_token": tk.launches(), "mix": mix, "pp512_graph": prompt_side(tk, be),
           "pp512": prefill_chain(tk, dev),
           "pp512_graph_f16": on_f16(prompt_side, tk, be), "pp512_f16": on_f16(prefill_chain, tk, dev)}
    del tk, be
    torch.cuda.empty_cache()
    return out


def host_cpu():
    """Host CPU model, logical CPUs of the machine and of this process's affinity."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    return model, os.cpu_count() or 1, aff


def cpu_quota():
    """CPUs this process's cgroup may use (cgroup v2 cpu.max quota / period), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            return None if q == "max" else int(q) / int(per)
        except (OSError, ValueError):
            pass
    try:  # cgroup v1
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def physical_cores():
    """Physical cores among the CPUs of this process's affinity (SMT siblings once)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1
    cores = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                cores.add(f.read().strip())
        except OSError:
            cores.add(str(c))
    return max(1, len(cores))


def cpu_baseline_token(tk, seconds):
    """The oracle's restated llm_build_llama token (ggml-cpu semantics op by op: the
    matmuls through the restated ggml_compute_forward_mul_mat — quantize_row_q8_K_ref,
    a persistent worker pool with 64-row chunks, the NEON-order vec_dot with AVX2
    integer parts (bit-identical to the scalar restatement); f16 attention, soft_max,
    rope, rms_norm, swiglu) on the same weights, tokens 0, 1, 2 ... from an empty cache.
    Legs as llama-bench runs them (BASELINE config 1 is `llama-bench -p 512 -n 128 -t 1`,
    README.md:186-195):
      * tg128 -t 1: all 128 tokens (config 1's -n 128 on one thread);
      * pp512 -t 1: the prompt's mul_mats at M = 512 (the restated batched
        ggml_compute_forward_mul_mat on one thread, q/k/v/o/gate/up/down of each layer), timed on
        as many whole layers as fit a bounded share of `seconds` and scaled to the model's layers
        (the output head runs on the batch's last token only, as llama-bench's pp does: one
        M = 1 mul_mat); attention, norms and rope of the prompt are not in the sample;
      * tg -t N with N the host threads available to this process (at most 16, the box's CPU
        share per GPU): the reported value."""
    from oracle import kq_ops_oracle as OO
    from oracle import kq_oracle as KO
    model_name, ncpu, aff = host_cpu()
    threads_n = max(1, min(16, aff))
    hp = tk.hp
    host = {k: ((v[0], v[1].cpu().numpy()) if isinstance(v, tuple) else v.cpu().numpy()) for k, v in tk.w.items()}
    layers = []
    for i in range(hp["n_layer"]):
        p = f"blk.{i}."
        layers.append({"attn_norm": host[p + "attn_norm"], "ffn_norm": host[p + "ffn_norm"],
                       "wq": host[p + "attn_q"], "wk": host[p + "attn_k"], "wv": host[p + "attn_v"],
                       "wo": host[p + "attn_output"], "w_gate": host[p + "ffn_gate"], "w_up": host[p + "ffn_up"],
                       "w_down": host[p + "ffn_down"]})
    model = {"hp": hp, "tok_embd": host["token_embd"], "output": host["output"], "output_norm": host["output_norm"],
             "layers": layers, "rope_table": OO.rope_table(tk.n_ctx, hp["head_dim"], hp["freq_base"])}
    kvw = hp["n_head_kv"] * hp["head_dim"]
    OO.lib()

    def leg(threads, budget, n_max=128):
        cache = [(np.zeros((tk.n_ctx, kvw), np.uint16), np.zeros((kvw, tk.n_ctx), np.uint16))
                 for _ in range(hp["n_layer"])]
        t0 = time.perf_counter()  # warm-up: workers started, host threads at speed
        while True:
            OO.decode_token(model, tk.tokens[0], 0, cache, n_threads=threads, variant="simd")
            if time.perf_counter() - t0 >= min(1.5, budget / 4):
                break
        for c in cache:
            c[0][:] = 0
            c[1][:] = 0
        tokens, t0 = 0, time.perf_counter()
        while True:
            OO.decode_token(model, tk.tokens[tokens % len(tk.tokens)], tokens, cache, n_threads=threads,
                            variant="simd")
            tokens += 1
            el = time.perf_counter() - t0
            if el >= budget or tokens >= n_max or tokens >= tk.n_ctx:
                break
        return tokens, el

    def pp_leg(budget, n_tok=512):
        """pp512 at -t 1: whole layers' mul_mats at M = n_tok until the budget, scaled."""
        rng = np.random.default_rng(7)
        E, F = hp["n_embd"], hp["n_ff"]
        x_e = rng.standard_normal((n_tok, E)).astype(np.float32)
        x_f = rng.standard_normal((n_tok, F)).astype(np.float32)
        x_q = rng.standard_normal((n_tok, hp["n_head"] * hp["head_dim"])).astype(np.float32)
        done, t0 = 0, time.perf_counter()
        for L in layers:
            for key, x in (("wq", x_e), ("wk", x_e), ("wv", x_e), ("wo", x_q), ("w_gate", x_e), ("w_up", x_e),
                           ("w_down", x_f)):
                KO.mul_mat(L[key][0], L[key][1], x, 1, "simd")
            done += 1
            if time.perf_counter() - t0 >= budget:
                break
        per_layer = (time.perf_counter() - t0) / done
        t1 = time.perf_counter()
        KO.mul_mat(model["output"][0], model["output"][1], x_e[-1:], 1, "simd")  # the last token's logits
        head = time.perf_counter() - t1
        total = per_layer * hp["n_layer"] + head
        return {"tok_s": round(n_tok / total, 3), "tokens": n_tok, "layers_timed": done,
                "seconds_timed": round(per_layer * done + head, 2), "seconds_scaled": round(total, 2),
                "note": f"mul_mats of {done} of {hp['n_layer']} layers at M = {n_tok} on one thread, scaled to "
                        f"{hp['n_layer']} layers, plus the output head on the last token"}

    phys = physical_cores()
    quota = cpu_quota()
    n1, e1 = leg(1, max(seconds, 12.0) * 2.0)  # tg128 -t 1 in full (config 1's -n 128)
    pp1 = pp_leg(seconds * 0.5)
    nn, en = leg(threads_n, seconds * 0.35)
    legs = {"t1": {"tok_s": round(n1 / e1, 3), "tokens": n1, "seconds": round(e1, 2),
                   "note": "tg128 -t 1 (BASELINE config 1's -n 128 -t 1)"},
            "pp512_t1": pp1,
            f"t{threads_n}": {"tok_s": round(nn / en, 3), "tokens": nn, "seconds": round(en, 2)}}
    if phys > threads_n and (quota is None or quota >= phys):  # one thread per physical core (a short leg)
        npn, epn = leg(phys, seconds * 0.25)
        legs[f"t{phys}"] = {"tok_s": round(npn / epn, 3), "tokens": npn, "seconds": round(epn, 2),
                            "note": "one thread per physical core of the process's affinity"}
    elif phys > threads_n:
        # a cgroup CPU quota below the core count: that many spinning workers time-slice on
        # the quota's CPUs (measured: 0.29 tok/s at -t 128 on a 16-CPU quota), so the leg
        # would time the scheduler, not ggml-cpu
        legs[f"t{phys}"] = {"skipped": f"cgroup CPU quota {quota:g} CPUs < {phys} physical cores"}
    return {"value": round(nn / en, 3), "unit": "tok/s", "cores": threads_n, "kind": "port",
            "legs": legs, "host_cpu": model_name, "host_logical_cpus": ncpu, "affinity_cpus": aff,
            "affinity_physical_cores": phys, "cgroup_cpu_quota": quota,
            "config1": {"pp512_t1_tok_s": pp1["tok_s"], "tg128_t1_tok_s": round(n1 / e1, 3), "tg_tokens": n1},
            "thread_cap": f"value is the -t {threads_n} leg: min(16, affinity) threads, the GPU box's CPU share "
                          f"per GPU; the -t {phys} leg uses every physical core of the affinity",
            "sample": f"tokens 0..n-1 from an empty KV cache of the full {tk.model} Q4_K_M decode graph through "
                      f"the oracle's restated llm_build_llama / ggml-cpu ops (mul_mat: quantize_row_q8_K_ref + "
                      f"NEON-order vec_dot with AVX2 integer parts, bit-identical to the scalar restatement, "
                      f"persistent pool); legs tg -t 1 ({n1} tokens, {e1:.1f} s), pp512 -t 1 ({pp1['note']}), "
                      f"-t {threads_n} ({nn} tokens, {en:.1f} s)" + (f", -t {phys}" if phys > threads_n else "") +
                      f"; value is the -t {threads_n} leg"}


def cpu_baseline(chain, seconds):
    """The oracle's restated ggml mul_mat (NEON-order scalar C, pthreads) on the same
    chain, timed on this host's cores for a bounded number of tokens."""
    from oracle import kq_oracle as O
    try:
        ncores = len(os.sched_getaffinity(0))
    except AttributeError:
        ncores = os.cpu_count() or 1
    threads = max(1, min(16, ncores))
    host = [[(typ, w.cpu().numpy()) for typ, w in ws] for ws in chain.w]
    xs = [x.cpu().numpy()[None] for x in chain.x]
    O.lib()
    tokens, t0 = 0, time.perf_counter()
    while True:
        for si, ws in enumerate(host):
            x = xs[si]
            if chain.dependent and si > 0:
                x = prev[:, :x.shape[1]]
            outs = [O.mul_mat(typ, w, x, n_threads=threads) for typ, w in ws]
            prev = outs[0]
        tokens += 1
        el = time.perf_counter() - t0
        if el >= seconds or tokens >= 50:
            break
    return {"value": tokens / el, "unit": "tok/s", "cores": threads, "kind": "port",
            "sample": f"{tokens} token(s) of the full {chain.model} Q4_K_M matmul chain (dependent stages) "
                      f"({chain.bytes_per_token / 1e6:.1f} MB/token) through the oracle's restated "
                      f"ggml_compute_forward_mul_mat (quantize_row_q8_K_ref + NEON-order vec_dot, "
                      f"{threads} pthreads), {el:.1f} s"}


def spawn_ranks(n):
    """`bench.py --gpus N` outside a launcher: start N rank processes (fresh
    interpreters, before this process touches a GPU) with the torch.distributed.run
    environment, wait for all of them and exit with the worst status."""
    import socket
    import subprocess
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # Poll every rank: when one fails (GPU fault, OOM) the others may wait forever in a
    # gloo barrier or in an RCCL collective inside the replayed hipGraph, so end them and
    # report the failing rank's status instead of blocking on them one by one.
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            print(json.dumps({"error": f"rank exited with status {bad[0]}", "statuses": [p.returncode for p in procs]}),
                  file=sys.stderr)
            sys.exit(bad[0] if bad[0] > 0 else 1)
        if all(rc == 0 for rc in rcs):
            sys.exit(0)
        time.sleep(0.2)


def spread(ms):
    """p10 / p50 / p90 (nearest rank) of per-step milliseconds, plus mean and sd."""
    v = sorted(ms)
    if not v:
        return None
    def pct(q):
        return round(v[min(len(v) - 1, max(0, int(round(q * (len(v) - 1)))))], 4)
    mean = sum(v) / len(v)
    sd = (sum((x - mean) ** 2 for x in v) / (len(v) - 1)) ** 0.5 if len(v) > 1 else 0.0
    return {"p10": pct(0.10), "p50": pct(0.50), "p90": pct(0.90), "mean": round(mean, 4), "sd": round(sd, 4),
            "n": len(v)}


def tg_side(tk, steps, barrier, reps=5):
    """llama-bench's tg128 on the same decoder: `steps` tokens from an empty KV cache
    (positions 0 .. steps-1), hipGraph replay, whatever --steps the headline used; run
    `reps` times, reported as llama-bench does (tok/s mean +- sd over the repetitions,
    README.md:192-193) beside the first run's figures. Every rank runs it (the row split's
    gathers are collective)."""
    st = torch.cuda.ExternalStream(tk.dec.b.stream)
    runs = []
    for r in range(reps):
        tk.dec.reset()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(steps):
            tk.dec.step(tk.tokens[i], i)
        e1.record(st)
        tk.dec.b.synchronize()
        barrier()
        el = time.perf_counter() - t0
        runs.append((el, e0.elapsed_time(e1)))
    el, gms = runs[0]
    rates = [steps / e for e, _ in runs]
    mean = sum(rates) / len(rates)
    sd = (sum((x - mean) ** 2 for x in rates) / (len(rates) - 1)) ** 0.5 if len(rates) > 1 else 0.0
    return {"tokens": steps, "tok_s": round(steps / el, 1), "ms_per_token": round(el / steps * 1e3, 4),
            "gpu_ms_per_token": round(gms / steps, 4),
            "reps": reps, "tok_s_mean": round(mean, 1), "tok_s_sd": round(sd, 1)}


def connect(be, world, rank):
    """RCCL communicator of the row split on backend `be`: the unique id from rank 0 over
    the gloo control plane, then mi355x_backend_set_comm on every rank. Returns None, or
    the error every rank agrees on (a failure on any rank fails all, so no rank waits in a
    collective the others never enter)."""
    err = None
    if os.environ.get("BENCH_ONE_DEVICE") and world > 1:
        # rehearsal of the N-rank job on ONE GPU (RCCL refuses two ranks on one device):
        # every rank runs its own split graph with the collectives emulated (loopback: no
        # data exchanged, so the values are not the model's) -- the control plane, the
        # line's fields and each rank's compute, never a scaling figure
        be.set_comm_loopback(rank, world)
        return None
    try:
        uid = torch.zeros(g.lib().mi355x_comm_id_size(), dtype=torch.uint8)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(g.comm_unique_id()), dtype=torch.uint8))
        if world > 1:
            import torch.distributed as dist
            dist.broadcast(uid, 0)
        be.set_comm(rank, world, bytes(uid.numpy().tobytes()))
    except Exception as e:  # noqa: BLE001 - reported in the JSON line
        err = f"{type(e).__name__}: {e}"
    if world > 1:
        import torch.distributed as dist
        bad = torch.tensor([0 if err is None else 1], dtype=torch.int32)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if bad.item() and err is None:
            err = "communicator setup failed on another rank"
    return err


def replicas_side(model, dev, world, rank, local, barrier, steps=64, warmup=8):
    """At N > 1 beside the row split: every rank decodes its own token stream with a full
    copy of the weights (no communicator, weak scaling), tokens of all ranks / the
    slowest rank's wall time. Collective: every rank calls it."""
    be = g.Backend(local)
    n_ctx = max(128, (max(steps, warmup) + 31) // 32 * 32)
    tk = Token(model, dev, 0x51A7 + rank, be, n_ctx)
    for i in range(warmup):
        tk.dec.step(tk.tokens[i], i)
    be.synchronize()
    tk.dec.reset()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        tk.dec.step(tk.tokens[i], i)
    be.synchronize()
    barrier()
    el = time.perf_counter() - t0
    import torch.distributed as dist
    t = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    out = {"model": model, "parallelism": f"replicas x{world}", "scaling": "weak", "tg_steps": steps,
           "tok_s": round(world * steps / el, 1), "tok_s_per_gpu": round(steps / el, 1),
           "ms_per_token": round(el / steps * 1e3, 4),
           "token_hbm_frac": round(tk.bytes_per_token * steps / el / 1e9 / HBM_PEAK_GBS, 4)}
    del tk, be
    torch.cuda.empty_cache()
    return out


def split_model_side(model, dev, world, rank, local, barrier, steps=16, warmup=4, mode="gather"):
    """BASELINE config 4 on the same executor: `model`'s full decode token split over the
    job's ranks — mode "gather" (every matrix by output rows, one RCCL ALL_GATHER node
    per stage, bit-exact) or "reduce" (attn_output / ffn_down split along K, one RCCL
    ALL_REDUCE per K-split stage: 2 per layer), DESIGN.md section 6 — or, at one rank,
    on one GPU without communicator: the scaling run's reference point. `steps` tokens
    from an empty KV cache, hipGraph replay, the wall time of the slowest rank.
    Collective: every rank calls it."""
    be = g.Backend(local)
    if world > 1:
        err = connect(be, world, rank)
        if err is not None:
            return {"model": model, "parallelism": f"rowsplit-{mode}{world}", "error": err}
    n_ctx = max(128, (max(steps, warmup) + 31) // 32 * 32)
    try:
        tk = Token(model, dev, 0x51A7 + rank, be, n_ctx, split=(world, rank, mode) if world > 1 else None)
    except ValueError as e:  # a split the plan cannot express (e.g. reduce mode's superblock grid)
        return {"model": model, "parallelism": f"rowsplit-{mode}{world}", "error": str(e)}
    for i in range(warmup):
        tk.dec.step(tk.tokens[i], i)
    be.synchronize()
    tk.dec.reset()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        tk.dec.step(tk.tokens[i], i)
    be.synchronize()
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el / steps * 1e3
    local_bytes = tk.bytes_per_token
    full_bytes = sum(N * (K // 256) * g.BLOCK_BYTES[typ] for st in q4km_chain(model) for _, typ, K, N in st)
    out = {"model": model, "parallelism": f"rowsplit-{mode}{world}" if world > 1 else "1 GPU", "tg_steps": steps,
           "tok_s": round(steps / el, 2), "ms_per_token": round(ms, 3),
           "weights_MB_per_token": round(full_bytes / 1e6, 1),
           "weights_MB_per_token_per_gpu": round(local_bytes / 1e6, 1),
           "token_hbm_frac": round(local_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "launches_per_token": tk.launches(),
           "collectives_per_token": tk.split.collectives_per_token() if tk.split is not None else 0}
    del tk, be
    torch.cuda.empty_cache()
    return out


def collective_side(dev, world, rank, local, barrier, n_chain=64, reps=20):
    """Per-collective cost on this job's ranks (the worksheet input of DESIGN.md §6):
    chains of `n_chain` dependent ALL_REDUCE / ALL_GATHER nodes of the decode token's
    message sizes (TinyLlama / Llama-3-70B hidden vectors: 2048 / 8192 f32), replayed from
    one hipGraph as the token's collectives are; us per collective, slowest rank.
    Collective: every rank calls it (at one rank: a 1-rank RCCL communicator)."""
    from ggml_mi355x import OP_ALL_GATHER, OP_ALL_REDUCE, make_tensor
    be = g.Backend(local)
    err = connect(be, world, rank)
    if err is not None:
        return {"error": err}
    out = {"world": world}
    st = torch.cuda.ExternalStream(be.stream)
    for label, op, n in (("all_reduce_8KB", OP_ALL_REDUCE, 2048), ("all_reduce_32KB", OP_ALL_REDUCE, 8192),
                         ("all_gather_8KB", OP_ALL_GATHER, 2048), ("all_gather_32KB", OP_ALL_GATHER, 8192)):
        if op == OP_ALL_GATHER and n % world:
            continue
        n_in = n if op == OP_ALL_REDUCE else n // world
        bufs = [torch.zeros(n, device=dev) for _ in range(n_chain + 1)]
        keep, nodes = [], []
        prev = make_tensor(g.TYPE_F32, n_in, 1, bufs[0].data_ptr())
        keep.append(prev)
        for k in range(n_chain):  # node k reads node k-1's output (its first n_in floats)
            t = make_tensor(g.TYPE_F32, n, 1, bufs[k + 1].data_ptr(), op=op, srcs=[prev])
            keep.append(t)
            nodes.append(t)
            prev = make_tensor(g.TYPE_F32, n_in, 1, bufs[k + 1].data_ptr())
            keep.append(prev)
        rc = be.graph_compute(nodes, use_graph=True)  # capture + warm-up replay
        if rc != 0:
            out[label] = {"error": rc}
            continue
        be.synchronize()
        barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            be.graph_compute(nodes, use_graph=True)
        e1.record(st)
        be.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (reps * n_chain)
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([us], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            us = float(t.item())
        out[label] = round(us, 2)
        barrier()
    del be
    torch.cuda.empty_cache()
    return out


def resolve_mode(mode, world):
    """--mode auto: one GPU decodes one token stream; at N > 1 the headline is the row split
    in the reduce schedule -- the multi-GPU path north_star names ("weight rows shard
    across the GPUs ... a single RCCL all-reduce ... >= 3.5x at 4 GPUs on the row-split
    path"), not data-parallel replicas."""
    if mode == "auto":
        return "rowsplit-reduce" if world > 1 else "replicas"
    return mode


def headline_fields(mode, world):
    """The line's scaling / parallelism for a resolved --mode (rowsplit* at N = 1 runs the
    same graph over a 1-rank RCCL communicator)."""
    if mode == "replicas":
        return {"scaling": "weak", "parallelism": f"replicas x{world}", "tokens_per_step": world}
    split_mode = "reduce" if mode == "rowsplit-reduce" else "gather"
    return {"scaling": "strong", "parallelism": f"rowsplit-{split_mode}{world}", "tokens_per_step": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--model", default="tinyllama-1.1b", choices=sorted(MODELS))
    ap.add_argument("--mode", default="auto", choices=["auto", "replicas", "rowsplit", "rowsplit-reduce"],
                    help="the headline at N GPUs: auto (default: N = 1 one token stream on one GPU; N > 1 "
                         "rowsplit-reduce, the north_star's row-split path), replicas (an independent token "
                         "stream per GPU, weak scaling), rowsplit (one token stream, the weight rows split over "
                         "the GPUs, one RCCL all-gather per stage: strong scaling) or rowsplit-reduce (one "
                         "stream, attn_output / ffn_down split along K, one RCCL all-reduce per K-split stage, "
                         "strong scaling). At N > 1 the line carries the replicas figure and both row splits of "
                         "TinyLlama and Llama-3-70B beside the headline")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-large", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--gguf", default=None,
                    help="run the chain on a real llama-architecture GGUF file's weights (Q4_K/Q5_K/Q6_K)")
    ap.add_argument("--impl", default="auto", choices=["auto", "rows", "tasks"],
                    help="auto/rows: kq_rows per stage (hipGraph replay); tasks: kq_gemv per stage")
    ap.add_argument("--no-prefill", action="store_true")
    ap.add_argument("--workload", default="token", choices=["token", "chain"],
                    help="token: the full decode graph (tg128: token i at position i of a fresh KV cache); "
                         "chain: the per-token MUL_MAT chain only")
    ap.add_argument("--no-chain", action="store_true", help="token workload: skip the matmul-chain side figure")
    ap.add_argument("--no-8b", action="store_true", help="skip the Llama-3-8B side figure (configs 3 and 5)")
    ap.add_argument("--tg", type=int, default=128, help="tokens of the tg side figure (0: skip)")
    ap.add_argument("--no-collectives", action="store_true", help="skip the per-collective RCCL timing")
    ap.add_argument("--no-device-warmup", action="store_true",
                    help="skip the ~0.3 s untimed device warm-up before the warmup steps")
    ap.add_argument("--no-70b", action="store_true",
                    help="skip the Llama-3-70B side figure (config 4: row split over the job's GPUs, 1 GPU at N = 1)")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="A/B runs only: set a library experiment knob (mi355x_debug_knob; the line records it)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args.gpus)  # exits
    if args.workload == "token" and (args.gguf or args.impl != "auto"):
        args.workload = "chain"  # the GGUF-file and kernel-A/B runs are matmul-chain modes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    mode = resolve_mode(args.mode, world)
    if mode != "replicas" and args.workload != "token":
        raise SystemExit("bench: the row split runs the decode token workload")
    if world > 1:
        # control plane only (barriers, the RCCL id, the max over ranks): gloo on the host;
        # the data path's collectives are the backend's own RCCL ALL_GATHER nodes
        import torch.distributed as dist
        dist.init_process_group("gloo")
    if os.environ.get("BENCH_ONE_DEVICE"):  # rehearsal of the multi-rank control plane on a 1-GPU box
        local = int(os.environ["BENCH_ONE_DEVICE"])
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    if not g.device_available():
        raise SystemExit("bench: no gfx950 device or libggml_mi355x.so not loadable")
    g.gemv_impl({"auto": g.GEMV_AUTO, "rows": g.GEMV_ROWS, "tasks": g.GEMV_TASKS}[args.impl])
    knobs = {}
    for kv in args.knob:
        name, val = kv.split("=", 1)
        g.debug_knob(name, float(val))
        knobs[name] = float(val)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    gguf = None
    if args.gguf:
        from ggml_mi355x.gguf import GGUFFile
        gguf = GGUFFile(args.gguf)
    rowsplit = mode != "replicas"  # (--mode rowsplit* at N = 1: the same graph, collectives over a 1-rank RCCL comm)
    split_mode = "reduce" if mode == "rowsplit-reduce" else "gather"
    comm_error = None
    if args.workload == "token":
        be = g.Backend(local)
        if rowsplit:
            comm_error = connect(be, world, rank)
            if comm_error is not None:
                # every rank saw the failure (agreed over gloo): measure replicas instead of
                # crashing the scaling run, and say so in the line
                rowsplit = False
                be = g.Backend(local)
        n_ctx = max(128, (max(args.steps, args.warmup, args.tg) + 31) // 32 * 32)
        chain = Token(args.model, dev, 0x51A7 + rank, be, n_ctx, split=(world, rank, split_mode) if rowsplit else None)
        stream = torch.cuda.ExternalStream(be.stream)
        use_graph = not args.no_graph
        pos = [0]

        def step():
            i = pos[0]
            chain.dec.step(chain.tokens[i], i, use_graph=use_graph)
            pos[0] = i + 1
    else:
        chain = Chain(args.model, dev, seed=0x51A7 + rank, gguf=gguf)
        be = g.Backend(local)
        stream = torch.cuda.ExternalStream(be.stream)
        use_graph = not args.no_graph

        def step():
            rc = be.graph_compute(chain.nodes, use_graph=use_graph)
            if rc != 0:
                raise RuntimeError(f"graph_compute failed: {rc}")

    # Device warm-up first (untimed, not a step of the run): on a fresh box the first few ms
    # of decode ran ~6 % slower than steady state (clocks leaving idle: 0.691 against
    # 0.656 ms/token in one process, gpurun_out r03c), which --warmup 5 (~3.5 ms of tokens)
    # does not cover. Decode 384 tokens from position 0 (cache reset after); then the W
    # warmup steps and the K timed steps of the contract, from an empty cache. A fixed
    # count, not a time: at N > 1 every rank must run the same collectives.
    if isinstance(chain, Token) and not args.no_device_warmup:
        for _ in range(12):  # 12 x 32 tokens (~0.25 s of TinyLlama decode)
            for i in range(min(32, chain.n_ctx)):
                chain.dec.step(chain.tokens[i], i, use_graph=use_graph)
            be.synchronize()
        chain.dec.reset()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    be.synchronize()
    if isinstance(chain, Token):  # tg128: the timed tokens start from an empty KV cache
        chain.dec.reset()
        torch.cuda.synchronize()
        pos[0] = 0
    barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # one event after every step on the launch stream (a marker packet between two graph
    # launches): the per-step spread p10/p50/p90 of the same timed steps
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step()
        evs[i].record(stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    be.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    step_ms = [(evs[i - 1] if i else ev0).elapsed_time(evs[i]) for i in range(args.steps)]
    t_max = elapsed
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t.item())
    head = headline_fields(mode if rowsplit else "replicas", world)  # (a failed communicator: replicas)
    tokens_total = args.steps * head["tokens_per_step"]
    value = tokens_total / t_max

    # per-launch kernel timing (every rank: the row split's eager steps are collective)
    per = {}
    if isinstance(chain, Token):
        chain.dec.reset()
        torch.cuda.synchronize()
        barrier()
    per, kinds = timed_kernel_stats(be, chain, tokens=4)
    tg = tg_side(chain, args.tg, barrier) if isinstance(chain, Token) and args.tg > 0 else None
    reps = None
    if isinstance(chain, Token) and rowsplit and world > 1:
        reps = replicas_side(args.model, dev, world, rank, local, barrier)
    splits = None  # N > 1: both row-split schedules of the headline model, one token stream each
    if isinstance(chain, Token) and world > 1:
        splits = {m: split_model_side(args.model, dev, world, rank, local, barrier, steps=32, warmup=4, mode=m)
                  for m in ("gather", "reduce") if not (rowsplit and m == split_mode)}
        if rowsplit:
            splits[split_mode] = "the headline"
    l70 = None
    if isinstance(chain, Token) and not args.no_70b and args.model != "llama-3-70b":
        if world > 1:
            l70 = {m: split_model_side("llama-3-70b", dev, world, rank, local, barrier, mode=m)
                   for m in ("gather", "reduce")}
        else:
            l70 = split_model_side("llama-3-70b", dev, world, rank, local, barrier)
    colls = None
    if isinstance(chain, Token) and not args.no_collectives:
        try:
            colls = collective_side(dev, world, rank, local, barrier)
        except Exception as e:  # noqa: BLE001 - a side figure; reported in the line
            colls = {"error": f"{type(e).__name__}: {e}"}

    result = None
    if rank == 0:
        # roofline of the dominant GEMV LAUNCH KIND (kernel + bytes per launch, so the q/k/v
        # and gate/up launches of one instantiation are not averaged), from per-launch
        # kernel timestamps (hipExtLaunchKernelGGL events on the launch stream)
        roof = None
        gemv = {k: v for k, v in kinds.items() if "kq_rows" in k or "kq_gemv" in k}
        if gemv:
            dom = max(gemv, key=lambda k: gemv[k]["ms"])
            d = kinds[dom]
            ach = d["bytes"] / (d["ms"] * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "kernel": d["kernel"],
                    "launch_kind": dom, "launches": d["launches"], "bytes_per_launch": d["bytes"] / d["launches"],
                    "us_per_launch": round(d["ms"] * 1e3 / d["launches"], 3)}
        if roof is not None and not rowsplit and isinstance(chain, Token):
            # the same launch kind from the committed rocprofv3 passes of this bench command:
            # graph-replayed duration (kernel trace) and HBM read (FETCH_SIZE x2, the gfx950
            # correction), per launch; frac_rocprof = the roofline at the replayed duration
            prof = os.path.join(ROOT, "profiles", "r06f_token_summary.json")
            if os.path.exists(prof):
                with open(prof) as f:
                    pk = json.load(f).get("by_kind", {}).get(roof["launch_kind"])
                if pk:
                    roof["traffic"] = round(pk["hbm_read_per_launch"], 0) if pk.get("hbm_read_per_launch") else None
                    roof["traffic_unit"] = "bytes/launch (HBM read, rocprofv3 FETCH_SIZE x2)"
                    roof["rocprof_source"] = "profiles/r06f_token_summary.json"
                    roof["rocprof_us_per_launch"] = round(pk["us_per_launch"], 3)
                    ach_r = roof["bytes_per_launch"] / (pk["us_per_launch"] * 1e-6) / 1e9
                    roof["frac_rocprof"] = round(ach_r / HBM_PEAK_GBS, 4)
        kernels = {k: {"launches": v["launches"], "us_per_launch": round(v["ms"] * 1e3 / v["launches"], 2),
                       "GBps": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1)} for k, v in per.items()}
        launch_kinds = {k: {"launches": v["launches"], "MB_per_launch": round(v["bytes"] / v["launches"] / 1e6, 3),
                            "us_per_launch": round(v["ms"] * 1e3 / v["launches"], 2),
                            "GBps": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1),
                            "frac": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                        for k, v in kinds.items() if v["bytes"] > 0}
        side = None
        if isinstance(chain, Token) and not args.no_chain and world == 1:
            side = chain_side(args.model, dev, be)
        large = None if args.no_large or world > 1 else large_gemv(dev)
        l3 = l3q5 = None
        if isinstance(chain, Token) and not args.no_8b and world == 1 and args.model != "llama-3-8b":
            l3 = model_side("llama-3-8b", dev)
            l3q5 = model_side("llama-3-8b", dev, mix="q5_k_m")  # BASELINE config 5
        prefill = None if args.no_prefill or world > 1 else prefill_chain(chain, dev)
        pp_graph = prefill_f16 = pp_graph_f16 = None
        if not args.no_prefill and world == 1:
            prefill_f16 = on_f16(prefill_chain, chain, dev)
        if isinstance(chain, Token) and not args.no_prefill and world == 1:
            pp_graph = prompt_side(chain, be)
            pp_graph_f16 = on_f16(prompt_side, chain, be)
        if prefill is not None:
            prefill["roofline"] = {"bound": "mfma", "achieved": prefill["int_TOPS"], "peak": I8_PEAK_TOPS,
                                   "unit": "TOPS (int8 dense)", "frac": round(prefill["int_TOPS"] / I8_PEAK_TOPS, 4),
                                   "mfma_pmc": "profiles/r05_prefill_mfma.md", "stall_pmc": "profiles/r06_prefill_stall.md"}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline_token(chain, args.cpu_seconds) if isinstance(chain, Token) else \
                cpu_baseline(chain, args.cpu_seconds)
        local_bytes = chain.bytes_per_token  # weight bytes one GPU streams per token
        if isinstance(chain, Token):
            executor = ("LlamaDecoder -> mi355x_backend_graph_compute: node fusion (norm/swiglu GEMV prologues, "
                        "residual/swiglu epilogues), kq_rows + kq_attn_decode" +
                        ((", RCCL ncclAllReduce per K-split stage (row split, reduce)" if split_mode == "reduce" else
                          ", RCCL ncclAllGather per stage (row split)") if rowsplit else "") + ", " +
                        ("hipGraph replay" if not args.no_graph else "eager"))
        else:
            executor = f"{'kq_gemv' if args.impl == 'tasks' else 'kq_rows'}: 1 launch per stage" + \
                ("" if args.no_graph else ", hipGraph replay")
        per_gpu_rate = value / (world if not rowsplit else 1)  # tokens/s each GPU streams its weights for
        result = {
            "metric": "tg128 tok/s + Q4_K GEMV achieved-HBM-GB/s, TinyLlama-1.1B Q4_K_M @1 GPU",
            "value": round(value, 2), "unit": "tok/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": head["scaling"],
            "vs_baseline": None, "dtype": "q4_K/q6_K x q8_K (u4/u6*i8 dot4 -> i32, f32 combine)",
            "data": (f"GGUF weights {os.path.basename(args.gguf)}; random f32 first activation" if args.gguf else
                     "synthetic (random valid K-quant blocks of the real shapes, f32 norms, random token ids)"
                     if isinstance(chain, Token) else
                     "synthetic (random valid K-quant blocks of the real shapes; random f32 activations)"),
            "config": {"workload": (f"{chain.model} Q4_K_M tg{args.steps}: full decode graph, token i at "
                                    f"position i of a fresh f16 KV cache" if isinstance(chain, Token) else
                                    f"{chain.model} Q4_K_M decode matmul chain (tg, 1 token/step)"),
                       "weights_MB_per_token": round(local_bytes * (world if rowsplit else 1) / 1e6, 1),
                       "weights_MB_per_token_per_gpu": round(local_bytes / 1e6, 1),
                       "stages_per_token": chain.launches(),
                       "executor": executor,
                       "parallelism": head["parallelism"],
                       "hipgraph": not args.no_graph},
            "gpu_ms_per_step": round(gpu_ms / args.steps, 4),
            "step_ms": spread(step_ms),
            "effective_GBps": round(per_gpu_rate * local_bytes / 1e9, 1),
            # the whole token (every launch, gap and gather included) against the HBM roofline, per GPU
            "token_hbm_frac": round(per_gpu_rate * local_bytes / 1e9 / HBM_PEAK_GBS, 4),
            "roofline": roof,
            "kernels": kernels, "launch_kinds": launch_kinds,
            "tg128": tg,
            "gemv_large": large,
            "prefill_pp512": prefill,
            "pp512": pp_graph,
            "prefill_pp512_f16": prefill_f16,
            "pp512_f16": pp_graph_f16,
            "matmul_chain": side,
            "llama3_8b": l3,
            "llama3_8b_q5_k_m": l3q5,
            "llama3_70b": l70,
            "replicas": reps,
            "rowsplit": splits,
            "collectives_us": colls,
            "rowsplit_error": comm_error,
            "debug_knobs": knobs or None,
            "rehearsal": ("BENCH_ONE_DEVICE: all ranks on one GPU, collectives emulated (loopback, no data "
                          "exchanged): fields and control plane only, not a measurement"
                          if os.environ.get("BENCH_ONE_DEVICE") and world > 1 else None),
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
