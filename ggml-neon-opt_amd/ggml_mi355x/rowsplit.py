"""Row split (tensor parallel) of the decode token over one process per GPU.

Every weight row's dot product is independent, so rank r of a
world of G owns a contiguous slice of each matrix's rows, computes it with the
unchanged single-GPU kernels (bit-identical per row) and the slices are combined
by one ALL_GATHER node per stage (RCCL ncclAllGather on the backend stream, in the
token's hipGraph; kq_backend.hip). An all_reduce(sum) over zero-padded slices
would give the same bits (x + 0 = x) at G times the bytes. Over xGMI the per-stage
messages (1-128 KB) are latency-bound: the split pays for large matrices
(Llama-3-70B), not for TinyLlama.
"""
from __future__ import annotations

import math


class TokenSplit:
    """Row split of one llama decode token over `world` GPUs (rank `rank`'s share).

    The reference splits each MUL_MAT's weight rows over its threads, every thread
    reading the same quantized activation (ggml_compute_forward_mul_mat's chunks,
    README.md:125-131, 136/156); here the same rows go to different GPUs:
      * attn_q rows of the rank's query heads [q0, q1) (nh / world heads each), attn_k
        / attn_v rows of the KV heads those query heads read (GQA group h // (nh/nkv));
        when world > n_head_kv, world/n_head_kv ranks hold the same KV head and each
        keeps its own copy of that head's cache rows (identical bits);
      * the attention of the rank's heads runs locally, on its KV-cache slice;
      * attn_output, ffn_down: rows [r*E/world, (r+1)*E/world) with the residual ADD of
        the same rows; ffn_gate / ffn_up: rows of F/world with the SWIGLU of those rows;
        output: V/world rows;
      * after every stage the slices are ALL_GATHERed (rank order = row order), so the
        next stage reads the full activation: 4 gathers per layer + 1 for the logits.
    Every row's dot product and every head's attention is the 1-GPU computation, so
    the gathered vectors are bit-identical to the single-GPU token (and to the oracle).
    """

    def __init__(self, hp: dict, world: int, rank: int):
        nh, nkv = hp["n_head"], hp["n_head_kv"]
        E, F, V = hp["n_embd"], hp["n_ff"], hp["n_vocab"]
        if world < 1 or not 0 <= rank < world:
            raise ValueError("bad world/rank")
        if nh % world:
            raise ValueError(f"n_head {nh} not divisible by world {world}")
        if nkv % world and world % nkv:
            raise ValueError(f"n_head_kv {nkv} and world {world}: one must divide the other")
        for n, what in ((E, "n_embd"), (F, "n_ff"), (V, "n_vocab")):
            if n % world:
                raise ValueError(f"{what} {n} not divisible by world {world}")
        self.hp, self.world, self.rank = hp, world, rank
        hd = hp["head_dim"]
        group = nh // nkv
        self.q0, self.q1 = rank * nh // world, (rank + 1) * nh // world
        self.kv0, self.kv1 = self.q0 // group, (self.q1 - 1) // group + 1
        self.n_head, self.n_head_kv = self.q1 - self.q0, self.kv1 - self.kv0
        self.rows = {
            "attn_q": (self.q0 * hd, self.q1 * hd),
            "attn_k": (self.kv0 * hd, self.kv1 * hd),
            "attn_v": (self.kv0 * hd, self.kv1 * hd),
            "attn_output": (rank * E // world, (rank + 1) * E // world),
            "ffn_gate": (rank * F // world, (rank + 1) * F // world),
            "ffn_up": (rank * F // world, (rank + 1) * F // world),
            "ffn_down": (rank * E // world, (rank + 1) * E // world),
            "output": (rank * V // world, (rank + 1) * V // world),
        }

    def rows_of(self, name: str):
        """Row range of a weight by its GGUF name (blk.N.attn_q, output, ...)."""
        return self.rows[name.split(".")[-1]]

    def slice_weights(self, weights: dict) -> dict:
        """The rank's share of a full weight dict (LlamaDecoder layout): K-quant
        matrices sliced by rows, everything else (token_embd, norms) replicated."""
        out = {}
        for k, v in weights.items():
            base = k.split(".")[-1]
            if isinstance(v, tuple) and base in self.rows:
                r0, r1 = self.rows[base]
                out[k] = (v[0], v[1][r0:r1].contiguous() if hasattr(v[1], "contiguous") else v[1][r0:r1])
            else:
                out[k] = v
        return out
