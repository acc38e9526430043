"""Row split (tensor parallel) of the decode token over one process per GPU.

Two exchange schedules (TokenSplit mode):
  * "gather" (bit-exact): every matrix split by output rows, one ALL_GATHER node after
    each stage, 4 per layer + 1;
  * "reduce" (the north_star's all-reduce, the Megatron pairing of SURVEY.md §8e): q/k/v
    and gate/up split by output rows (heads / ffn rows), attn_output and ffn_down split
    along K at 256-element superblock boundaries (the rank's heads / ffn rows ARE its K
    slice), one ALL_REDUCE(sum) on their partial outputs: 2 per layer + 1 gather of the
    logits. Integer parts and each rank's fp32 chain over its superblocks are exact; the
    sum over ranks re-associates the chain (SURVEY.md §8c's fp32 bound).

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

    def __init__(self, hp: dict, world: int, rank: int, mode: str = "gather"):
        nh, nkv = hp["n_head"], hp["n_head_kv"]
        E, F, V = hp["n_embd"], hp["n_ff"], hp["n_vocab"]
        if world < 1 or not 0 <= rank < world:
            raise ValueError("bad world/rank")
        if mode not in ("gather", "reduce"):
            raise ValueError(f"mode {mode!r}: 'gather' or 'reduce'")
        self.mode = mode
        if nh % world:
            raise ValueError(f"n_head {nh} not divisible by world {world}")
        if nkv % world and world % nkv:
            raise ValueError(f"n_head_kv {nkv} and world {world}: one must divide the other")
        for n, what in ((E, "n_embd"), (F, "n_ff"), (V, "n_vocab")) if mode == "gather" else ((V, "n_vocab"),):
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
        # K-split ("reduce") mode: superblock columns of the K-split matrices
        self.cols = {}
        if mode == "reduce":
            qk = (self.q1 - self.q0) * hd  # the rank's attention output = its K slice of attn_output
            if (self.q0 * hd) % 256 or qk % 256:
                raise ValueError(f"reduce mode: the rank's {self.q1 - self.q0} heads x {hd} are not whole "
                                 f"256-element superblocks of attn_output's K")
            if F % 256:
                raise ValueError(f"reduce mode: n_ff {F} is not whole superblocks")
            nbf = F // 256
            if nbf < world:
                raise ValueError(f"reduce mode: {nbf} ffn superblocks < world {world}")
            f0, f1 = rank * nbf // world, (rank + 1) * nbf // world  # (uneven when world does not divide)
            self.cols = {"attn_output": (self.q0 * hd // 256, self.q1 * hd // 256), "ffn_down": (f0, f1)}
            self.rows["attn_output"] = (0, E)
            self.rows["ffn_down"] = (0, E)
            self.rows["ffn_gate"] = self.rows["ffn_up"] = (256 * f0, 256 * f1)

    def rows_of(self, name: str):
        """Row range of a weight by its GGUF name (blk.N.attn_q, output, ...)."""
        return self.rows[name.split(".")[-1]]

    def slice_weights(self, weights: dict) -> dict:
        """The rank's share of a full weight dict (LlamaDecoder layout): K-quant
        matrices sliced by rows (and, in reduce mode, attn_output / ffn_down by superblock
        columns: the GGUF bytes of those superblocks, unchanged), everything else
        (token_embd, norms) replicated."""
        from . import BLOCK_BYTES
        out = {}
        for k, v in weights.items():
            base = k.split(".")[-1]
            if isinstance(v, tuple) and base in self.rows:
                r0, r1 = self.rows[base]
                w = v[1][r0:r1]
                if base in self.cols:
                    c0, c1 = self.cols[base]
                    B = BLOCK_BYTES[v[0]]
                    w = w[:, c0 * B:c1 * B]
                out[k] = (v[0], w.contiguous() if hasattr(w, "contiguous") else w.copy())
            else:
                out[k] = v
        return out

    def collectives_per_token(self) -> int:
        """Exchange nodes of one decode token: 4 ALL_GATHERs per layer + 1 (gather mode) or
        2 ALL_REDUCEs per layer + 1 ALL_GATHER of the logits (reduce mode)."""
        L = self.hp["n_layer"]
        return (4 * L + 1) if self.mode == "gather" else (2 * L + 1)
