"""Row-split (tensor-parallel) GEMV over one process per GPU.

Every weight row's dot product is independent, so rank r of a
world of G owns a contiguous, 8-row-aligned slice of each matrix's rows (the
GEMV kernel's task granularity), computes it with the unchanged single-GPU
kernel (bit-identical per row) and the slices are combined with ONE collective
per stage: all_gather of the padded slices (N/G floats per rank), or
all_reduce(sum) over a zero-padded full-length vector (x + 0 = x, still exact).
Over RCCL/xGMI these per-stage messages (1-112 KB) are latency-bound, which is
why the row split only pays for large matrices (multi-GPU).
"""
from __future__ import annotations

import math


def shard_rows(n_rows: int, world: int, rank: int, align: int = 8):
    """Contiguous row slice of `rank`: (r0, r1, per) with per = padded slice size."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    per = int(math.ceil(math.ceil(n_rows / world) / align) * align) if n_rows else 0
    r0 = min(rank * per, n_rows)
    r1 = min(r0 + per, n_rows)
    return r0, r1, per


class StageGather:
    """Packs the local slices of the matrices of one fused stage into one buffer and
    reassembles the full outputs after one collective."""

    def __init__(self, n_rows_list, world, rank, device, dtype=None, collective="all_gather", group=None):
        import torch
        self.world, self.rank, self.group = world, rank, group
        self.collective = collective
        self.n_rows = list(n_rows_list)
        self.shards = [shard_rows(n, world, rank) for n in self.n_rows]
        self.per = [s[2] for s in self.shards]
        self.offs = [sum(self.per[:i]) for i in range(len(self.per))]
        self.total = sum(self.per)
        dtype = dtype or torch.float32
        self.local = torch.zeros(self.total, device=device, dtype=dtype)
        if collective == "all_gather":
            self.gathered = torch.zeros(world * self.total, device=device, dtype=dtype)
        elif collective == "all_reduce":
            self.full = torch.zeros(world * self.total, device=device, dtype=dtype)
        else:
            raise ValueError(collective)

    def local_view(self, i):
        """The slice of the packed local buffer that matrix i's GEMV writes."""
        r0, r1, _ = self.shards[i]
        return self.local[self.offs[i]:self.offs[i] + (r1 - r0)]

    def exchange(self):
        import torch.distributed as dist
        if self.collective == "all_gather":
            if self.world == 1:
                self.gathered.copy_(self.local)
            elif dist.get_backend(self.group) == "gloo":
                parts = list(self.gathered.chunk(self.world))
                dist.all_gather(parts, self.local, group=self.group)
            else:
                dist.all_gather_into_tensor(self.gathered, self.local, group=self.group)
        else:
            self.full.zero_()
            self.full[self.rank * self.total:(self.rank + 1) * self.total].copy_(self.local)
            if self.world > 1:
                dist.all_reduce(self.full, group=self.group)

    def output(self, i):
        """Full output of matrix i (length n_rows[i]) after exchange()."""
        buf = self.gathered if self.collective == "all_gather" else self.full
        v = buf.view(self.world, self.total)[:, self.offs[i]:self.offs[i] + self.per[i]]
        return v.reshape(-1)[:self.n_rows[i]]


class RowSplitChain:
    """A model's per-token GEMV chain with every matrix row-split over the ranks;
    one collective per stage (bench.py --mode rowsplit)."""

    def __init__(self, model, device, rank, world, make_chain, collective="all_gather"):
        import ggml_mi355x as g
        self.g = g
        self.chain = make_chain(model, device, seed=0x51A7, row_shard=lambda n: shard_rows(n, world, rank)[:2])
        self.gathers = []
        for stage in self.chain.stages:
            self.gathers.append(StageGather([n for _, _, _, n in stage], world, rank, device, collective=collective))

    def step(self):
        g = self.g
        for si, stage in enumerate(self.chain.stages):
            sg = self.gathers[si]
            mats = [(typ, w, sg.local_view(i)) for i, (typ, w) in enumerate(self.chain.w[si])]
            g.gemv_fused(mats, self.chain.x[si])
            sg.exchange()
