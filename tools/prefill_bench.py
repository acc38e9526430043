"""Prefill (M = 512) K-quant matmul timing: kq_quantize_q8L + kq_mmq per shape,
launch-timing hook (hipExtLaunchKernelGGL events). Reports integer TOPS (2*N*K*M)
against the int8 dense MFMA peak (~5 POPS, MI355X_MICROARCH.md)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()  # the MI355X_* A/B environment -> explicit library calls

from bench import random_kquant  # noqa: E402

SHAPES = [("l3 q/o", 12, 4096, 4096), ("l3 up", 12, 4096, 14336), ("l3 down", 12, 14336, 4096),
          ("tl gate", 12, 2048, 5632), ("l3 v q5", 13, 4096, 1024), ("tl out q6", 14, 2048, 32000),
          ("l3 down q6", 14, 14336, 4096), ("l3 q/o q5", 13, 4096, 4096), ("l3 up q5", 13, 4096, 14336),
          ("l3 down q5", 13, 14336, 4096), ("tl q/o", 12, 2048, 2048), ("tl gate+up", 12, 2048, 11264),
          ("tl down", 12, 5632, 2048), ("tl down q6", 14, 5632, 2048), ("tl v q6", 14, 2048, 256)]


def main(M=512, reps=10, only=None):
    dev = torch.device("cuda:0")
    f16 = os.environ.get("MI355X_PREFILL") == "f16"
    if f16:
        g.prefill_precision(g.PREFILL_F16)
    peak = 2.5e15 if f16 else 5e15
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    for label, typ, K, N in SHAPES:
        if only and typ not in only:
            continue
        if os.environ.get("PREFILL_SHAPES") and not label.startswith(os.environ["PREFILL_SHAPES"]):
            continue
        w = random_kquant(typ, N, K, gen, dev)
        x = torch.randn(M, K, device=dev, generator=gen)
        y = torch.empty(M, N, device=dev)
        g.mul_mat(typ, w, K, x, out=y)
        g.timing_enable(True)
        for _ in range(reps):
            g.mul_mat(typ, w, K, x, out=y)
        rows = g.timing_read()
        g.timing_enable(False)
        per = len(rows) // reps
        names = [r[0] for r in rows[:per]]
        tot = np.median([sum(r[2] for r in rows[i * per:(i + 1) * per]) for i in range(reps)])
        mm = np.median([sum(r[2] for r in rows[i * per:(i + 1) * per] if "quantize" not in r[0]) for i in range(reps)])
        ops = 2.0 * N * K * M
        print(f"{label:8s} K={K:6d} N={N:6d} M={M}: total {tot * 1e3:8.1f} us ({ops / (tot * 1e-3) / 1e12:7.1f} TOPS), "
              f"gemm {mm * 1e3:8.1f} us ({ops / (mm * 1e-3) / 1e12:7.1f} TOPS, {ops / (mm * 1e-3) / peak * 100:5.1f} % of {peak / 1e15:.1f} P) "
              f"{'+'.join(names)}", flush=True)


if __name__ == "__main__":
    main(only=[int(t) for t in os.environ["PREFILL_TYPES"].split(",")] if os.environ.get("PREFILL_TYPES") else None)
