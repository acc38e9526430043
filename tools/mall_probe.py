"""Does a decode GEMV run faster when its weights are already in the 256 MB Infinity
Cache (MALL)? Times kq_rows on the TinyLlama shapes three ways:
  cold      weight buffers rotated over > 600 MB (what the token sees today)
  hot       the same buffer every call (MALL/L2 resident upper bound)
  prefetch  rotated, but a plain read of the buffer (torch sum) runs just before
            the GEMV, as a side-stream prefetcher would leave it
  cold_fx / hot_fx  as cold / hot, but the activation is rewritten by another kernel just
            before each GEMV (as in the token: x is the previous launch's output), so only
            the weights' residency differs between the two
Only the GEMV launches are timed (library launch-timing hook)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from bench import random_kquant  # noqa: E402

SHAPES = [("tl q/o", 12, 2048, 2048), ("tl gate", 12, 2048, 5632), ("tl down", 12, 5632, 2048),
          ("tl gate+up", 12, 2048, 11264), ("tl out q6", 14, 2048, 32000), ("l3 up", 12, 4096, 14336)]


def main(reps=30):
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    for label, typ, K, N in SHAPES:
        nbytes = N * (K // 256) * g.BLOCK_BYTES[typ]
        nbuf = max(2, int(np.ceil(640e6 / nbytes)))
        ws = [random_kquant(typ, N, K, gen, dev) for _ in range(nbuf)]
        x = torch.randn(1, K, device=dev, generator=gen)
        y = torch.empty(1, N, device=dev)
        sink = torch.zeros(1, dtype=torch.int64, device=dev)
        res = {}
        for mode in ("cold", "hot", "prefetch", "cold_fx", "hot_fx"):
            for w in ws[:4]:
                g.mul_mat(typ, w, K, x, out=y)
            torch.cuda.synchronize()
            g.timing_enable(True)
            for r in range(reps):
                w = ws[0] if mode.startswith("hot") else ws[r % nbuf]
                if mode.endswith("_fx"):
                    x.mul_(1.0)  # the activation freshly written by another kernel
                if mode == "prefetch":
                    sink += w.view(torch.int32).sum(dtype=torch.int64)
                g.mul_mat(typ, w, K, x, out=y)
            torch.cuda.synchronize()
            rows = g.timing_read()
            g.timing_enable(False)
            us = [r[2] * 1e3 for r in rows if r[0].startswith("kq::kq_rows")]
            res[mode] = float(np.median(us))
        mb = nbytes / 1e6
        print(f"{label:12s} {mb:7.2f} MB  " + "  ".join(f"{m} {v:6.2f} us ({mb / v:6.0f} GB/s)" for m, v in res.items()),
              flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
