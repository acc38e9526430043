"""Cost of the fused GEMV prologues / epilogue (diagnostic): TinyLlama-shaped kq_rows
launches with no prologue, the rms_norm+mul prologue, the swiglu prologue, and the
residual epilogue. Median per-launch kernel time from the library's launch events,
weights rotated over > 600 MB (no Infinity Cache hits)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from bench import random_kquant  # noqa: E402


def main(reps=40):
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    cases = [("o 2048->2048 q4", 2048, [(12, 2048)]), ("gate+up 2048->2x5632 q4", 2048, [(12, 5632), (12, 5632)]),
             ("down 5632->2048 q4", 5632, [(12, 2048)]), ("down 5632->2048 q6", 5632, [(14, 2048)])]
    for label, K, mats in cases:
        nbytes = sum(N * (K // 256) * g.BLOCK_BYTES[t] for t, N in mats)
        nbuf = max(2, int(np.ceil(640e6 / nbytes)))
        wsets = [[random_kquant(t, N, K, gen, dev) for t, N in mats] for _ in range(nbuf)]
        x = torch.randn(K, device=dev, generator=gen)
        x2 = torch.rand(K, device=dev, generator=gen) + 0.5
        ys = [torch.empty(N, device=dev) for _, N in mats]
        res = [torch.randn(N, device=dev, generator=gen) for _, N in mats]
        for pname, pro in (("none", g.PRO_NONE), ("norm", g.PRO_RMS_NORM), ("swiglu", g.PRO_SWIGLU)):
            for use_res in (False, True):
                def call(i):
                    g.gemv_fused_ext([(t, w, y) for (t, _), w, y in zip(mats, wsets[i % nbuf], ys)], x, prologue=pro,
                                     x2=None if pro == g.PRO_NONE else x2, eps=1e-5,
                                     residual=res if use_res else None)
                for i in range(nbuf):
                    call(i)
                g.timing_enable(True)
                for i in range(reps):
                    call(i)
                rows = g.timing_read()
                g.timing_enable(False)
                us = np.median([r[2] for r in rows]) * 1e3
                print(f"{label:26s} pro={pname:6s} res={int(use_res)} {rows[0][0]:28s} {us:6.2f} us "
                      f"{nbytes / (us * 1e-6) / 1e9:7.1f} GB/s", flush=True)
        del wsets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
