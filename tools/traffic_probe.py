"""Where a decode GEMV's HBM read beyond its weights comes from (diagnostic, run under
`rocprofv3 --pmc FETCH_SIZE`): single kq_rows launches (mi355x_mul_mat, M = 1, x 16-B
aligned so the activation is quantized inside the GEMV) of one type and K at growing N,
REPS launches per shape, in this order; tools/traffic_fit.py fits FETCH = a + b * bytes
per shape group: `b` > 1 is stream over-fetch, `a` the per-launch fixed read (the
activation per XCD, code, kernel arguments)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from bench import random_kquant  # noqa: E402

REPS = 6
SHAPES = [(g.TYPE_Q4_K, 2048, n) for n in (256, 1024, 2048, 4096, 8192, 16384, 32768)] + \
         [(g.TYPE_Q6_K, 2048, n) for n in (256, 1024, 4096, 16384)] + \
         [(g.TYPE_Q4_K, 5632, n) for n in (512, 2048, 8192)]


def main():
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    for typ, K, N in SHAPES:
        w = random_kquant(typ, N, K, gen, dev, rms_keep=True)
        x = torch.randn(K, device=dev, generator=gen)
        y = torch.empty(1, N, device=dev)
        for _ in range(REPS):
            g.mul_mat(typ, w, K, x, out=y)
        torch.cuda.synchronize()
        print(f"shape type {typ} K {K} N {N} bytes {w.numel()} reps {REPS}", flush=True)


if __name__ == "__main__":
    main()
