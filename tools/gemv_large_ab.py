"""bench.large_gemv under the current environment (A/B of decode-GEMV knobs)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()  # the MI355X_* A/B environment -> explicit library calls


out = bench.large_gemv(torch.device("cuda:0"))
for k, v in out.items():
    print(f"{k:42s} {v['us_median']:8.2f} us  frac {v['frac_median']:.3f}  stream {v['stream_us']:8.2f} us "
          f"({v['stream_frac']:.3f})  of ceiling {v['of_stream_ceiling']:.3f}  {v['kernel']}")
