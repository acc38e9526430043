"""Per-launch overhead on the GPU timeline: back-to-back launches of (a) the GEMV
kernel in its 'empty' diagnostic mode, (b) a tiny torch kernel, eager and inside a
CUDA/HIP graph. Prints microseconds per launch (torch events around N launches)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()  # the MI355X_* A/B environment -> explicit library calls

from bench import random_kquant  # noqa: E402


def timeit(fn, n=2000):
    s = torch.cuda.current_stream()
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def graphed(fn, reps=100):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    return lambda: gr.replay(), reps


def main():
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    out = {}
    t = torch.zeros(1, device=dev)
    out["torch add_ eager"] = timeit(lambda: t.add_(1.0))
    f, reps = graphed(lambda: t.add_(1.0))
    out["torch add_ graph"] = timeit(f, 50) / reps
    for label, K, N in (("gemv tl q 2048x2048", 2048, 2048), ("gemv tl 8 rows", 2048, 8)):
        w = random_kquant(g.TYPE_Q4_K, N, K, gen, dev)
        x = torch.randn(1, K, device=dev)
        y = torch.empty(1, N, device=dev)
        fn = lambda: g.mul_mat(g.TYPE_Q4_K, w, K, x, out=y)  # noqa: E731
        out[label + " eager"] = timeit(fn)
        f, reps = graphed(fn)
        out[label + " graph"] = timeit(f, 50) / reps
    for k, v in out.items():
        print(f"{os.environ.get('MI355X_GEMV_DIAG', '0'):>2s} {k:40s} {v:8.2f} us/launch")


if __name__ == "__main__":
    main()
