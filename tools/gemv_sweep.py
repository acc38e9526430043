"""GEMV microbenchmark: achieved algorithmic GB/s per shape/type, kernel timestamps
from the library's launch-timing hook (hipExtLaunchKernelGGL events). Weight buffers
rotate over > 600 MB so the 256 MB Infinity Cache cannot serve them."""
import json
import os
import subprocess
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

SHAPES = [("tl q/o", 12, 2048, 2048), ("tl qkv-fused", 12, 2048, 2560), ("tl gate", 12, 2048, 5632),
          ("tl down", 12, 5632, 2048), ("tl out q6", 14, 2048, 32000), ("l3 up", 12, 4096, 14336),
          ("l3 down", 12, 14336, 4096), ("70b down", 12, 28672, 8192), ("l3 q6 down", 14, 14336, 4096)]


def run(reps=20):
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    out = []
    for label, typ, K, N in SHAPES:
        nbytes = N * (K // 256) * g.BLOCK_BYTES[typ]
        nbuf = max(2, int(np.ceil(640e6 / nbytes)))
        ws = [random_kquant(typ, N, K, gen, dev) for _ in range(nbuf)]
        x = torch.randn(1, K, device=dev, generator=gen)
        y = torch.empty(1, N, device=dev)
        for w in ws:
            g.mul_mat(typ, w, K, x, out=y)
        g.timing_enable(True)
        for r in range(reps):
            g.mul_mat(typ, ws[r % nbuf], K, x, out=y)
        rows = g.timing_read()
        g.timing_enable(False)
        per_call = len(rows) // reps  # 2 launches (quantize + GEMV) above K = 8192
        ms = np.array([sum(r[2] for r in rows[i * per_call:(i + 1) * per_call]) for i in range(reps)])
        b = nbytes + K * 4 + N * 4  # algorithmic: weights + f32 activation + f32 output
        med = float(np.median(ms))
        out.append({"shape": label, "type": typ, "K": K, "N": N, "kernel": "+".join(r[0] for r in rows[:per_call]),
                    "MB": round(b / 1e6, 2), "us": round(med * 1e3, 2), "GBps": round(b / (med * 1e-3) / 1e9, 1)})
        del ws
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        sys.argv = sys.argv[:1]
        print(json.dumps(run()))
        sys.exit(0)
    modes = sys.argv[1:] or ["auto", "prologue"]
    for mode in modes:
        env = dict(os.environ)
        for kv in mode.split(":"):  # generic overrides: "pre0=0", "lib=path", combined with ':'
            if kv.startswith("pre0="):
                env["MI355X_GEMV_PRE0"] = kv[5:]
            elif kv.startswith("bal="):
                env["MI355X_GEMV_BAL"] = kv[4:]
            elif kv.startswith("prio="):
                env["MI355X_GEMV_PRIO"] = kv[5:]
            elif kv.startswith("pf="):
                env["MI355X_GEMV_PF"] = kv[3:]
            elif kv.startswith("wpc="):
                env["MI355X_GEMV_WPC"] = kv[4:]
            elif kv.startswith("lib="):
                env["MI355X_LIB"] = os.path.join(ROOT, kv[4:])
        if mode in ("prologue", "empty", "quantonly", "dmaonly"):  # diagnostics: compile-time build only
            env.setdefault("MI355X_LIB", os.path.join(ROOT, "ggml-neon-opt_amd/lib/variants/libdiag.so"))
        if mode == "prologue":
            env["MI355X_GEMV_DIAG"] = "1"
        elif mode == "empty":
            env["MI355X_GEMV_DIAG"] = "2"
        elif mode == "quantonly":
            env["MI355X_GEMV_DIAG"] = "5"
        elif mode == "dmaonly":
            env["MI355X_GEMV_DIAG"] = "8"
        elif mode == "tasks":
            env["MI355X_GEMV_IMPL"] = "tasks"
        elif mode.startswith("ring"):
            env["MI355X_GEMV_RING"] = mode[4:]
        elif mode != "auto" and "=" not in mode:
            env["MI355X_GEMV_MODE"] = mode
        r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            sys.exit(r.returncode)
        for row in json.loads(r.stdout.strip().splitlines()[-1]):
            print(f"{mode:6s} {row['shape']:14s} K={row['K']:6d} N={row['N']:6d} {row['MB']:8.2f} MB "
                  f"{row['us']:8.2f} us {row['GBps']:8.1f} GB/s  {row['kernel']}")
