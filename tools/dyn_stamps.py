"""Round 6: per-wave stamps of the static kq_rows and the claimed-row kq_rows_dyn on the
large shapes (diagnostic build libdiag.so): prologue, loop, loop-end spread by wave index
(age class on its SIMD) and, for kq_rows_dyn, the units each wave took."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
os.environ.setdefault("MI355X_LIB", os.path.join(ROOT, "ggml-neon-opt_amd/lib/variants/libdiag.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
from bench import random_kquant  # noqa: E402

SHAPES = [("l3 up", 12, 4096, 14336), ("70b down", 12, 28672, 8192), ("l3 out q6", 14, 4096, 128256)]
dev = torch.device("cuda:0")
gen = torch.Generator(device=dev)
gen.manual_seed(3)
buf = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
for label, typ, K, N in SHAPES:
    ws = [random_kquant(typ, N, K, gen, dev) for _ in range(max(2, int(600e6 // (N * K // 256 * 144))))]
    x = torch.randn(1, K, device=dev)
    y = torch.empty(1, N, device=dev)
    for dyn in (0.0, 2.5):
        g.debug_knob("GEMV_DYN", dyn)
        for w in ws:
            g.mul_mat(typ, w, K, x, out=y)
        rows = []
        for r in range(4):
            buf.zero_()
            torch.cuda.synchronize()
            torch.cuda._sleep(20_000_000)
            for i in range(40):
                if i == 39:
                    g.lib().mi355x_diag_stamps(buf.data_ptr(), buf.numel() * 8)
                g.mul_mat(typ, ws[(r * 40 + i) % len(ws)], K, x, out=y)
            torch.cuda.synchronize()
            g.lib().mi355x_diag_stamps(None, 0)
            st = buf.cpu().numpy().astype(np.int64).reshape(-1, 8)[:256 * 12]
            idx = np.nonzero(st[:, 0])[0]
            st = st[idx]
            wave = idx % 12
            t0 = st[:, 0].min()
            rel = (st[:, :7] - t0) * 10 / 1000.0
            pro = np.median(rel[:, 1] - rel[:, 0])
            lend = rel[:, 2]
            cls = [np.median(lend[(wave >= 4 * c) & (wave < 4 * c + 4)]) for c in range(3)]
            units = [np.mean(st[(wave >= 4 * c) & (wave < 4 * c + 4), 7]) for c in range(3)] if dyn else [0, 0, 0]
            rows.append((pro, np.median(lend), lend.max(), rel[:, 3].max(), *cls, *units))
        a = np.array(rows)[1:].mean(0)
        print(f"{label:10s} {'dyn' if dyn else 'static':6s} prologue {a[0]:5.2f} loop-end med/max {a[1]:6.2f}/{a[2]:6.2f} "
              f"end {a[3]:6.2f} | loop end by wave class {a[4]:6.2f} {a[5]:6.2f} {a[6]:6.2f} | units {a[7]:4.2f} {a[8]:4.2f} {a[9]:4.2f}",
              flush=True)
    g.debug_knob("GEMV_DYN")
