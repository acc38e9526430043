"""In-kernel timeline of one GEMV launch (diagnostic build path): per-wave
s_memrealtime stamps at entry / after prologue / after main loop / exit."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
# stamps exist only in the diagnostic build:
#   make -C ggml-neon-opt_amd variant NAME=diag VFLAGS="-DKQ_ROWS_DIAG=1 -DKQ_GEMV_DIAG=1"
os.environ.setdefault("MI355X_LIB", os.path.join(ROOT, "ggml-neon-opt_amd/lib/variants/libdiag.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggml_mi355x as g  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()  # the MI355X_* A/B environment -> explicit library calls

from bench import random_kquant  # noqa: E402

SHAPES = [("tl q", 12, 2048, 2048), ("tl 8rows", 12, 2048, 8), ("tl gate+up", 12, 2048, 11264),
          ("tl down", 12, 5632, 2048), ("tl out q6", 14, 2048, 32000), ("l3 up", 12, 4096, 14336),
          ("70b down", 12, 28672, 8192)]


PRO = os.environ.get("STAMPS_PRO", "none")  # none | norm | swiglu: fused prologue (kq_rows only)
# STAMPS_SLEEP=1: a spin kernel (torch.cuda._sleep, ~10 ms) ahead of the burst, so the burst's
# launches queue behind it and run back to back, as in the graph-replayed token. Without it
# the GPU idles between the eager launches of a short kernel and its XCDs wake in turn
# (tools/xcd_skew.hip: 0.1 .. 1.4 us apart), which the entry stamps then show.
SLEEP = os.environ.get("STAMPS_SLEEP", "0") == "1"


def main(impl):
    g.gemv_impl(impl)
    pro = {"none": g.PRO_NONE, "norm": g.PRO_RMS_NORM, "swiglu": g.PRO_SWIGLU}[PRO]
    tag = ("rows " if impl == 0 else "tasks") + ("" if PRO == "none" else "/" + PRO)
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    buf = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
    for label, typ, K, N in SHAPES:
        ws = [random_kquant(typ, N, K, gen, dev) for _ in range(max(2, int(600e6 // (N * K // 256 * 144))))]
        x = torch.randn(1, K, device=dev)
        x2 = torch.rand(K, device=dev) + 0.5
        y = torch.empty(1, N, device=dev)

        def mm(w):
            if pro == g.PRO_NONE:
                g.mul_mat(typ, w, K, x, out=y)
            else:
                g.gemv_fused_ext([(typ, w, y[0])], x[0], prologue=pro, x2=x2, eps=1e-5)
        for w in ws:
            mm(w)
        res = []
        for r in range(5):
            buf.zero_()
            torch.cuda.synchronize()
            if SLEEP:
                torch.cuda._sleep(20_000_000)
            # warm the clocks with a burst; stamps of the LAST launch of the burst survive
            for i in range(60):
                if i == 59:
                    g.lib().mi355x_diag_stamps(buf.data_ptr(), buf.numel() * 8)
                mm(ws[(r * 60 + i) % len(ws)])
            torch.cuda.synchronize()
            g.lib().mi355x_diag_stamps(None, 0)
            st = buf.cpu().numpy().astype(np.int64).reshape(-1, 8)
            if os.environ.get("STAMPS_DUMP") and r == 4:  # raw per-(block, wave) rows for offline analysis
                np.save(os.environ["STAMPS_DUMP"] + "_" + label.replace(" ", "_") + ".npy", st[:256 * 12])
            st = st[st[:, 0] != 0]
            t0 = st[:, 0].min()
            rel = (st - t0) * 10 / 1000.0  # 100 MHz ticks -> us
            med = lambda v: float(np.median(v))  # noqa: E731
            if impl == 0:  # kq_rows: [entry, ring filled, loop end, exit, x landed, x quantized, first step]
                ok = rel[:, 4] > 0
                res.append((len(st), rel[:, 0].max(), med(rel[ok, 4] - rel[ok, 0]), med(rel[ok, 5] - rel[ok, 4]),
                            med(rel[:, 1] - rel[:, 5]), med(rel[ok, 6] - rel[ok, 1]),
                            med(rel[:, 1] - rel[:, 0]), med(rel[:, 2] - rel[:, 1]), np.max(rel[:, 2] - rel[:, 1]),
                            rel[:, 3].max(), rel[:, 2].max(), med(rel[:, 2])))
                continue
            res.append((len(st), rel[:, 0].max(), med(rel[:, 4] - rel[:, 0]), med(rel[:, 5] - rel[:, 4]),
                        med(rel[:, 6] - rel[:, 5]), med(rel[:, 1] - rel[:, 6]),
                        med(rel[:, 1] - rel[:, 0]), med(rel[:, 2] - rel[:, 1]), np.max(rel[:, 2] - rel[:, 1]),
                        rel[:, 3].max()))
        a = np.array(res)[1:].mean(0)
        if impl == 0:
            print(f"{tag} {label:12s} waves={int(a[0]):5d} start_spread={a[1]:5.2f}us | x-wait {a[2]:4.2f} quant {a[3]:4.2f} "
                  f"barrier+fill {a[4]:4.2f} = prologue {a[6]:4.2f} | first step {a[5]:4.2f} loop med/max={a[7]:5.2f}/{a[8]:5.2f} "
                  f"loop end med/max={a[11]:6.2f}/{a[10]:6.2f} end={a[9]:6.2f}us")
            continue
        print(f"{tag} {label:12s} waves={int(a[0]):5d} start_spread={a[1]:5.2f}us | lookup {a[2]:4.2f} issue {a[3]:4.2f} "
              f"wait {a[4]:4.2f} quant {a[5]:4.2f} = prologue {a[6]:4.2f} | loop med/max={a[7]:5.2f}/{a[8]:5.2f} "
              f"end={a[9]:6.2f}us")


if __name__ == "__main__":
    for impl in ((0,) if PRO != "none" or "rows" in sys.argv else (0, 1)):
        main(impl)
