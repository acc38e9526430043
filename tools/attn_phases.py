"""Where the time of one decode-attention launch goes (diagnostic): kq_attn_decode at
TinyLlama / Llama-3 head shapes, stopped after its loads (MI355X_ATTN_DIAG=1), after KQ
(2), after soft_max (3), empty (4) or complete (0) (ATTN_PHASES_DIAGS: which of them; the
stops need the KQ_ATTN_DIAG build). Per-launch kernel time from the
library's launch events, and back-to-back launches per microsecond of stream time."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]


def child():
    import numpy as np
    import torch
    import ggml_mi355x as g
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import knobs
    knobs.apply_env()  # MI355X_ATTN_DIAG -> the library knob (KQ_ATTN_DIAG builds only)
    dev = torch.device("cuda:0")
    out = []
    for hd, nh, nkv, n_ctx in ((64, 32, 4, 128), (64, 32, 4, 1024), (128, 32, 8, 512)):
        kvw = nkv * hd
        tab = g.rope_table(n_ctx, hd, 10000.0, 1.0, device=dev)
        kc = (torch.randn((n_ctx, kvw), device=dev) * 0.5).half().view(torch.int16)
        vc = (torch.randn((kvw, n_ctx), device=dev) * 0.5).half().view(torch.int16)
        q, k, v = (torch.randn(n * hd, device=dev) for n in (nh, nkv, nkv))
        y = torch.empty(nh * hd, device=dev)
        for p in sorted({0, 63, n_ctx // 2 - 1, n_ctx - 1}):
            pos = torch.tensor([p], dtype=torch.int32, device=dev)
            # ATTN_PHASES_ROPE_ROW=1: only the position's rope row (as the model's graph passes it)
            rr = os.environ.get("ATTN_PHASES_ROPE_ROW", "0") == "1"
            tb = tab[p].contiguous() if rr else tab
            for _ in range(20):
                g.attn_decode(q, k, v, pos, tb, kc, vc, nh, nkv, hd, 0.125, out=y, rope_row=rr)
            g.timing_enable(True)
            for _ in range(50):
                g.attn_decode(q, k, v, pos, tb, kc, vc, nh, nkv, hd, 0.125, out=y, rope_row=rr)
            rows = g.timing_read()
            g.timing_enable(False)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                g.attn_decode(q, k, v, pos, tb, kc, vc, nh, nkv, hd, 0.125, out=y, rope_row=rr)
            e1.record()
            torch.cuda.synchronize()
            out.append({"hd": hd, "n_ctx": n_ctx, "pos": p, "kernel_us": float(np.median([r[2] for r in rows]) * 1e3),
                        "stream_us_per_launch": e0.elapsed_time(e1) * 1e3 / 200})
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
        sys.exit(0)
    for diag in os.environ.get("ATTN_PHASES_DIAGS", "4 1 2 3 0").split():
        env = dict(os.environ, MI355X_ATTN_DIAG=diag)
        r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(r.stderr[-2000:])
            sys.exit(r.returncode)
        for row in json.loads(r.stdout.strip().splitlines()[-1]):
            print(f"diag={diag} hd={row['hd']:3d} n_ctx={row['n_ctx']:4d} pos={row['pos']:4d} "
                  f"kernel {row['kernel_us']:6.2f} us  stream {row['stream_us_per_launch']:6.2f} us/launch", flush=True)
