"""Summarise the rocprofv3 runs of tools/profile_r1.sh (kernel trace + separate
FETCH_SIZE / WRITE_SIZE PMC passes of the same bench command) into one JSON +
markdown table under profiles/.

The bench's graph-replayed token is `launches` dispatches of the kq kernels; the
first `warmup` tokens are skipped and the next `steps` tokens form the timed
region. Per launch position in the token: kernel, mean duration (kernel trace),
HBM bytes read = FETCH_SIZE (KB) x 1024 x 2 (gfx950: FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, MI355X_MICROARCH.md HBM section) and
bytes written = WRITE_SIZE (KB) x 1024.

usage: python tools/prof_summary.py gpurun_out/prof_r01 profiles/r01 --warmup 8 --steps 64 --launches 89
"""
import argparse
import csv
import json
import os
import statistics


def kq_rows(path):
    """kq dispatches in execution order (the CSV is not time-sorted for graph launches)."""
    with open(path) as f:
        rows = [r for r in csv.DictReader(f) if "kq::" in r["Kernel_Name"]]
    key = "Start_Timestamp" if rows and "Start_Timestamp" in rows[0] else "Dispatch_Id"
    rows.sort(key=lambda r: int(r[key]))
    return rows


def short(name):
    name = name.replace("void ", "")
    return name.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst_prefix")
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--launches", type=int, default=89)
    ap.add_argument("--pmc-warmup", type=int, default=None, help="PMC passes: warmup tokens (default: --warmup)")
    ap.add_argument("--pmc-steps", type=int, default=None, help="PMC passes: timed tokens (default: --steps)")
    ap.add_argument("--bench-json", default=None, help="bench JSON line (for the algorithmic bytes)")
    ap.add_argument("--kinds", default=None, help="bench BENCH_KINDS_OUT file: launch kind of every position")
    a = ap.parse_args()
    L, W, K = a.launches, a.warmup, a.steps
    PW = a.warmup if a.pmc_warmup is None else a.pmc_warmup
    PK = a.steps if a.pmc_steps is None else a.pmc_steps
    tr = kq_rows(os.path.join(a.src, "trace", "run_kernel_trace.csv"))
    timed = tr[W * L:(W + K) * L]
    assert len(timed) == K * L, (len(tr), len(timed))
    fetch = write = None
    pf = os.path.join(a.src, "pmc_fetch", "run_counter_collection.csv")
    pw = os.path.join(a.src, "pmc_write", "run_counter_collection.csv")
    if os.path.exists(pf):
        fetch = [float(r["Counter_Value"]) * 1024 * 2 for r in kq_rows(pf)][PW * L:(PW + PK) * L]
    if os.path.exists(pw):
        write = [float(r["Counter_Value"]) * 1024 for r in kq_rows(pw)][PW * L:(PW + PK) * L]

    def dur(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us

    per_pos = []
    for p in range(L):
        idx = [t * L + p for t in range(K)]
        names = {short(timed[i]["Kernel_Name"]) for i in idx}
        assert len(names) == 1, names
        e = {"pos": p, "kernel": names.pop(), "grid": int(timed[idx[0]]["Grid_Size_X"]),
             "lds": int(timed[idx[0]]["LDS_Block_Size"]),
             "us_mean": statistics.mean(dur(timed[i]) for i in idx),
             "us_median": statistics.median(dur(timed[i]) for i in idx)}
        pidx = [t * L + p for t in range(PK)]
        if fetch:
            e["hbm_read_bytes"] = statistics.median(fetch[i] for i in pidx)
        if write:
            e["hbm_write_bytes"] = statistics.median(write[i] for i in pidx)
        per_pos.append(e)
    by_kernel = {}
    for e in per_pos:
        k = by_kernel.setdefault(e["kernel"], {"launches_per_token": 0, "us_per_token": 0.0, "hbm_read_per_token": 0.0})
        k["launches_per_token"] += 1
        k["us_per_token"] += e["us_mean"]
        k["hbm_read_per_token"] += e.get("hbm_read_bytes", 0.0)
    for k in by_kernel.values():
        k["us_per_launch"] = k["us_per_token"] / k["launches_per_token"]
        k["hbm_read_per_launch"] = k["hbm_read_per_token"] / k["launches_per_token"]
    by_kind = {}
    if a.kinds:  # launch kinds (kernel @ algorithmic MB per launch), as bench.py's roofline keys them
        with open(a.kinds) as f:
            kinds = json.load(f)
        assert len(kinds) == L, (len(kinds), L)
        for e, kname in zip(per_pos, kinds):
            # (the library's launch names omit defaulted template arguments that rocprofv3 prints)
            assert kname.split(" @ ")[0].split("<")[0] == e["kernel"].split("<")[0], (kname, e["kernel"])
            e["kind"] = kname
            k = by_kind.setdefault(kname, {"launches_per_token": 0, "us_per_token": 0.0, "hbm_read_per_token": 0.0,
                                           "MB_per_launch": float(kname.split(" @ ")[1].split()[0])})
            k["launches_per_token"] += 1
            k["us_per_token"] += e["us_mean"]
            k["hbm_read_per_token"] += e.get("hbm_read_bytes", 0.0)
        for k in by_kind.values():
            k["us_per_launch"] = k["us_per_token"] / k["launches_per_token"]
            k["hbm_read_per_launch"] = k["hbm_read_per_token"] / k["launches_per_token"]
            k["GBps"] = k["MB_per_launch"] * 1e6 / (k["us_per_launch"] * 1e-6) / 1e9
            k["frac"] = k["GBps"] / 8000.0
            k["traffic_over_algorithmic"] = (k["hbm_read_per_launch"] / (k["MB_per_launch"] * 1e6)
                                             if k["MB_per_launch"] > 0 and fetch else None)
    span = (int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e3 / K
    busy = sum(dur(r) for r in timed) / 1e3 / K * 1e3
    out = {"source": a.src, "warmup": W, "steps": K, "launches_per_token": L,
           "token_span_us": span, "kernel_busy_us_per_token": busy,
           "hbm_read_MB_per_token": sum(e.get("hbm_read_bytes", 0) for e in per_pos) / 1e6 if fetch else None,
           "hbm_write_MB_per_token": sum(e.get("hbm_write_bytes", 0) for e in per_pos) / 1e6 if write else None,
           "by_kernel": by_kernel, "by_kind": by_kind, "per_position": per_pos}
    if a.bench_json:
        with open(a.bench_json) as f:
            out["bench"] = json.loads([ln for ln in f if ln.startswith("{")][-1])
    with open(a.dst_prefix + "_summary.json", "w") as f:
        json.dump(out, f, indent=1)
    with open(a.dst_prefix + "_summary.md", "w") as f:
        f.write(f"# rocprofv3 summary ({a.src})\n\n")
        f.write(f"Timed region: tokens {W}..{W + K - 1}, {L} kq launches per token.\n\n")
        f.write(f"* token span (first start -> last end): {span:.1f} us; kernel busy {busy:.1f} us/token\n")
        if fetch:
            f.write(f"* HBM read (FETCH_SIZE x2): {out['hbm_read_MB_per_token']:.1f} MB/token\n")
        if write:
            f.write(f"* HBM write (WRITE_SIZE): {out['hbm_write_MB_per_token']:.3f} MB/token\n")
        f.write("\n| kernel | launches/token | us/launch | HBM read/launch (MB) |\n|---|---|---|---|\n")
        for name, k in sorted(by_kernel.items(), key=lambda kv: -kv[1]["us_per_token"]):
            f.write(f"| `{name}` | {k['launches_per_token']} | {k['us_per_launch']:.2f} | "
                    f"{k['hbm_read_per_launch'] / 1e6:.2f} |\n")
        if by_kind:
            f.write("\n| launch kind (kernel @ algorithmic MB) | launches/token | us/launch (replayed) | GB/s | "
                    "frac of 8 TB/s | HBM read/launch (MB) | read / algorithmic |\n|---|---|---|---|---|---|---|\n")
            for name, k in sorted(by_kind.items(), key=lambda kv: -kv[1]["us_per_token"]):
                ratio = k["traffic_over_algorithmic"]
                f.write(f"| `{name}` | {k['launches_per_token']} | {k['us_per_launch']:.2f} | {k['GBps']:.0f} | "
                        f"{k['frac']:.3f} | {k['hbm_read_per_launch'] / 1e6:.2f} | "
                        f"{'' if ratio is None else f'{ratio:.2f}'} |\n")
        f.write("\n| pos | kernel | grid | LDS | us (mean) | HBM read (MB) |\n|---|---|---|---|---|---|\n")
        for e in per_pos[:8] + per_pos[-1:]:
            f.write(f"| {e['pos']} | `{e['kernel']}` | {e['grid']} | {e['lds']} | {e['us_mean']:.2f} | "
                    f"{e.get('hbm_read_bytes', 0) / 1e6:.2f} |\n")
    print(open(a.dst_prefix + "_summary.md").read())


if __name__ == "__main__":
    main()
