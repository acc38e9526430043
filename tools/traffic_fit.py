"""Fit the FETCH_SIZE pass of tools/traffic_probe.py: per shape the mean HBM read per kq_rows
launch (FETCH_SIZE x 1024 x 2, the gfx950 correction) against its weight bytes, and per
(type, K) group a least-squares line read = a + b * bytes.
usage: python tools/traffic_fit.py gpurun_out/traffic/pmc_fetch/run_counter_collection.csv [out.md]"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(path, out=None):
    from traffic_probe import REPS, SHAPES, g  # noqa: F401
    rows = [r for r in csv.DictReader(open(path)) if "kq_rows" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    vals = [float(r["Counter_Value"]) * 1024 * 2 for r in rows]
    assert len(vals) == REPS * len(SHAPES), (len(vals), REPS * len(SHAPES))
    bpb = {g.TYPE_Q4_K: 144, g.TYPE_Q5_K: 176, g.TYPE_Q6_K: 210}
    lines = ["| type | K | N | weight MB | read MB/launch | read / weight | excess KB |", "|---|---|---|---|---|---|---|"]
    groups = {}
    for i, (typ, K, N) in enumerate(SHAPES):
        v = vals[i * REPS + 1:(i + 1) * REPS]  # the first launch of a shape warms code and tables
        m = sum(v) / len(v)
        wb = N * (K // 256) * bpb[typ]
        groups.setdefault((typ, K), []).append((wb, m))
        lines.append(f"| {typ} | {K} | {N} | {wb / 1e6:.3f} | {m / 1e6:.3f} | {m / wb:.3f} | {(m - wb) / 1e3:.0f} |")
    lines += ["", "| type | K | fixed read a (KB/launch) | slope b (read per weight byte) |", "|---|---|---|---|"]
    for (typ, K), pts in groups.items():
        n = len(pts)
        sx = sum(p[0] for p in pts)
        sy = sum(p[1] for p in pts)
        sxx = sum(p[0] ** 2 for p in pts)
        sxy = sum(p[0] * p[1] for p in pts)
        b = (n * sxy - sx * sy) / (n * sxx - sx * sx)
        a = (sy - b * sx) / n
        lines.append(f"| {typ} | {K} | {a / 1e3:.0f} | {b:.4f} |")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
