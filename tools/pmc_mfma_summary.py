"""Summarise a rocprofv3 --pmc MFMA pass (tools/prof_prefill.sh) per kq kernel:
MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 256 CUs * 4 SIMDs),
VALU activity, and the clock implied by GRBM_GUI_ACTIVE over the dispatch duration."""
import collections
import csv
import sys


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in rows:
        k = r["Kernel_Name"]
        if "kq::" not in k:
            continue
        key = (r["Dispatch_Id"], k.split("(")[0].replace("void ", ""), r["Grid_Size"])
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    lines = ["| kernel | grid | dispatches | us (mean) | MFMA busy | VALU active | I8 MFMA MOPS | F32 MFMA MOPS |",
             "|---|---|---|---|---|---|---|---|"]
    groups = collections.OrderedDict()  # (name, grid) in first-dispatch order -> dispatch keys
    for key in sorted(agg, key=lambda k: int(k[0])):
        groups.setdefault(key[1:], []).append(key)
    for (name, grid), keys in groups.items():
        c = collections.defaultdict(float)
        for k in keys:
            for n, v in agg[k].items():
                c[n] += v / len(keys)
        t = sum(meta[k] for k in keys) / len(keys)
        key = (None, name, grid)
        gui = c["GRBM_GUI_ACTIVE"]
        simd_cyc = gui / 8 * 256 * 4
        lines.append(f"| `{key[1]}` | {key[2]} | {len(keys)} | {t / 1e3:.1f} | {c['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cyc * 100:.1f} % | "
                     f"{c['SQ_ACTIVE_INST_VALU'] / max(1.0, c['SQ_WAVE_CYCLES']) * 100:.0f} % | "
                     f"{c['SQ_INSTS_VALU_MFMA_MOPS_I8']:.3g} | {c['SQ_INSTS_VALU_MFMA_MOPS_F32']:.3g} |")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
