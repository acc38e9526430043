"""Per-kernel means of every counter in a rocprofv3 --pmc run (counter_collection.csv):
one row per (kernel, grid), counters as columns, plus the mean dispatch duration.
Usage: python3 tools/pmc_table.py <counter_collection.csv> [filter-substring]"""
import collections
import csv
import sys


def main(path, filt=None):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in rows:
        k = r["Kernel_Name"]
        if "kq::" not in k or (filt and filt not in k):
            continue
        key = (int(r["Dispatch_Id"]), k.split("(")[0].replace("void ", ""), r["Grid_Size"])
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    groups = collections.OrderedDict()
    for key in sorted(agg):
        groups.setdefault(key[1:], []).append(key)
    names = sorted({n for k in agg for n in agg[k]})
    print("| kernel | grid | n | us | " + " | ".join(names) + " |")
    print("|---" * (4 + len(names)) + "|")
    for (name, grid), keys in groups.items():
        mean = {n: sum(agg[k][n] for k in keys) / len(keys) for n in names}
        t = sum(dur[k] for k in keys) / len(keys) / 1e3
        print(f"| `{name}` | {grid} | {len(keys)} | {t:.1f} | " + " | ".join(f"{mean[n]:.4g}" for n in names) + " |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
