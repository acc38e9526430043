"""Summarise tools/prof_prompt.sh traces (4 graph-replayed prompts per model) into
profiles/r02_pp512_summary.md: kq kernels per prompt."""
import csv
import os
import shutil
import sys

TAG = os.environ.get("TAG", "r02")
SRC = sys.argv[1] if len(sys.argv) > 1 else f"gpurun_out/prof_prompt_{TAG}"
MODELS = (("TinyLlama-1.1B Q4_K_M", "tinyllama-1.1b", "tinyllama"), ("Llama-3-8B Q4_K_M", "llama-3-8b", "llama3_8b"))
out = [f"# pp512 through the graph — rocprofv3 kernel trace ({TAG})", "",
       "Command: `tools/prof_prompt.sh` (rocprofv3 --kernel-trace --stats -- python3 tools/prompt_graph_run.py",
       "<model>): four graph-replayed 512-token prompts after the capture (the bench's `pp512` figure), kq",
       "kernels only (the torch kernels of the weight generation are left out). Per prompt = total / 4.", ""]
for title, d, tag in MODELS:
    dst = f"profiles/{TAG}_pp512_{tag}_rocprof_kernel_stats.csv"
    shutil.copy(f"{SRC}/{d}/run_kernel_stats.csv", dst)
    rows = [r for r in csv.DictReader(open(dst)) if "kq::" in r["Name"]]
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / 4
    out += [f"## {title}: {tot / 1e3:.0f} us of kq kernels per prompt", "",
            "| kernel | launches/prompt | us/prompt | share |", "|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"]) / 4
        out.append(f"| `{r['Name'].replace('void ', '').split('(')[0]}` | {int(r['Calls']) // 4} | {t / 1e3:.1f} | "
                   f"{t / tot * 100:.1f} % |")
    out.append("")
open(f"profiles/{TAG}_pp512_summary.md", "w").write("\n".join(out))
print("\n".join(out))
