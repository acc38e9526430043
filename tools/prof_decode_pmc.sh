#!/bin/bash
# Wave-state PMC pass of the TinyLlama decode token (eager, 16 tokens): where the waves of each
# kernel spend their cycles (SQ_WAIT_ANY: parked on s_waitcnt / barrier; SQ_WAIT_INST_ANY:
# issue-stalled; SQ_ACTIVE_INST_ANY: issuing) and what they issue. One pass, 8 SQ counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_decode_pmc${TAG:+_$TAG}
mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_INSTS_VMEM SQ_WAVES --output-format csv -d $OUT/pmc -o run -- \
    python3 bench.py --steps 16 --warmup 2 --no-graph --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b \
    --tg 0 --no-collectives ${KNOBS:-} > $OUT/bench.log 2>&1 || exit $?
python3 - $OUT/pmc/run_counter_collection.csv <<'PY'
import collections, csv, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "kq::" not in k: continue
    name = k.split("(")[0].replace("void ", "")
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": n[name] += 1
print("| kernel | dispatches | waves/dispatch | wave-cycles parked (waitcnt/barrier) | issue-stalled | issuing | VALU / LDS / VMEM instr per wave |")
print("|---|---|---|---|---|---|---|")
for name, c in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    wc = c["SQ_WAVE_CYCLES"] or 1; w = c["SQ_WAVES"] or 1
    print(f"| `{name}` | {n[name]} | {w / max(n[name], 1):.0f} | {100 * c['SQ_WAIT_ANY'] / wc:.0f} % | {100 * c['SQ_WAIT_INST_ANY'] / wc:.0f} % | "
          f"{100 * c['SQ_ACTIVE_INST_ANY'] / wc:.0f} % | {c['SQ_INSTS_VALU'] / w:.0f} / {c['SQ_INSTS_LDS'] / w:.0f} / {c['SQ_INSTS_VMEM'] / w:.0f} |")
PY
rm -f $OUT/pmc/run_counter_collection.csv
