#!/bin/bash
# HBM read per decode GEMV launch against its weight bytes (tools/traffic_probe.py under a
# FETCH_SIZE pass; tools/traffic_fit.py fits read = a + b * bytes on the CPU afterwards).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/traffic
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 tools/traffic_probe.py > $OUT/probe.log 2>&1 || exit $?
tail -2 $OUT/probe.log
