#!/bin/bash
# Per-kernel VGPR / SGPR / scratch / occupancy of one HIP source as hipcc reports them
# (-Rpass-analysis=kernel-resource-usage), one line per kernel.
#   tools/resource_usage.sh ggml-neon-opt_amd/csrc/kq_rows.hip [extra hipcc flags]
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
src="$1"; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  -I"$ROOT/include" -I"$ROOT/ggml-neon-opt_amd/csrc" --cuda-device-only -c -Rpass-analysis=kernel-resource-usage "$@" \
  "$src" -o /tmp/_ru.o 2>&1 | python3 -c '
import re, sys
cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("sgpr", r" SGPRs: (\d+)"),
                     ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur:
            rows[cur][key] = int(m.group(1))
for k, v in rows.items():
    print("%-70s " % k + " ".join("%s=%s" % (f, v.get(f)) for f in ("vgpr", "agpr", "sgpr", "scratch", "occ")))
'
