#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy / LDS of the HIP module, from the
# compiler's resource-usage remarks (same flags as parmmg_amd/build.py).
#   bash tools/resource_usage.sh [kernel-name-regex]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-sched-strategy=max-memory-clause -std=c++17 \
  -ffp-contract=off -fPIC -c --offload-device-only -Rpass-analysis=kernel-resource-usage ${EXTRA_FLAGS} \
  -I"$ROOT/include" -o "$OUT/hip.o" "$ROOT/parmmg_amd/csrc/pmmg_hip.hip" 2> "$OUT/usage.txt"
python3 - "$OUT/usage.txt" "${1:-.}" <<'PY'
import re, sys, subprocess
pat = re.compile(sys.argv[2])
cur = None
rows = []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \[bytes/lane\]", "Occupancy \[waves/SIMD\]", "LDS Size \[bytes/block\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0]] = int(m.group(1))
for r in rows:
    try:
        dn = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    except Exception:
        dn = r["name"]
    if pat.search(dn):
        print(f'{dn[:90]:90s} vgpr {r.get("VGPRs")} scratch {r.get("ScratchSize")} occ {r.get("Occupancy")} lds {r.get("LDS")}')
PY
rm -rf "$OUT"
