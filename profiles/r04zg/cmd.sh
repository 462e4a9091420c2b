#!/bin/bash
# r04zg: the groups leg after a large call in the same process (measurement
# build): default, no stream priority at all, lanes' streams both at the
# highest priority
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zg}
mkdir -p $OUT
export PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so
for rep in 1 2; do for v in "" "PMMG_HIP_SRFPRIO=0" "PMMG_HIP_LANE_STREAMS=3"; do echo "== $v"; env $v timeout -k 10 300 python3 -u tools/groups_after_big.py cfg3 > $OUT/gab_$rep.log 2>&1 && grep -E "big call|groups:" $OUT/gab_$rep.log || exit 1; done; done
