#!/bin/bash
# r03ac: non-temporal per-lane rows again: surface branch alone, static and
# dynamic split
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ac}
mkdir -p $OUT
for v in "BDYBPX=512" "BDYDYN=1"; do
  timeout -k 10 200 python3 -u tools/surface_solo.py --steps 6 --env $v > $OUT/srf_$v.log 2>&1 || exit $?
  echo "$v $(tail -1 $OUT/srf_$v.log)"
done
