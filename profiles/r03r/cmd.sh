#!/bin/bash
# r03r: surface seed grid density (cells per tria) for the surface branch alone
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03r}
mkdir -p $OUT
for m in 1 4 8 16 32; do
  timeout -k 10 200 python3 -u tools/surface_solo.py --steps 4 --env SRFMULT=$m > $OUT/srf_$m.log 2>&1 || exit $?
  echo "SRFMULT=$m $(tail -1 $OUT/srf_$m.log)"
done
