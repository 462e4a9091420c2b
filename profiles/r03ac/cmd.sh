#!/bin/bash
# r03ac: (1) non-temporal per-lane rows again: surface branch alone (beside
# the seed grid kernels, and after them: SRFSOLO=1), static
# and dynamic split; (2) the background's brick renumbering
# (PMMG_HIP_BRICK=b, measurement only) inside the cfg4 step, and its kernels
# in a trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ac}
mkdir -p $OUT
for v in "BDYBPX=512" "BDYDYN=1" "SRFSOLO=1" "SRFSOLO=1,BDYDYN=1"; do
  timeout -k 10 200 python3 -u tools/surface_solo.py --steps 6 --env $v > $OUT/srf_$v.log 2>&1 || exit $?
  echo "$v $(tail -1 $OUT/srf_$v.log)"
done
timeout -k 10 700 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 4 --variants "BRICK=0;BRICK=8;BRICK=4" > $OUT/sweep_brick.txt 2>&1 \
&& cat $OUT/sweep_brick.txt \
&& PMMG_HIP_BRICK=4 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_brick4 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-shuffled --no-snapshot --no-surface-solo --no-graded > $OUT/prof_brick4.log 2>&1 \
&& tail -2 $OUT/prof_brick4.log
