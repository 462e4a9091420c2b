#!/bin/bash
# r03ab: k_bdy grid of one round (512 blocks per XCD) vs 256, dynamic claiming:
# surface branch alone, cfg4 sweep, one 8-way rank
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ab}
mkdir -p $OUT
for v in "BDYBPX=512" "BDYBPX=256" "BDYDYN=1"; do
  timeout -k 10 200 python3 -u tools/surface_solo.py --steps 6 --env $v > $OUT/srf_$v.log 2>&1 || exit $?
  echo "$v $(tail -1 $OUT/srf_$v.log)"
done
timeout -k 10 700 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 4 --variants "sort=0;BDYBPX=256" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10 --variants ";BDYBPX=256" > $OUT/shard.txt 2>&1 \
&& grep "'rank'" $OUT/shard.txt
