#!/bin/bash
# r03aa: plain stores for the per-lane scattered rows (surface path, exact
# continuation, fallbacks): surface branch alone, cfg4 step, one 8-way rank
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03aa}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/surface_solo.py --steps 6 > $OUT/surface_solo.log 2>&1 \
&& tail -2 $OUT/surface_solo.log \
&& timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 4 --variants "sort=0" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 10 > $OUT/shard.txt 2>&1 \
&& grep "'rank'" $OUT/shard.txt
