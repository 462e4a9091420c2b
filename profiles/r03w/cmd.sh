#!/bin/bash
# r03w: every rank of the 8-way cfg4 halo split timed alone on one GPU
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03w}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,1,2,3,4,5,6,7 --steps 10 > $OUT/shard_step_cfg4_world8.txt 2>&1 \
&& echo "ok" && grep "'rank'" $OUT/shard_step_cfg4_world8.txt
