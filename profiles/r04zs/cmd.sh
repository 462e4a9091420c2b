#!/bin/bash
# r04zs: the 8-way rank step (ranks 0 and 7 timed alone) with the final code
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zs}
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,7 --steps 10 > $OUT/shard_step_cfg4_world8.txt 2>&1 \
&& tail -3 $OUT/shard_step_cfg4_world8.txt
