#!/bin/bash
# r03ak: the frame finalised by the last k_bbox block (default)
# vs by its own one-thread kernel (FRAMEK=1): cfg4 sweep, two 8-way ranks,
# the whole GPU suite (shard_step runs new, old, new: its first variant
# runs ~0.02 ms slow)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ak}
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 4 --variants "sort=0;FRAMEK=1" > $OUT/sweep_framek.txt 2>&1 \
&& cat $OUT/sweep_framek.txt \
&& timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 10 --variants ";FRAMEK=1;" > $OUT/shard_framek.txt 2>&1 \
&& grep "'rank'" $OUT/shard_framek.txt | cut -c1-330 \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && tail -2 $OUT/pytest_gpu.log
