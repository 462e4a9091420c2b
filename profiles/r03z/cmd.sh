#!/bin/bash
# r03z: fixed-point copy beside the seed grid (QPAR=1) against the default,
# on cfg4 and on one rank of the 8-way split
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03z}
mkdir -p $OUT
timeout -k 10 700 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 4 --variants "sort=0;QPAR=1" > $OUT/sweep_qpar.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep_qpar.txt \
&& timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10 --variants ";QPAR=1" > $OUT/shard_qpar.txt 2>&1 \
&& echo "shard ok" && grep "'rank'" $OUT/shard_qpar.txt
