#!/bin/bash
# r03y: per-rank 8-way split variants: default; static surface split; input
# order forced (no read-back of the coherence flag)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03y}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 10 --variants ";BDYDYN=2;sort=0;sort=0,BDYDYN=2" > $OUT/shard_variants.txt 2>&1 \
&& echo "ok" && grep "'rank'" $OUT/shard_variants.txt
