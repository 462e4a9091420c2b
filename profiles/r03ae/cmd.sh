#!/bin/bash
# r03ae: what made the shuffled / Mmg-like steps faster between r03v and
# r03ad: k_bdy's grid cap (256 vs 512 blocks per XCD) on both numberings
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ae}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 4 --variants "perm=shuffle;perm=shuffle,BDYBPX=256;perm=mmg;perm=mmg,BDYBPX=256" > $OUT/sweep_orders.txt 2>&1 \
&& cat $OUT/sweep_orders.txt
