#!/bin/bash
# r04m: XCD run length sweep of k_vol (measurement build), the default bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04m}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0;sort=0,XCDRUN=16;sort=0,XCDRUN=32;sort=0,XCDRUN=128;sort=0,XCDRUN=256;perm=mmg,XCDRUN=16;perm=mmg;perm=mmg,XCDRUN=256" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 900 python3 -u bench.py > $OUT/bench.log 2>&1 \
&& tail -1 $OUT/bench.log | head -c 3000
