#!/bin/bash
# r04zq: surface seeds beside the seed grid, k_bdy after it (SRFSOLO=-1
# default) against the surface branch wholly after it (SRFSOLO=1) and
# beside it (SRFSOLO=0)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zq}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 4 --steps 3 --variants "sort=0;sort=0,SRFSOLO=1;sort=0,SRFSOLO=0;perm=mmg;perm=mmg,SRFSOLO=1" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt
