#!/bin/bash
# r04zh: the surface tail without stream priority — the volume kernel after
# the surface branch (BDYFIRST) against the high-priority surface stream
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zh}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 3 --variants "sort=0;sort=0,SRFPRIO=0;sort=0,SRFPRIO=0,BDYFIRST=1;perm=mmg,SRFPRIO=0;perm=mmg,SRFPRIO=0,BDYFIRST=1;perm=mmg" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt
