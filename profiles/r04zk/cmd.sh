#!/bin/bash
# r04zk: XCD run length of the volume kernel on the Mmg-like numbering
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zk}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 3 --variants "perm=mmg;perm=mmg,XCDRUN=16;perm=mmg,XCDRUN=256;perm=mmg,XCDRUN=1024;sort=0;sort=0,XCDRUN=256" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt
