#!/bin/bash
# r03af: on a shuffled numbering, with the binning now beside the seed grid:
# coordinates copied in processing order (BINQS=1), coarser fine cells
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03af}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 4 --variants "perm=shuffle;perm=shuffle,BINQS=1;perm=shuffle,sort=1,BINBITS=6;perm=shuffle,sort=1,BINBITS=6,BINQS=1" > $OUT/sweep_shuffle.txt 2>&1 \
&& cat $OUT/sweep_shuffle.txt
