#!/bin/bash
# r03l: Morton binning knobs (key bits per axis, coordinate copy) on the
# lattice (forced bins), Mmg-like (forced bins) and shuffled numberings
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03l}
mkdir -p $OUT
timeout -k 10 700 python3 -u tools/sweep.py --config cfg4 --rounds 1 --steps 4 --variants "sort=0;sort=1;sort=1,BINQS=2;sort=1,BINBITS=5;sort=1,BINBITS=5,BINQS=2;perm=mmg,sort=1,BINQS=2;perm=mmg,sort=1,BINBITS=5,BINQS=2;perm=shuffle;perm=shuffle,BINQS=2;perm=shuffle,BINBITS=6,BINQS=2;perm=shuffle,BINBITS=5,BINQS=2" > $OUT/sweep_bin.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep_bin.txt
