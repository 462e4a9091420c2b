#!/bin/bash
# r04zo: the surface branch after the seed grid (SRFSOLO=1) — k_seed_vol ran
# at 455 us beside k_bdy against 261 alone (r04zl trace)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zo}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 3 --variants "sort=0;sort=0,SRFSOLO=1;perm=mmg;perm=mmg,SRFSOLO=1;perm=shuffle;perm=shuffle,SRFSOLO=1" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt
