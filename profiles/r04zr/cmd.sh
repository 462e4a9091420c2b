#!/bin/bash
# r04zr: seed grid density (tetra per cell) with the surface branch after the
# seed grid
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zr}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 3 --variants "sort=0;sort=0,TPC=6;sort=0,TPC=12;sort=0,TPC=4" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt
