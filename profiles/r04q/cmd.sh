#!/bin/bash
# r04q: staged Morton records (runtime layouts excluded), tile-looped gated
# sort kernels, the surface stream at high priority (A/B: measurement build
# PMMG_HIP_SRFPRIO=0); GPU suite, cfg4 / cfg3 order sweeps
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04q}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log \
&& timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0;sort=0,SRFPRIO=0;perm=shuffle;perm=shuffle,SRFPRIO=0;sort=1;perm=mmg" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 600 python3 -u tools/sweep.py --config cfg3 --rounds 2 --steps 3 --variants "sort=0;perm=shuffle" > $OUT/sweep_cfg3.txt 2>&1 \
&& cat $OUT/sweep_cfg3.txt
