#!/bin/bash
# Interleaved in-process sweep of module settings (tools/sweep.py), own time limit.
#   TAG=x SWEEP_ARGS='--config cfg4 --variants "TPC=8;TPC=4"' bash tools/gpu_sweep.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
eval timeout -k 10 ${SWEEP_TIMEOUT:-400} python -u tools/sweep.py ${SWEEP_ARGS} > $OUT/sweep.txt 2> $OUT/sweep.err \
&& echo "sweep ok" && cat $OUT/sweep.txt
