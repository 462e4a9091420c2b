#!/bin/bash
# r04zf: round-4 final measurement — kernel trace + FETCH / WRITE passes of
# the bench step (tools/gpu_prof.sh), the GPU suite, the default bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zf}
mkdir -p $OUT
TAG=${TAG:-r04zf} bash tools/gpu_prof.sh \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log \
&& timeout -k 10 900 python3 -u bench.py > $OUT/bench_full.log 2>&1 \
&& tail -1 $OUT/bench_full.log | cut -c1-400
