#!/bin/bash
# r03c: changed GPU tests, lane-pair walk A/B (locate only), quick cfg4 bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_snapshot.py tests/test_gpu_hits.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& timeout -k 10 600 python -u tools/sweep.py --config cfg4 --variants "sol=none;sol=none,PAIR=1" --rounds 3 --steps 4 > $OUT/sweep_pair.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep_pair.txt \
&& TAG=r03c BENCH_CONFIGS="cfg4" bash tools/gpu_bench_quick.sh
