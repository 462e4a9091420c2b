#!/bin/bash
# GPU session: parity tests, a default bench line (CPU baseline + full-size
# parity), a rocprofv3 kernel-trace summary.  Every GPU step has its own time
# limit; steps are chained with && (stop at the first failure).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 \
&& echo "pytest ok" \
&& timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok" && cat $OUT/bench.json \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py ${BENCH_ARGS} --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --steps 5 --warmup 2 > $OUT/prof_bench.log 2>&1 \
&& echo "rocprof ok"
