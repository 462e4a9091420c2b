#!/bin/bash
# GPU session: rocprofv3 kernel-trace summary and two PMC passes (FETCH_SIZE,
# WRITE_SIZE: they cannot share one pass) of the bench step alone (no side
# legs).  Each GPU step has its own time limit; steps are chained with &&.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
ARGS="${BENCH_ARGS}"
true \
&& echo "trace next" \
&& timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u bench.py $ARGS --no-cpu-baseline --no-host-mode --no-shuffled --no-quality --no-snapshot --no-graded --no-surface-solo --no-groups --steps 5 --warmup 1 > $OUT/trace.log 2>&1 \
&& echo "trace ok" \
&& timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 -u bench.py $ARGS --no-cpu-baseline --no-host-mode --no-shuffled --no-quality --no-snapshot --no-graded --no-surface-solo --no-groups --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1 \
&& echo "pmc fetch ok" \
&& timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 -u bench.py $ARGS --no-cpu-baseline --no-host-mode --no-shuffled --no-quality --no-snapshot --no-graded --no-surface-solo --no-groups --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1 \
&& echo "pmc write ok"
