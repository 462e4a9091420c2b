#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 --pmc run per counter set;
# each pass has its own hard time limit, chained with &&).
#   TAG=x BENCH_ARGS="--config cfg4" bash tools/gpu_pmc.sh "SQ_WAVES SQ_WAVE_CYCLES" "TCC_HIT_sum TCC_MISS_sum"
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
i=0
rc=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 -u bench.py ${BENCH_ARGS} --no-cpu-baseline --steps 1 --warmup 1 > $OUT/p$i.log 2>&1 || { rc=$?; echo "pass $i failed rc=$rc"; break; }
  echo "pass $i ok: $set"
done
exit $rc
