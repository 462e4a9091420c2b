#!/bin/bash
# GPU session: one short bench line per config in BENCH_CONFIGS (no CPU
# baseline, no side legs unless BENCH_ARGS adds them).  Each step has its own
# time limit; steps are chained with &&.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
rc=0
for cfg in ${BENCH_CONFIGS:-cfg4}; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-graded ${BENCH_ARGS} > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { rc=$?; echo "bench $cfg failed rc=$rc"; break; }
  echo "bench $cfg ok"; cat $OUT/bench_$cfg.json
done
exit $rc
