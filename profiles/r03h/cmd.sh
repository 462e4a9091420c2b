#!/bin/bash
# r03h: two-level Morton binning, per-axis seed-grid map, stochastic walk
# rule: binned-path parity tests + graded test, then a quick cfg4 bench with
# the renumbered legs and the graded leg.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03h}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_edge.py tests/test_gpu_configs.py -v -s --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok" && cat $OUT/bench.json
