#!/bin/bash
# r03i: graded test with the fallback-cause counters, then a quick cfg4 bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03i}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest "tests/test_gpu_configs.py::test_cfgG_graded_full_size_visit_range" -v -s --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-graded > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok" && cat $OUT/bench.json
