#!/bin/bash
# r03g: quick cfg4 bench (shuffled + Mmg-like legs, graded leg), then the
# graded-mesh parity test and the binned-path parity tests.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03g}
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok" && cat $OUT/bench.json \
&& timeout -k 10 600 python -u -m pytest "tests/test_gpu_configs.py::test_cfgG_graded_full_size_visit_range" tests/test_gpu_parity.py tests/test_gpu_hits.py -x -v -s --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok"
