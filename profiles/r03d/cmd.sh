#!/bin/bash
# r03d: graded / snapshot / hits GPU tests, then the default bench line
# (CPU baseline, parity, every side leg).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_graded.py tests/test_gpu_snapshot.py tests/test_gpu_hits.py "tests/test_gpu_configs.py::test_cfgG_graded_full_size_every_point" -x -v -s --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok" && cat $OUT/bench.json
