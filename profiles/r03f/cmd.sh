#!/bin/bash
# r03f: Morton binning without global atomics + cooperative scattered row
# stores: GPU parity tests that cover the binned path, then a quick cfg4 bench
# line with the shuffled and Mmg-like numbering legs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_hits.py "tests/test_gpu_configs.py" -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-graded > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok" && cat $OUT/bench.json
