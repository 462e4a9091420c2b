#!/bin/bash
# r03j: rocPRIM Morton binning: binned-path parity tests, the graded test,
# the order sweep, then a quick cfg4 bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03j}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_hits.py tests/test_gpu_configs.py -v -s --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 -u tools/sweep.py --config cfg4 --rounds 1 --steps 4 --variants "sort=0;sort=1;perm=mmg,sort=0;perm=mmg,sort=1;perm=shuffle" > $OUT/sweep_orders.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep_orders.txt \
&& timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok"
