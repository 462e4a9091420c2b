#!/bin/bash
# r03k: graded test (window-based axis map, wider seed ring), kernel trace of
# the Morton-binned lattice step, the order sweep
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03k}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest "tests/test_gpu_configs.py::test_cfgG_graded_full_size_visit_range" -v -s --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sort -o run --output-format csv -- python3 -u tools/sweep.py --config cfg4 --steps 3 --child sort=1 > $OUT/prof_sort.log 2>&1 \
&& echo "prof sort ok" \
&& timeout -k 10 400 python3 -u tools/sweep.py --config cfg4 --rounds 1 --steps 4 --variants "sort=0;sort=1;perm=mmg,sort=1;perm=shuffle" > $OUT/sweep_orders.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep_orders.txt
