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
# the shuffled numbering alone under the kernel tracer (binning kernels)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_shuf -o run --output-format csv -- python3 -u tools/sweep.py --config cfg4 --steps 3 --child perm=shuffle > $OUT/prof_shuf.log 2>&1 \
&& echo "prof shuffled ok"
# input order against Morton bins on the lattice, Mmg-like and shuffled numberings
timeout -k 10 400 python3 -u tools/sweep.py --config cfg4 --rounds 1 --steps 4 --variants "sort=0;sort=1;perm=mmg,sort=0;perm=mmg,sort=1;perm=shuffle" > $OUT/sweep_orders.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep_orders.txt
