#!/bin/bash
# r04g: the query order decided on the device (no host read in the call; own
# gated radix sort instead of rocPRIM) with the per-lane walk restored —
# shuffled numberings at cfg2 / cfg3 with forced orders (the small-group
# rule), the GPU suite, cfg4 order variants A/B against the previous commit,
# the default bench line, a kernel trace of the bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04g}
mkdir -p $OUT
B=so=parmmg_amd/libpmmg_hip_measure_base.so
V="sort=0;sort=1;perm=shuffle,sort=0;perm=shuffle,sort=1;perm=shuffle;perm=mmg,sort=0;perm=mmg,sort=1"
timeout -k 10 300 python3 -u tools/sweep.py --config cfg2 --rounds 2 --steps 5 --variants "$V" > $OUT/sweep_cfg2.txt 2>&1 \
&& cat $OUT/sweep_cfg2.txt \
&& timeout -k 10 300 python3 -u tools/sweep.py --config cfg3 --rounds 2 --steps 3 --variants "$V" > $OUT/sweep_cfg3.txt 2>&1 \
&& cat $OUT/sweep_cfg3.txt \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect "tests/test_gpu_edge.py::test_query_order_detection" > $OUT/pytest.log 2>&1 \
&& tail -3 $OUT/pytest.log \
&& timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "$B;;sort=1;$B,sort=1;perm=shuffle;$B,perm=shuffle;perm=mmg;$B,perm=mmg" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 600 python3 -u bench.py > $OUT/bench.log 2>&1 \
&& tail -3 $OUT/bench.log \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-graded --no-surface-solo --steps 5 --warmup 2 > $OUT/prof_bench.log 2>&1 \
&& tail -2 $OUT/prof_bench.log
