#!/bin/bash
# r04f: pair-loaded walk records (one sector access per record and step),
# coalesced-lane seed grid with batched trips — GPU parity suites, cfg4 A/B
# against the previous commit (libpmmg_hip_measure_base.so), seed density
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04f}
mkdir -p $OUT
B=so=parmmg_amd/libpmmg_hip_measure_base.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -3 $OUT/pytest.log \
&& timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "$B,sort=0;sort=0;sort=0,TPC=6;sort=0,TPC=4;$B,sort=0,perm=mmg;sort=0,perm=mmg" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-mode --no-shuffled --no-quality --no-snapshot --no-graded --no-surface-solo --steps 5 --warmup 2 > $OUT/prof_bench.log 2>&1 \
&& tail -2 $OUT/prof_bench.log
