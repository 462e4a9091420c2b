#!/bin/bash
# r03p: class compaction restored, sparser bbox / axis-histogram sampling:
# parity tests, sweep against the old sampling, quick bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03p}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& timeout -k 10 700 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 4 --variants "sort=0;BBOX=16,HIST=64" > $OUT/sweep_prep.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep_prep.txt \
&& TAG=r03p BENCH_CONFIGS="cfg4 cfg3" bash tools/gpu_bench_quick.sh
