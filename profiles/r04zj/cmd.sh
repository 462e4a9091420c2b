#!/bin/bash
# r04zj: radix sort scatter ranked per wave (4 barriers per tile): tests that
# run the sorted order, the shuffled step, its kernel trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zn}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_parity.py tests/test_gpu_groups.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log \
&& timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 3 --variants "perm=shuffle;sort=1;sort=0" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/shuf -o run --output-format csv -- python3 -u tools/sweep.py --config cfg4 --rounds 1 --steps 2 --variants "perm=shuffle" > $OUT/shuf.log 2>&1 && echo shuffle trace ok
