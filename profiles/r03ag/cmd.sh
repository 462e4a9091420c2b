#!/bin/bash
# r03ag: the seed grid's axis histogram + map on a third stream beside
# k_quantize (default) vs on the main stream before it (MAPMAIN=1): cfg4
# sweep, one 8-way rank; then the GPU parity tests on the new default
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ag}
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 4 --variants "sort=0;MAPMAIN=1" > $OUT/sweep_map.txt 2>&1 \
&& cat $OUT/sweep_map.txt \
&& timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 10 --variants ";MAPMAIN=1" > $OUT/shard_map.txt 2>&1 \
&& grep "'rank'" $OUT/shard_map.txt \
&& timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_parity.log 2>&1 \
&& tail -2 $OUT/pytest_parity.log
