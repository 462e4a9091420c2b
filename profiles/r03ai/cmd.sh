#!/bin/bash
# r03ai: the query order passed to the volume kernel as an argument (default)
# vs written by k_set_order between the seed grid and the volume kernel
# (SETORDER=1): cfg4 sweep, two 8-way ranks, the GPU parity tests; then the
# PMC passes of r03ah on the new default
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03ai}
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 4 --variants "sort=0;SETORDER=1" > $OUT/sweep_setorder.txt 2>&1 \
&& cat $OUT/sweep_setorder.txt \
&& timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 10 --variants ";SETORDER=1" > $OUT/shard_setorder.txt 2>&1 \
&& grep "'rank'" $OUT/shard_setorder.txt | cut -c1-330 \
&& timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_hits.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_parity.log 2>&1 \
&& tail -2 $OUT/pytest_parity.log \
&& TAG=r03ai_pmc bash tools/gpu_r03ah.sh
