#!/bin/bash
# r03x: coherence test first (flag read back beside the frame kernels):
# parity tests, quick bench, 8-way per-rank timing
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& TAG=r03x BENCH_CONFIGS="cfg4 cfg2" bash tools/gpu_bench_quick.sh \
&& timeout -k 10 900 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,1,2,3,4,5,6,7 --steps 10 > $OUT/shard_step_cfg4_world8.txt 2>&1 \
&& echo "shard ok" && grep "'rank'" $OUT/shard_step_cfg4_world8.txt
