#!/bin/bash
# r04zu: the second stream starts after k_bbox instead of after the axis maps;
# suite subset, sweep, groups leg
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zu}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_parity.py tests/test_gpu_groups.py tests/test_gpu_hits.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log \
&& timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 3 --variants "sort=0;perm=shuffle;perm=mmg" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2.log 2>&1 \
&& grep -o '"ms_per_group_[a-z_]*": [0-9.]*' $OUT/bench_cfg2.log
