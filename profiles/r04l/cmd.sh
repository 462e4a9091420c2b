#!/bin/bash
# r04l: the axis-map fold reverted; groups leg twice, cfg4 sweep, the 8-way
# split's per-rank step (tools/shard_step.py, ranks 0 and 7), a kernel trace
# of the cfg2 groups leg
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04l}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_hits.py tests/test_gpu_parity.py tests/test_gpu_groups.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log \
&& for r in 1 2; do timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2_$r.log 2>&1 || exit 1; grep -o '"groups": {[^}]*}' $OUT/bench_cfg2_$r.log; done \
&& timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0;perm=mmg" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 600 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,7 --steps 10 > $OUT/shard_step_cfg4_world8.txt 2>&1 \
&& tail -8 $OUT/shard_step_cfg4_world8.txt \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/groups -o run --output-format csv -- python3 -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/groups_prof.log 2>&1 \
&& echo done
