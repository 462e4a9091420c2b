#!/bin/bash
# r04s: the seed grid's axis maps on the second stream beside the fixed-point
# copy (A/B: measurement build PMMG_HIP_MAPSTREAM=0); the C test with the
# groups and carry-over checks; GPU suite; groups leg; 8-way rank step
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04s}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log \
&& timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 3 --variants "sort=0;sort=0,MAPSTREAM=0;perm=shuffle;perm=shuffle,MAPSTREAM=0" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2.log 2>&1 \
&& grep -o '"groups": {[^}]*}' $OUT/bench_cfg2.log \
&& timeout -k 10 600 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0,7 --steps 10 --variants ";MAPSTREAM=0" > $OUT/shard_step_cfg4_world8.txt 2>&1 \
&& tail -6 $OUT/shard_step_cfg4_world8.txt
