#!/bin/bash
# r04k: fewer launches per call (forced order's flag in k_reset, frame and
# axis maps finished by the last blocks, exhaustive passes merged and
# finished by the last block), snapshot kernels in XCD-contiguous order —
# the GPU suite, the groups leg, the snapshot alone, cfg4 sweep
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04k}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -3 $OUT/pytest.log \
&& timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2.log 2>&1 \
&& grep -o '"groups": {[^}]*}' $OUT/bench_cfg2.log \
&& timeout -k 10 300 python3 -u tools/snap_only.py cfg4 4 > $OUT/snap.log 2>&1 \
&& cat $OUT/snap.log \
&& timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0;;perm=mmg" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt
