#!/bin/bash
# r04j: kernel traces of the device snapshot at cfg4 and of the groups leg
# (10 cfg2-size groups, 4 lanes)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04j}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_hits.py tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_groups.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -3 $OUT/pytest.log \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/snap -o run --output-format csv -- python3 -u tools/snap_only.py cfg4 4 > $OUT/snap.log 2>&1 \
&& cat $OUT/snap.log \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/groups -o run --output-format csv -- python3 -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/groups.log 2>&1 \
&& grep -o '"groups": {[^}]*}' $OUT/groups.log
