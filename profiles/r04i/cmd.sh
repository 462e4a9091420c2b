#!/bin/bash
# r04i: groups enqueued from one host thread per lane; Morton-order store
# cost isolated (measurement build: PMMG_HIP_PAD bit 30 = coalesced stores at
# the processing position, bit 29 = no interpolation); the default bench line
# (snapshot, carry-over iteration 2, groups leg, shuffled / Mmg-like legs)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04i}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_carry.py tests/test_gpu_snapshot.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -3 $OUT/pytest.log \
&& for L in 1 2 4; do PMMG_HIP_GROUP_LANES=$L timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2_lanes$L.log 2>&1 || exit 1; grep -o '"groups": {[^}]*}' $OUT/bench_cfg2_lanes$L.log; done \
&& timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0;perm=shuffle;perm=shuffle,PAD=1073741824;perm=shuffle,PAD=536870912;sort=0,sol=none;perm=shuffle,sol=none" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 900 python3 -u bench.py > $OUT/bench.log 2>&1 \
&& tail -1 $OUT/bench.log | head -c 6000
