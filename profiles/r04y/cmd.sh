#!/bin/bash
# r04y: high-priority surface stream only for large calls (dropped by a
# groups call): groups leg vs the r04m build; cfg4 priority A/B; GPU suite
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04y}
mkdir -p $OUT
for v in cur r04m cur r04m; do so=parmmg_amd/libpmmg_hip.so; [ $v = r04m ] && so=parmmg_amd/libpmmg_hip_r04m.so; PMMG_HIP_SO=$so timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2_$v.log 2>&1 && echo "$v $(grep -o '"ms_per_group_[a-z_]*": [0-9.]*' $OUT/bench_cfg2_$v.log | tr '\n' ' ')" || exit 1; done \
&& timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 3 --variants "sort=0;sort=0,SRFPRIO=0" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log
