#!/bin/bash
# r04x: groups leg — does a high-priority stream anywhere in the process slow
# the lanes?  (measurement build, PMMG_HIP_SRFPRIO=0: no stream priority at all)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04x}
mkdir -p $OUT
for v in cur noprio r04m cur noprio r04m; do so=parmmg_amd/libpmmg_hip.so; env=""; [ $v = r04m ] && so=parmmg_amd/libpmmg_hip_r04m.so; [ $v = noprio ] && so=parmmg_amd/libpmmg_hip_measure.so && env="PMMG_HIP_SRFPRIO=0"; env $env PMMG_HIP_SO=$so timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2_$v.log 2>&1 && echo "$v $(grep -o '"ms_per_group_[a-z_]*": [0-9.]*' $OUT/bench_cfg2_$v.log | tr '\n' ' ')" || exit 1; done
