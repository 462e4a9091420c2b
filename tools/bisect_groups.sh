#!/bin/bash
# groups leg: libraries built at several commits (PMMG_HIP_SO), interleaved
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-bisect}
mkdir -p $OUT
for v in r04m 4302073 8f076de cur r04m 4302073 8f076de cur; do so=parmmg_amd/libpmmg_hip_$v.so; [ $v = cur ] && so=parmmg_amd/libpmmg_hip.so; PMMG_HIP_SO=$so timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2_$v.log 2>&1 && echo "$v $(grep -o '"ms_per_group_[a-z_]*": [0-9.]*' $OUT/bench_cfg2_$v.log | tr '\n' ' ')" || exit 1; done
