#!/bin/bash
# r04v: groups leg — the r04m build against the current product build
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04v}
mkdir -p $OUT
for v in r04m cur r04m cur; do so=parmmg_amd/libpmmg_hip.so; [ $v = r04m ] && so=parmmg_amd/libpmmg_hip_r04m.so; PMMG_HIP_SO=$so timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2_$v.log 2>&1 && echo "$v $(grep -o '"ms_per_group_[a-z_]*": [0-9.]*' $OUT/bench_cfg2_$v.log | tr '\n' ' ') $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_cfg2_$v.log)" || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/shuf -o run --output-format csv -- python3 -u tools/sweep.py --config cfg4 --rounds 1 --steps 2 --variants "perm=shuffle" > $OUT/shuf.log 2>&1 && echo shuffle trace ok
