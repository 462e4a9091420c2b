#!/bin/bash
# r04z: groups call — lanes x streams per lane (measurement build)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04z}
mkdir -p $OUT
for rep in 1 2; do for v in "4 2" "4 1" "6 1" "8 1" "6 2"; do set -- $v; PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_GROUP_LANES=$1 PMMG_HIP_LANE_STREAMS=$2 timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_l$1_s$2.log 2>&1 && echo "lanes=$1 streams=$2 $(grep -o '"ms_per_group_groups_call": [0-9.]*' $OUT/bench_l$1_s$2.log)" || exit 1; done; done
