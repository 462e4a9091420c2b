#!/bin/bash
# r04u: snapshot (no-return count atomics, slots from cursors in the
# scatter, persistent match, boundary candidate lists): tests + trace; groups
# leg with 1 vs 2 streams per lane (measurement build)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04u}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_snapshot.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log \
&& timeout -k 10 300 python3 -u tools/snap_only.py cfg4 4 > $OUT/snap.txt 2>&1 \
&& cat $OUT/snap.txt \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u tools/snap_only.py cfg4 3 > $OUT/trace.log 2>&1 \
&& echo trace ok \
&& for ls in 3 2 1 3 2 1; do PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_LANE_STREAMS=$ls timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2_ls$ls.log 2>&1 && echo "lane_streams=$ls $(grep -o '"ms_per_group_groups_call": [0-9.]*' $OUT/bench_cfg2_ls$ls.log)" || exit 1; done
