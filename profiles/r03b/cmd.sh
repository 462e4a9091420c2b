#!/bin/bash
# r03b: CPU share probe, the changed GPU tests, a quick cfg4 bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03b
mkdir -p $OUT
{ echo "nproc=$(nproc)"; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/status | grep -i cpus_allowed_list; } > $OUT/cpu_probe.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_snapshot.py tests/test_gpu_hits.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& TAG=r03b BENCH_CONFIGS="cfg4" bash tools/gpu_bench_quick.sh
