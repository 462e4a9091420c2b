#!/bin/bash
# r04e: the volume kernel at 5 waves per SIMD (amdgpu_waves_per_eu(5), 8
# VGPRs spilled) against 4; then a kernel trace of the product bench step
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04e}
mkdir -p $OUT
W5=so=parmmg_amd/libpmmg_hip_measure_w5.so
timeout -k 10 800 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0;$W5,sort=0;sort=0,DMA=0;$W5,sort=0,DMA=0" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-mode --no-shuffled --no-quality --no-snapshot --no-graded --no-surface-solo --steps 5 --warmup 2 > $OUT/prof_bench.log 2>&1 \
&& tail -3 $OUT/prof_bench.log
