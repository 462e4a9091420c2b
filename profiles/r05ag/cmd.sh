B="--steps 20 --warmup 3 --no-host-mode --no-snapshot --no-quality --no-graded --no-groups --no-shuffled --no-surface-solo --no-cpu-baseline --config cfg3"
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r05ag \
 "bench $M PMMG_HIP_STREAM3=1 $B" \
 "bench $M PMMG_HIP_STREAM3=0 $B" \
 "bench $M PMMG_HIP_STREAM3=1 $B" \
 "bench $M PMMG_HIP_STREAM3=0 $B" \
 "bench $M PMMG_HIP_STREAM3=0 $B --sort off"
