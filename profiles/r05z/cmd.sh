B="--steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-snapshot --no-quality --no-graded --no-shuffled --no-surface-solo"
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r05z \
 "bench $B --sort on" \
 "bench $M PMMG_HIP_STREAM3=0 $B" \
 "bench $B --config cfg3" \
 "bench $B --config cfg3 --sort off" \
 "bench $B"
