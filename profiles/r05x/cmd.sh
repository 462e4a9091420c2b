B="--steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-snapshot --no-quality --no-graded --no-shuffled --no-surface-solo"
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r05x \
 "bench $M PMMG_HIP_STREAM3=1 $B" \
 "bench $M PMMG_HIP_STREAM3=0 $B" \
 "bench $M PMMG_HIP_STREAM3=2 $B" \
 "py $M PMMG_HIP_STREAM3=0 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_STREAM3=2 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_STREAM3=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
