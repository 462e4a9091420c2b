B="--steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-snapshot --no-quality --no-graded --no-groups --no-shuffled"
python3 tools/gpu_job.py --tag r05u \
 "bench PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_NOTREC=1 $B" \
 "bench PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so $B" \
 "bench PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_NOTREC=1 $B" \
 "bench PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so $B" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_NOTREC=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
