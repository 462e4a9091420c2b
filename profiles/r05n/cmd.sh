python3 tools/gpu_job.py --tag r05n \
 "pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_hits.py tests/test_gpu_carry.py tests/test_gpu_groups.py tests/test_gpu_records.py -rP" \
 "tracepy tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_BDYBPX=64 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_SRFSOLO=0 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "sweep --config cfg4 --variants sort=0;perm=mmg;perm=shuffle --rounds 2 --steps 3" \
 "py tools/groups_only.py --no-parity"
