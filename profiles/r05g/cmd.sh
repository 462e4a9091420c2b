python3 tools/gpu_job.py --tag r05g \
 "pytest tests/test_gpu_records.py tests/test_gpu_hits.py tests/test_gpu_parity.py tests/test_gpu_carry.py tests/test_gpu_groups.py tests/test_gpu_comm.py -rP" \
 "py tools/host_mode.py --config cfg4 --reps 1" \
 "sweep --config cfg4 --variants sort=0;perm=shuffle;perm=shuffle,packed=1,packpass=2;perm=shuffle,packed=1,packpass=2,recout=1 --rounds 2 --steps 3" \
 "py tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=8 PMMG_HIP_GROUP_LANES=8 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=16 PMMG_HIP_GROUP_LANES=8 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=16 PMMG_HIP_GROUP_LANES=12 tools/groups_only.py --no-parity" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
