python3 tools/gpu_job.py --tag r05f \
 "py tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=8 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=8 PMMG_HIP_GROUP_LANES=8 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=16 PMMG_HIP_GROUP_LANES=8 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=16 PMMG_HIP_GROUP_LANES=5 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=16 PMMG_HIP_GROUP_LANES=10 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=16 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
