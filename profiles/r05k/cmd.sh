python3 tools/gpu_job.py --tag r05k \
 "tracepy tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=8 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=8 PMMG_HIP_GROUP_LANES=5 tools/groups_only.py --no-parity" \
 "py PMMG_HIP_GROUP_LANES=5 tools/groups_only.py --no-parity" \
 "py GPU_MAX_HW_QUEUES=12 PMMG_HIP_GROUP_LANES=6 tools/groups_only.py --no-parity" \
 "py PMMG_HIP_GROUP_LANES=8 tools/groups_only.py --no-parity" \
 "py PMMG_HIP_GROUP_LANES=10 tools/groups_only.py --no-parity"
