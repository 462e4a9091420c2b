python3 tools/gpu_job.py --tag r05l \
 "pytest tests/test_gpu_groups.py tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_carry.py tests/test_gpu_configs.py -rP" \
 "py tools/groups_only.py" \
 "py PMMG_HIP_GROUP_LANES=4 tools/groups_only.py --no-parity" \
 "tracepy tools/groups_only.py --no-parity" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
