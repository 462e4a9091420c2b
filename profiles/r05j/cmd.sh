python3 tools/gpu_job.py --tag r05j \
 "pytest tests/ -m gpu -rP" \
 "sweep --config cfg4 --variants sort=0;perm=mmg;perm=shuffle;perm=shuffle,packed=1,recout=1 --rounds 2 --steps 3" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py tools/groups_only.py --no-parity" \
 "py PMMG_HIP_GROUP_LANES=6 tools/groups_only.py --no-parity"
