python3 tools/gpu_job.py --tag r05e \
 "pytest tests/test_gpu_fallback_scale.py tests/test_gpu_records.py tests/test_gpu_hits.py tests/test_gpu_parity.py tests/test_gpu_carry.py tests/test_gpu_groups.py tests/test_gpu_comm.py -rP" \
 "py tools/host_mode.py --config cfg4 --reps 1" \
 "sweep --config cfg4 --variants sort=0;perm=shuffle;perm=shuffle,packed=1,packpass=2 --rounds 2 --steps 3"
