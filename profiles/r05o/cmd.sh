python3 tools/gpu_job.py --tag r05o \
 "pytest tests/test_gpu_configs.py::test_cfg3_shuffled_numbering_auto_order tests/test_gpu_configs.py::test_cfg3_full_size_every_point tests/test_gpu_groups.py tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_carry.py tests/test_gpu_records.py tests/test_shard.py -rP" \
 "tracepy tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0,7 --steps 10" \
 "sweep --config cfg4 --variants sort=0;perm=shuffle --rounds 2 --steps 3" \
 "py tools/groups_only.py --no-parity"
