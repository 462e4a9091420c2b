python3 tools/gpu_job.py --tag r05p \
 "pytest tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_edge.py tests/test_gpu_configs.py::test_cfg3_shuffled_numbering_auto_order tests/test_gpu_configs.py::test_cfg4_full_size_visit_range tests/test_gpu_groups.py tests/test_shard.py -rP" \
 "tracepy tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0,7 --steps 10" \
 "sweep --config cfg4 --variants sort=0;perm=shuffle --rounds 2 --steps 3" \
 "bench --steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-snapshot --no-quality --no-graded --no-groups --no-shuffled"
