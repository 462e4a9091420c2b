B="--steps 20 --warmup 3 --no-host-mode --no-snapshot --no-quality --no-graded --no-groups --no-surface-solo --no-cpu-baseline"
python3 tools/gpu_job.py --tag r05ah \
 "pytest tests/test_gpu_configs.py::test_cfg3_shuffled_numbering_auto_order tests/test_gpu_configs.py::test_cfg3_full_size_every_point tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_groups.py tests/test_shard.py -rP" \
 "bench $B --config cfg3" \
 "bench $B --config cfg3 --sort off --no-shuffled" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "bench --steps 5 --warmup 2 --no-host-mode --no-snapshot --no-quality --no-graded --no-groups --no-surface-solo --no-cpu-baseline"
