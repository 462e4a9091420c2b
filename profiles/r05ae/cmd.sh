python3 tools/gpu_job.py --tag r05ae \
 "pytest tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_groups.py tests/test_gpu_configs.py::test_cfg3_shuffled_numbering_auto_order -rP" \
 "sweep --config cfg4 --variants sort=0;perm=mmg;SRFSOLO=0,sort=0 --rounds 3 --steps 3" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
