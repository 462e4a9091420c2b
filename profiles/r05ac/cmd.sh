python3 tools/gpu_job.py --tag r05ac \
 "pytest tests/test_gpu_configs.py::test_cfg3_shuffled_numbering_auto_order tests/test_gpu_configs.py::test_cfg3_full_size_every_point tests/test_gpu_parity.py -rP" \
 "sweep --config cfg4 --variants sort=0;QNT=0,sort=0 --rounds 3 --steps 3" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_QNT=0 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
