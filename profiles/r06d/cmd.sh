python3 tools/gpu_job.py --tag r06d \
 "pytest tests/test_gpu_configs.py -k split -q" \
 "bench"
