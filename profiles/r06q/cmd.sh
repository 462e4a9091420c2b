python3 tools/gpu_job.py --tag r06q \
 "pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_hits.py tests/test_gpu_records.py -m gpu -q" \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;PAD=268435456" \
 "sweep --config cfg3 --rounds 2 --steps 5 --variants TPC=8;PAD=268435456"
