python3 tools/gpu_job.py --tag r06e \
 "pytest tests/test_gpu_hits.py tests/test_gpu_comm.py tests/test_c_abi.py -q"
