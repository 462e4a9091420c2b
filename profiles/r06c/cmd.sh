python3 tools/gpu_job.py --tag r06c \
 "pytest PMMG_HIP_VOLSPLIT=1 PMMG_HIP_VOLCHUNKS=3 tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_records.py -q" \
 "sweep --config cfg4 --rounds 2 --variants VOLSPLIT=0;VOLSPLIT=1,VOLCHUNKS=4;VOLSPLIT=1,VOLCHUNKS=8;packed=1,PACKPASS=1,VOLSPLIT=1,VOLCHUNKS=4;packed=1,PACKPASS=1,VOLSPLIT=1,VOLCHUNKS=8;packed=1,PACKPASS=1,VOLSPLIT=1,VOLCHUNKS=8,IXCDRUN=0;packed=1,PACKPASS=1,VOLSPLIT=0"
