python3 tools/gpu_job.py --tag r06a \
 "pytest PMMG_HIP_VOLSPLIT=1 tests/ -m gpu -q" \
 "sweep --config cfg4 --rounds 2 --variants VOLSPLIT=0;VOLSPLIT=1;packed=1,VOLSPLIT=0;packed=1,VOLSPLIT=1;packed=1,PACKPASS=1,VOLSPLIT=1;packed=1,recout=1,VOLSPLIT=1"
