python3 tools/gpu_job.py --tag r05d \
 "pytest tests/test_gpu_fallback_scale.py tests/test_gpu_comm.py -rP" \
 "sweep --config cfg4 --variants sort=0;packed=1,sort=0;packed=1,packpass=2,sort=0;seedv0=1,sort=0 --rounds 2 --steps 3" \
 "py tools/host_mode.py --config cfg4 --reps 1" \
 "pmc cfg4 sort=0 'SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES'" \
 "pmc cfg4 packed=1,sort=0 'SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES'" \
 "pmc cfg4 packed=1,packpass=2,sort=0 'SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES'" \
 "pmc cfg4 sort=0 'TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE'" \
 "pmc cfg4 packed=1,sort=0 'TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE'" \
 "pmc cfg4 packed=1,packpass=2,sort=0 'TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE'"
