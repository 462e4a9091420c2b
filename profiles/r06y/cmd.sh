python3 tools/gpu_job.py --tag r06y \
 "pmc cfg4 TPC=8 'TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum'" \
 "pmc cfg4 TPC=8 'TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE'"
