python3 tools/gpu_job.py --tag r06za \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;SEEDSORT=1;PAD=268435456;SEEDSORT=1,PAD=268435456" \
 "pmc cfg4 PAD=268435456 'TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE'" \
 "pmc cfg4 TPC=8 'TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE'"
