python3 tools/gpu_job.py --tag r06h \
 "pmcpy k_bdy 'SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS' tools/surface_solo.py --steps 2" \
 "pmcpy k_bdy 'TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD' tools/surface_solo.py --steps 2" \
 "sweep --config cfg4 --rounds 2 --steps 5 --variants TPC=8;TPC=8,SEEDV0=1;TPC=6,SEEDV0=1;TPC=4,SEEDV0=1;TPC=4"
