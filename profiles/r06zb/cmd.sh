python3 tools/gpu_job.py --tag r06zb \
 "tracepy tools/snap_only.py cfg4 3" \
 "pmcpy k_ 'SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE' tools/snap_only.py cfg4 1" \
 "pmcpy k_ 'TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE' tools/snap_only.py cfg4 1" \
 "pmcpy k_ 'SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE' tools/snap_only.py cfg4 1"
