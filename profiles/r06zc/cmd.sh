python3 tools/gpu_job.py --tag r06zc \
 "pytest tests/test_gpu_snapshot.py -q" \
 "tracepy tools/snap_only.py cfg4 3" \
 "pmcpy k_ 'SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE' tools/snap_only.py cfg4 1"
