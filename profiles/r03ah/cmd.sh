#!/bin/bash
# r03ah: PMC passes over the final round-3 code (cfg4 bench step alone):
# HBM bytes, L1->L2 requests and miss stalls, texture-data busy / stalls
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03ah} BENCH_ARGS="--config cfg4 --no-host-mode --no-quality --no-snapshot --no-shuffled --no-graded --no-surface-solo" bash tools/gpu_pmc.sh \
 "FETCH_SIZE" \
 "WRITE_SIZE" \
 "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
 "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
 "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS"
