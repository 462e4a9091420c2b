#!/bin/bash
# counter list of the box + PMC passes over a short cfg4 bench (one pass per run)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "list failed"
TAG=${TAG:-pmc} BENCH_ARGS="--config cfg4 --no-host-mode --no-quality --no-snapshot --no-cpu-baseline" bash tools/gpu_pmc.sh \
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
 "TCC_HIT_sum TCC_MISS_sum" \
 "FETCH_SIZE" \
 "WRITE_SIZE" \
 "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
 "TA_BUSY_avr TA_TA_BUSY_sum" \
 "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
