#!/bin/bash
# r04a: the volume kernel's bound model.
# Per-query L1->L2 read requests, their latency, L1 accesses, L2 hits / misses
# and fabric requests, TA / TD busy and the wave-instruction counts of k_vol,
# for the full kernel, the walk alone (no solutions), chunks of 64 queries in
# Morton order (L2 locality) and the Mmg-like numbering in input order
# (locality loss).  One rocprofv3 --pmc run per (variant, counter set).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r04a} VARIANTS="sort=0;sort=0,sol=none;sort=0,perm=rods6;sort=0,perm=mmg" \
SETS_OVERRIDE="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE;TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE;TD_TD_BUSY_sum TD_TC_STALL_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
bash tools/gpu_pmc_variants.sh
