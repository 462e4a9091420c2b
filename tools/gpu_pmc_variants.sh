#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) over tools/sweep.py, one
# module variant per run:   TAG=x VARIANTS="sol=none;sol=all" bash tools/gpu_pmc_variants.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcv}
mkdir -p $OUT
IFS=';' read -ra VS <<< "${VARIANTS:-sol=none;sol=all}"
if [ -n "$SETS_OVERRIDE" ]; then IFS=';' read -ra SETS <<< "$SETS_OVERRIDE"; else SETS=("FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"); fi
vi=0
for v in "${VS[@]}"; do
  vi=$((vi+1))
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/v${vi}/p$i -o run --output-format csv -- python3 -u tools/sweep.py --config ${CONFIG:-cfg4} --variants "$v" --rounds 1 --steps 1 > $OUT/v${vi}_p$i.log 2>&1 || { echo "variant $v pass $i failed"; exit 1; }
  done
  echo "variant $vi ($v) ok"
done
