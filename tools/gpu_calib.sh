#!/bin/bash
# FETCH_SIZE calibration on the box: tools/calib/fetch_calib (known-byte read
# patterns) plain, then one rocprofv3 --pmc pass per counter set.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-calib}
mkdir -p $OUT
timeout -k 10 120 ./tools/calib/fetch_calib > $OUT/calib.txt 2>&1 || { echo "calib run failed"; exit 1; }
i=0
for set in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_DRAM_sum" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- ./tools/calib/fetch_calib > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok: $set"
done
