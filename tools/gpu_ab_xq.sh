#!/bin/bash
# A/B of two builds of the module in alternating processes (sweep.py, cfg4)
set -o pipefail
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 200 python -u tools/sweep.py --config cfg4 --variants "${VARIANTS:-sol=all;packed=1}" --rounds 2 > $OUT/a$r.txt 2>&1 || exit 1
  timeout -k 10 200 env PMMG_HIP_SO=${ALT_SO} python -u tools/sweep.py --config cfg4 --variants "${VARIANTS:-sol=all;packed=1}" --rounds 2 > $OUT/b$r.txt 2>&1 || exit 1
done
