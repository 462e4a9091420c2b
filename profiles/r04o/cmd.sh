#!/bin/bash
# r04o: kernel trace + FETCH / WRITE passes of the bench step (tools/gpu_prof.sh),
# then a seed-grid density sweep (TPC)
set -o pipefail
export TMPDIR=/tmp
TAG=r04o bash tools/gpu_prof.sh \
&& timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0;sort=0,TPC=12;sort=0,TPC=16;sort=0,TPC=6" > gpurun_out/r04o/sweep_tpc.txt 2>&1 \
&& cat gpurun_out/r04o/sweep_tpc.txt
