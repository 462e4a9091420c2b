#!/bin/bash
# r03o: surface list by rocPRIM select, dynamic work claiming in k_bdy:
# parity tests, then the preparation knobs (bbox / axis-histogram sampling,
# sampled records per seed run)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03o}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_hits.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& timeout -k 10 700 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 4 --variants "sort=0;BBOX=64,HIST=256;SEEDLANES=2;SEEDLANES=1;BBOX=64,HIST=256,SEEDLANES=1" > $OUT/sweep_prep.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep_prep.txt
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok" && cat $OUT/bench.json
