#!/bin/bash
# r04d: LDS-DMA interpolation gathers (96 VGPRs: 5 waves per SIMD) and the XCD
# run length — GPU parity suites, then a cfg4 sweep (measurement build)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04d}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -3 $OUT/pytest.log \
&& timeout -k 10 1000 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0,DMA=0,XCDRUN=0;sort=0,DMA=0;sort=0;sort=0,XCDRUN=16;sort=0,XCDRUN=256;sort=0,perm=mmg;sort=0,perm=mmg,XCDRUN=16" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt
