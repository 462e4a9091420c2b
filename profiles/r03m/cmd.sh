#!/bin/bash
# r03m: staged Morton path (records in processing order + k_vol_unpermute):
# parity tests, then the order sweep
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03m}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 1 --steps 4 --variants "sort=0;perm=mmg;perm=mmg,sort=0;perm=shuffle;perm=shuffle,STAGE=2;sort=1,STAGE=3;perm=mmg,sort=1,STAGE=3" > $OUT/sweep.txt 2>&1 \
&& echo "sweep ok" && cat $OUT/sweep.txt
