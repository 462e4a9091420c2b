#!/bin/bash
# r03u: the opt-in cfg5 full-size halo split on one GPU, with stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03u}
mkdir -p $OUT
PMMG_TEST_CFG5=1 timeout -k 10 900 python -u -m pytest "tests/test_shard.py::test_halo_shards_gpu_cfg5_full_size" -x -v -s --timeout 850 --timeout-method thread > $OUT/pytest_cfg5.log 2>&1
rc=$?; grep -E "^cfg5|^group run|^part|^same|^checked" $OUT/pytest_cfg5.log; exit $rc
