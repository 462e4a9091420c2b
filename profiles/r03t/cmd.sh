#!/bin/bash
# r03t: hit-kind tests (incl. surface walks from one far seed), shard GPU
# tests, then the opt-in cfg5 full-size halo split on one GPU
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03t}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_hits.py tests/test_shard.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& echo "pytest ok" \
&& PMMG_TEST_CFG5=1 timeout -k 10 900 python -u -m pytest "tests/test_shard.py::test_halo_shards_gpu_cfg5_full_size" -x -v -s --timeout 850 --timeout-method thread > $OUT/pytest_cfg5.log 2>&1 \
&& echo "cfg5 ok" && tail -15 $OUT/pytest_cfg5.log
