#!/bin/bash
# r04b: the unique-vertex row image in k_vol — GPU parity suites, cfg4 A/B
# against the per-vertex gathers (PMMG_HIP_UROWS=0, measurement build), and the
# L1 access count of both
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04b}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -3 $OUT/pytest.log \
&& timeout -k 10 600 python3 -u tools/sweep.py --config cfg4 --rounds 3 --steps 4 --variants "sort=0,UROWS=0;sort=0" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& TAG=${TAG:-r04b}/pmc VARIANTS="sort=0,UROWS=0;sort=0" SETS_OVERRIDE="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES" bash tools/gpu_pmc_variants.sh \
&& python3 tools/pmc_table.py $OUT/pmc/v1 "k_vol<" && python3 tools/pmc_table.py $OUT/pmc/v2 "k_vol<"
