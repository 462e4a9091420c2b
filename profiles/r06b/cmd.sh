set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06b \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants VOLSPLIT=1" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants packed=1,PACKPASS=1,VOLSPLIT=1" && \
TAG=r06b VARIANTS="VOLSPLIT=1;packed=1,PACKPASS=1,VOLSPLIT=1" \
SETS_OVERRIDE="FETCH_SIZE;WRITE_SIZE;TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
bash tools/gpu_pmc_variants.sh && for v in 1 2; do python3 tools/pmc_table.py gpurun_out/r06b/v$v k_vol > gpurun_out/r06b/pmc_v$v.txt; done
