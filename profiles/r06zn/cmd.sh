set -o pipefail
export TMPDIR=/tmp
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
for v in "PMMG_HIP_TPC=8" "PMMG_HIP_SRFSOLO=0" "PMMG_HIP_HOSTORDER=0" "PMMG_HIP_FUSECONT=0" "PMMG_HIP_TPC=8" "PMMG_HIP_SRFSOLO=0" "PMMG_HIP_HOSTORDER=0" "PMMG_HIP_FUSECONT=0"; do
  python3 tools/gpu_job.py --tag r06zn/v "py $M $v tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20" || exit 1
  echo "== $v" >> gpurun_out/r06zn/variants.txt; grep "^{'rank'" gpurun_out/r06zn/v/py.log >> gpurun_out/r06zn/variants.txt
done
python3 tools/gpu_job.py --tag r06zn \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;SRFSOLO=0;HOSTORDER=0;FUSECONT=0" \
 "py $M PMMG_HIP_FUSECONT=0 tools/groups_only.py --no-parity" \
 "py $M tools/groups_only.py --no-parity" \
 "tracepy $M PMMG_HIP_SRFSOLO=0 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 4"
