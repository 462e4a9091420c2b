set -o pipefail
export TMPDIR=/tmp
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
for v in "PMMG_HIP_SRFPRIO=0" "PMMG_HIP_SRFPRIO=1" "PMMG_HIP_SRFPRIO=0" "PMMG_HIP_SRFPRIO=1"; do
  python3 tools/gpu_job.py --tag r06zm/v "py $M $v tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20" || exit 1
  echo "== $v" >> gpurun_out/r06zm/variants.txt; grep "^{'rank'" gpurun_out/r06zm/v/py.log >> gpurun_out/r06zm/variants.txt
done
python3 tools/gpu_job.py --tag r06zm \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants SRFPRIO=0;SRFPRIO=1" \
 "py $M PMMG_HIP_SRFPRIO=1 tools/groups_after_big.py cfg3" \
 "py $M PMMG_HIP_SRFPRIO=0 tools/groups_after_big.py cfg3" \
 "tracepy $M PMMG_HIP_SRFPRIO=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 4"
