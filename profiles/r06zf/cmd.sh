set -o pipefail
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
for v in "PMMG_HIP_EVFLAGS=0" "PMMG_HIP_EVFLAGS=1" "PMMG_HIP_EVFLAGS=2" "PMMG_HIP_EVFLAGS=0" "PMMG_HIP_EVFLAGS=1"; do
  python3 tools/gpu_job.py --tag r06zf/v "py $M $v tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20" || exit 1
  echo "== $v" >> gpurun_out/r06zf/variants.txt; grep "^{'rank'" gpurun_out/r06zf/v/py.log >> gpurun_out/r06zf/variants.txt
done
python3 tools/gpu_job.py --tag r06zf \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants EVFLAGS=0;EVFLAGS=1;EVFLAGS=2" \
 "tracepy $M PMMG_HIP_EVFLAGS=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 4"
