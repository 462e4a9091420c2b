M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06zd \
 "tracepy tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 6" \
 "tracepy $M PMMG_HIP_BDYWAVE=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 6"
for v in "" "PMMG_HIP_VOLWAIT=1" "PMMG_HIP_BDYWAVE=1 PMMG_HIP_VOLWAIT=1" "PMMG_HIP_BDYFIRST=1" "PMMG_HIP_BDYWAVE=1 PMMG_HIP_BDYFIRST=1"; do
  python3 tools/gpu_job.py --tag r06zd/v "py $M $v tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 10" || exit 1
  echo "== $v" >> gpurun_out/r06zd/variants.txt; grep "^{'rank'" gpurun_out/r06zd/v/py.log >> gpurun_out/r06zd/variants.txt
done
