M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06x \
 "pytest tests/test_gpu_hits.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge.py tests/test_gpu_records.py tests/test_gpu_groups.py tests/test_gpu_fallback_scale.py -m gpu -q" \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06x/wt_coop4.bin tools/surface_solo.py --steps 3 --env WAVETIME=1,BDYWAVE=1" \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06x/wt_coop3.bin tools/surface_solo.py --steps 3 --env WAVETIME=1,BDYWAVE=1,BDYOCC4=0" \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06x/wt_lane.bin tools/surface_solo.py --steps 3 --env WAVETIME=1,BDYWAVE=1,BDYLANE=1" \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;BDYOCC4=0;BDYLANE=1" \
 "py $M tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_BDYLANE=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
