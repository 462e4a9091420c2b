python3 tools/gpu_job.py --tag r06w \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06w/wt_default.bin tools/surface_solo.py --steps 3 --env WAVETIME=1,BDYWAVE=1" \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06w/wt_nointerp.bin tools/surface_solo.py --steps 3 --env WAVETIME=1,BDYWAVE=1,BDYNOINTERP=1"
