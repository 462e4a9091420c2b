python3 tools/gpu_job.py --tag r06k \
 "pytest tests -m gpu -q" \
 "sweep --config cfg4 --rounds 2 --steps 5 --variants TPC=8;BDYWAVE=1" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants BDYWAVE=1" \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06k/wt_solo_wave.bin tools/surface_solo.py --steps 3 --env WAVETIME=1,BDYWAVE=1"
