M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06o \
 "pytest tests/test_gpu_snapshot.py tests/test_gpu_hits.py tests/test_gpu_parity.py tests/test_gpu_edge.py -m gpu -q" \
 "py $M tools/snap_only.py cfg4 5" \
 "py $M PMMG_HIP_SNAPGLOBAL=1 tools/snap_only.py cfg4 5" \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06o/wt_solo.bin tools/surface_solo.py --steps 3 --env WAVETIME=1" \
 "sweep --config cfg4 --rounds 2 --steps 5 --variants TPC=8" \
 "tracepy tools/snap_only.py cfg4 3"
