M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06i \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06i/wt_solo.bin tools/surface_solo.py --steps 3 --env WAVETIME=1" \
 "py $M PMMG_HIP_WAVETIME=1 PMMG_HIP_WAVETIME_OUT=gpurun_out/r06i/wt_rank0.bin tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 3" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants TPC=8" \
 "py tools/groups_probe.py --rounds 2 --variants base;big_auto;big_noauto" \
 "GPU_MAX_HW_QUEUES=16 py tools/groups_probe.py --rounds 2 --variants base;big_auto"
