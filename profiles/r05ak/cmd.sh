M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r05ak \
 "sweep --config cfg4 --variants sort=0;BDYWAVES=5,sort=0;BDYWAVES=6,sort=0 --rounds 3 --steps 3" \
 "py $M tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_BDYWAVES=5 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_BDYWAVES=6 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
