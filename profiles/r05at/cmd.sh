M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r05at \
 "sweep --config cfg4 --variants sort=0;BDYBPX=256,sort=0;BDYBPX=1024,sort=0;BDYBPX=2048,sort=0 --rounds 3 --steps 3" \
 "py $M tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_BDYBPX=64 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_BDYBPX=128 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
