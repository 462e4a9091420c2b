M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06p \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;BDYWAVE=1" \
 "sweep --config cfg3 --rounds 2 --steps 5 --variants TPC=8;BDYWAVE=1" \
 "py $M tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_BDYWAVE=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants TPC=8"
