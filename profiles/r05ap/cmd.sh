M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r05ap \
 "sweep --config cfg4 --variants sort=0;VOLWAIT=1,sort=0;BDYFIRST=1,sort=0;sort=0,so=parmmg_amd/libpmmg_hip_prev.so --rounds 4 --steps 3" \
 "pytest tests/test_gpu_parity.py -x" \
 "sweep --config cfg4 --variants perm=mmg;perm=mmg,VOLWAIT=1 --rounds 3 --steps 3" \
 "py $M tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10" \
 "py $M PMMG_HIP_VOLWAIT=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
