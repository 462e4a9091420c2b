set -o pipefail
export TMPDIR=/tmp
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06zs \
 "sweep --config cfg4 --rounds 4 --steps 5 --variants TPC=8;SRFSOLO=0;SRFSOLO=0,BDYFIRST=1" \
 "tracepy $M PMMG_HIP_SRFSOLO=0 PMMG_HIP_BDYFIRST=1 tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants TPC=8" \
 "py $M PMMG_HIP_SRFSOLO=0 PMMG_HIP_BDYFIRST=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20" \
 "py $M tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20"
