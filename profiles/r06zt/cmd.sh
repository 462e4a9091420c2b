set -o pipefail
export TMPDIR=/tmp
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06zt \
 "sweep --config cfg4 --rounds 5 --steps 5 --variants TPC=8;SRFSOLO=0,BDYFIRST=1" \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants perm=mmg;perm=mmg,SRFSOLO=0,BDYFIRST=1;perm=shuffle;perm=shuffle,SRFSOLO=0,BDYFIRST=1" \
 "sweep --config cfg3 --rounds 3 --steps 5 --variants TPC=8;SRFSOLO=0,BDYFIRST=1" \
 "py $M PMMG_HIP_SRFSOLO=0 PMMG_HIP_BDYFIRST=1 tools/groups_only.py --no-parity" \
 "py $M tools/groups_only.py --no-parity" \
 "py $M PMMG_HIP_SRFSOLO=0 PMMG_HIP_BDYFIRST=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0,1,2,3,4,5,6,7 --steps 20"
