set -o pipefail
export TMPDIR=/tmp
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06zz \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;NOFB=1" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants NOFB=1"
