set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06zr \
 "sweep --config cfg4 --rounds 4 --steps 5 --variants TPC=6;TPC=8;TPC=10;TPC=12"
