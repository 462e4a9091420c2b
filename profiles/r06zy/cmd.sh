set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06zy \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;SEEDLANES=3;SEEDLANES=2;TPC=6,SEEDLANES=3;TPC=4,SEEDLANES=2"
