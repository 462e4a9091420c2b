set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06zl "pytest tests -m gpu -q -x" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0,1,2,3,4,5,6,7 --steps 20" \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;HOSTORDER=0" \
 "py tools/groups_only.py" \
 "tracepy tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 4"
