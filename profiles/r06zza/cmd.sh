set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06zza "pytest tests -m gpu -q -x" \
 "sweep --config cfg4 --rounds 4 --steps 5 --variants TPC=8;SRFSOLO=0,BDYFIRST=1" \
 "sweep --config cfg4 --rounds 2 --steps 5 --variants perm=mmg;perm=mmg,SRFSOLO=0,BDYFIRST=1" \
 "sweep --config cfg3 --rounds 2 --steps 5 --variants TPC=8;SRFSOLO=0,BDYFIRST=1" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20 --variants TPC=8;SRFSOLO=0,BDYFIRST=1;TPC=8" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants SRFSOLO=0,BDYFIRST=1"
