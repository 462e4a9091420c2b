set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06zw \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20 --variants TPC=8;BDYSPLIT=1;SRFSOLO=0;SRFSOLO=0,BDYFIRST=1;BDYWAVE=1;EVFLAGS=1;SRFPRIO=1;TPC=8" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 1,5 --steps 20 --variants TPC=8;BDYSPLIT=1;SRFSOLO=0;SRFSOLO=0,BDYFIRST=1;TPC=8" \
 "tracepy tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 4 --variants BDYSPLIT=1"
