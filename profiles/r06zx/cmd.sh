set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06zx \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants XCDRUN=32;XCDRUN=64;XCDRUN=128;XCDRUN=256" \
 "sweep --config cfg4 --rounds 2 --steps 5 --variants perm=mmg,XCDRUN=32;perm=mmg,XCDRUN=64;perm=mmg,XCDRUN=128"
