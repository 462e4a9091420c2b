python3 tools/gpu_job.py --tag r06v \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;BDYFIRST=1;BDYFIRST=1,BDYWAVE=1" \
 "sweep --config cfg3 --rounds 2 --steps 5 --variants TPC=8;BDYFIRST=1" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants BDYFIRST=1"
