python3 tools/gpu_job.py --tag r06s \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;SRFSOLO=0;SRFSOLO=0,BDYWAVE=1;BDYWAVE=1" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants SRFSOLO=0"
