python3 tools/gpu_job.py --tag r05ad \
 "sweep --config cfg4 --variants sort=0;BDYBPX=256,sort=0;BDYBPX=128,sort=0;BDYBPX=1024,sort=0;SRFSOLO=0,sort=0 --rounds 3 --steps 3"
