python3 tools/gpu_job.py --tag r05an \
 "sweep --config cfg4 --variants perm=shuffle;perm=shuffle,packed=1,recout=1;sort=0 --rounds 5 --steps 3"
