python3 tools/gpu_job.py --tag r05aj \
 "sweep --config cfg4 --variants sort=0;perm=mmg;perm=mmg,XCDRUN=16;perm=mmg,XCDRUN=32;perm=mmg,XCDRUN=128;XCDRUN=32,sort=0;XCDRUN=128,sort=0 --rounds 2 --steps 3"
