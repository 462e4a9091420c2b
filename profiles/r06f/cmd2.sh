python3 tools/gpu_job.py --tag r06f2 \
 "py tools/groups_probe.py --rounds 2 --variants base;keepstreams1;keepstreams2;keepstreams3;keepstreams4;nullcopy;big_auto" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0,1,2,3,4,5,6,7 --steps 10" \
 "tracepy tools/surface_solo.py --steps 5"
