python3 tools/gpu_job.py --tag r06g \
 "py tools/groups_probe.py --rounds 2 --variants base;big_auto;host;nullcopy;keepstreams1"
