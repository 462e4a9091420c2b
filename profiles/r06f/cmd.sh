python3 tools/gpu_job.py --tag r06f \
 "py tools/groups_probe.py --rounds 2 --variants base;big_auto;big_noauto;host;streams1;streams2;keepstreams1;alloc16"
