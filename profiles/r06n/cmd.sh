python3 tools/gpu_job.py --tag r06n \
 "pytest tests -m gpu -q" \
 "py tools/groups_probe.py --rounds 3 --variants base;big_auto;host" \
 "bench"
