python3 tools/gpu_job.py --tag r05h \
 "tracepy tools/groups_only.py --no-parity" \
 "py tools/groups_only.py --no-parity"
