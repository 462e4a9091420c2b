python3 tools/gpu_job.py --tag r05ar \
 "pytest tests/ -m gpu -rP" \
 "py -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench"
