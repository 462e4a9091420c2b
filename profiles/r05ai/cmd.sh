python3 tools/gpu_job.py --tag r05ai \
 "pytest tests/ -m gpu -rP" \
 "py -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench" && TAG=r05ai/prof bash tools/gpu_prof.sh
