set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06zu "pytest tests -m gpu -q" "bench" \
 "py tools/shard_step.py --config cfg4 --world 8 --ranks 0,1,2,3,4,5,6,7 --steps 10" && \
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06zu/smoke.txt 2>&1 && \
TAG=r06zu bash tools/gpu_prof.sh
