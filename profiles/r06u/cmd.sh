set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06u "pytest tests -m gpu -q" "bench" && \
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06u/smoke.txt 2>&1 && \
TAG=r06u bash tools/gpu_prof.sh
