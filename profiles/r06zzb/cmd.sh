set -o pipefail
export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r06zzb "pytest tests -m gpu -q" "bench --steps 20 --warmup 3 --no-cpu-baseline" && \
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06zzb/smoke.txt 2>&1
