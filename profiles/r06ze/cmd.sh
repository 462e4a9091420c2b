set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06ze
mkdir -p $OUT
python3 tools/gpu_job.py --tag r06ze "py tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 10" \
 "pytest tests/test_gpu_parity.py tests/test_gpu_hits.py -q" && \
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $OUT/hip -o run --output-format csv -- python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 4 > $OUT/hiptrace.log 2>&1
