export TMPDIR=/tmp
python3 tools/gpu_job.py --tag r05ao \
 "pytest tests/ -m gpu" \
 "sweep --config cfg4 --variants sort=0;sort=0,so=parmmg_amd/libpmmg_hip_prev.so --rounds 5 --steps 3" \
 && mkdir -p gpurun_out/r05ao \
 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ao/trace -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-mode --no-shuffled --no-quality --no-snapshot --no-graded --no-surface-solo --no-groups --steps 5 --warmup 1 > gpurun_out/r05ao/trace.log 2>&1
