B="--steps 10 --warmup 2 --no-host-mode --no-snapshot --no-quality --no-graded --no-groups --no-shuffled --no-surface-solo --cpu-baseline-seconds 10"
python3 tools/gpu_job.py --tag r05af \
 "bench $B --config cfg2" \
 "bench $B --config cfg3" \
 "bench --steps 5 --warmup 1 --no-host-mode --no-snapshot --no-quality --no-graded --no-groups --no-shuffled --no-surface-solo --no-cpu-baseline --config cfg5"
