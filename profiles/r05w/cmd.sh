python3 tools/gpu_job.py --tag r05w \
 "bench --steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-snapshot --no-quality --no-graded --no-shuffled --no-surface-solo" \
 "py tools/groups_only.py --no-parity" \
 "bench --steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-snapshot --no-quality --no-graded --no-shuffled --no-surface-solo --sort off"
