set -o pipefail
mkdir -p gpurun_out/r06j
timeout -k 10 120 ./tools/calib/atomic_same > gpurun_out/r06j/atomic_same.txt 2>&1 && \
python3 tools/gpu_job.py --tag r06j \
 "py GPU_MAX_HW_QUEUES=16 tools/groups_probe.py --rounds 3 --variants base;big_auto" \
 "sweep --config cfg4 --rounds 2 --steps 5 --variants TPC=8;SEEDNOATOM=1"
