#!/bin/bash
# r03n: the full GPU suite, the default bench line (CPU baseline + parity),
# a kernel-trace profile of the bench step, then a 2-rank rehearsal of the
# multi-GPU bench (both ranks on the box's one GPU, gloo host collectives)
# with the split-mode parity check.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03n}
mkdir -p $OUT
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
&& echo "pytest ok" \
&& timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
&& echo "bench ok" && cat $OUT/bench.json \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-graded --steps 5 --warmup 2 > $OUT/prof_bench.log 2>&1 \
&& echo "rocprof ok" \
&& PMMG_BENCH_BACKEND=gloo timeout -k 10 600 $RUN bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/cfg4_rcb2_gloo.json 2> $OUT/cfg4_rcb2_gloo.err \
&& echo "gloo x2 ok" && cat $OUT/cfg4_rcb2_gloo.json
