#!/bin/bash
# GPU session for the halo-sharded background: shard parity
# tests, cfg5 as one group on one GPU, and 2-rank halo splits rehearsed on the
# one GPU of the box (gloo host collectives, both ranks on cuda:0).  Each GPU
# step has its own time limit; steps are chained with &&.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-halo}
mkdir -p $OUT
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533"
timeout -k 10 200 python -u -m pytest tests/test_shard.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_shard.log 2>&1 \
&& echo "shard tests ok" \
&& timeout -k 10 300 python -u bench.py --config cfg3 --shard halo --no-cpu-baseline --steps 5 --warmup 2 > $OUT/cfg3_halo1.json 2> $OUT/cfg3_halo1.err \
&& echo "cfg3 halo x1 ok" && cat $OUT/cfg3_halo1.json \
&& PMMG_BENCH_BACKEND=gloo timeout -k 10 300 $RUN bench.py --gpus 2 --config cfg3 --shard halo --steps 5 --warmup 2 > $OUT/cfg3_halo2.json 2> $OUT/cfg3_halo2.err \
&& echo "cfg3 halo x2 ok" && cat $OUT/cfg3_halo2.json \
&& timeout -k 10 400 python -u bench.py --config cfg5 --no-cpu-baseline --no-snapshot --steps 5 --warmup 2 > $OUT/cfg5_group.json 2> $OUT/cfg5_group.err \
&& echo "cfg5 group ok" && cat $OUT/cfg5_group.json \
&& PMMG_BENCH_BACKEND=gloo timeout -k 10 500 $RUN bench.py --gpus 2 --config cfg5 --shard halo --steps 5 --warmup 2 > $OUT/cfg5_halo2.json 2> $OUT/cfg5_halo2.err \
&& echo "cfg5 halo x2 ok" && cat $OUT/cfg5_halo2.json
