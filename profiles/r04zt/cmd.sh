#!/bin/bash
# r04zt: is the 8-way rank's surface branch (0.44 ms for 75k points) a tail
# of long walks?  maxstep variants (measurement of the cap only)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04zt}
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10 --variants ";MAXSTEP=256;MAXSTEP=64;MAXSTEP=32" > $OUT/shard.txt 2>&1 \
&& grep -o "'variant'[^}]*" $OUT/shard.txt | sed -e "s/'world.*'nbdy_exhaust'/ nbdy_exhaust/" -e "s/'points.*'ms_total'/ ms_total/"
