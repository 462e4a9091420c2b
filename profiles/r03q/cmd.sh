#!/bin/bash
# r03q: the surface branch alone under the kernel tracer
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03q}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_srf -o run --output-format csv -- python3 -u tools/surface_solo.py --steps 5 > $OUT/surface_solo.log 2>&1 \
&& echo "prof ok" && cat $OUT/surface_solo.log
