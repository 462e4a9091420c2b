#!/bin/bash
# r04t: snapshot — the count's atomics with one round trip per wave (sorted
# wave keys); snapshot tests; kernel trace of the snapshot alone at cfg4
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04t}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_snapshot.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -2 $OUT/pytest.log \
&& timeout -k 10 300 python3 -u tools/snap_only.py cfg4 4 > $OUT/snap.txt 2>&1 \
&& cat $OUT/snap.txt \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u tools/snap_only.py cfg4 3 > $OUT/trace.log 2>&1 \
&& echo trace ok
