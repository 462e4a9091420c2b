#!/bin/bash
# r04c: price VALU and L1 accesses in the walk step (PMMG_HIP_PAD, on the
# previous build kept as libpmmg_hip_measure_base.so), the leaner walk step
# (packed slot map, fused fp32 geometry, fast face pick, 32-bit LDS slots), and
# the XCD run interleave (PMMG_HIP_XCDRUN) on the lattice and the Mmg-like
# numbering — cfg4, measurement builds
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04c}
mkdir -p $OUT
B=so=parmmg_amd/libpmmg_hip_measure_base.so
timeout -k 10 1000 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "$B,sort=0,UROWS=0;$B,sort=0,UROWS=0,PAD=64;$B,sort=0,UROWS=0,PAD=131072;sort=0,UROWS=0;sort=0,UROWS=0,XCDRUN=64;$B,sort=0,UROWS=0,perm=mmg;sort=0,UROWS=0,perm=mmg,XCDRUN=64" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt
