#!/bin/bash
# r04h: radix sort ranking tiles in LDS (coalesced runs) + first digit table
# from the key kernel; small-group threshold 2^20; the groups call (tests,
# bench leg at 1-4 lanes); cfg4 order / layout variants; PMC of k_vol in
# input order vs Morton-binned (shuffled numbering)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04h}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& tail -3 $OUT/pytest.log \
&& timeout -k 10 900 python3 -u tools/sweep.py --config cfg4 --rounds 2 --steps 3 --variants "sort=0;perm=shuffle;perm=mmg;perm=mmg,sort=0;packed=1;sol=none" > $OUT/sweep.txt 2>&1 \
&& cat $OUT/sweep.txt \
&& for L in 1 2 3 4; do PMMG_HIP_GROUP_LANES=$L timeout -k 10 300 python3 -u bench.py --config cfg2 --steps 5 --warmup 2 --no-cpu-baseline --no-host-mode --no-quality --no-snapshot --no-shuffled --no-surface-solo > $OUT/bench_cfg2_lanes$L.log 2>&1 || exit 1; grep -o '"groups": {[^}]*}' $OUT/bench_cfg2_lanes$L.log; done \
&& for v in "sort=0" "perm=shuffle"; do i=0; for set in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do i=$((i+1)); timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_${v//=/_}/p$i -o run --output-format csv -- python3 -u tools/sweep.py --config cfg4 --variants "$v" --rounds 1 --steps 1 > $OUT/pmc_${v//=/_}_p$i.log 2>&1 || exit 1; done; python3 tools/pmc_table.py $OUT/pmc_${v//=/_} "k_vol<" ; done
