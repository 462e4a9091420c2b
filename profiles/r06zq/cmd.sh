set -o pipefail
export TMPDIR=/tmp
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06zq \
 "pytest tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_configs.py -q -x" \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06zq/wt_touch.bin tools/surface_solo.py --steps 3 --env WAVETIME=1" \
 "py PMMG_HIP_WAVETIME_OUT=gpurun_out/r06zq/wt_notouch.bin tools/surface_solo.py --steps 3 --env WAVETIME=1,BDYNOTOUCH=1" \
 "sweep --config cfg4 --rounds 4 --steps 5 --variants TPC=8;BDYNOTOUCH=1" \
 "py $M tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20" \
 "py $M PMMG_HIP_BDYNOTOUCH=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20"
