set -o pipefail
export TMPDIR=/tmp
M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06zv \
 "pytest tests/test_gpu_parity.py tests/test_gpu_hits.py -q -x" \
 "pytest PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_BDYSPLIT=1 tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_gpu_fallback_scale.py -q -x" \
 "sweep --config cfg4 --rounds 4 --steps 5 --variants TPC=8;BDYSPLIT=1" \
 "sweep --config cfg3 --rounds 3 --steps 5 --variants TPC=8;BDYSPLIT=1" \
 "py $M PMMG_HIP_BDYSPLIT=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20" \
 "py $M tools/shard_step.py --config cfg4 --world 8 --ranks 0,3 --steps 20" \
 "py $M PMMG_HIP_BDYSPLIT=1 tools/groups_only.py" \
 "tracepy $M PMMG_HIP_BDYSPLIT=1 tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 4"
