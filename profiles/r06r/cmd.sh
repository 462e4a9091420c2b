M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06r \
 "pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_hits.py tests/test_gpu_records.py tests/test_gpu_fallback_scale.py tests/test_gpu_groups.py -m gpu -q" \
 "sweep --config cfg4 --rounds 3 --steps 5 --variants TPC=8;FUSECONT=0" \
 "sweep --config cfg3 --rounds 2 --steps 5 --variants TPC=8;FUSECONT=0" \
 "py $M tools/groups_probe.py --rounds 2 --variants base" \
 "py $M PMMG_HIP_FUSECONT=0 tools/groups_probe.py --rounds 2 --variants base" \
 "tracepy tools/sweep.py --config cfg4 --rounds 1 --steps 3 --variants TPC=8"
