python3 tools/gpu_job.py --tag r05m \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so tools/groups_only.py --no-parity" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_NOFB=1 tools/groups_only.py --no-parity" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_LANE_STREAMS=1 tools/groups_only.py --no-parity" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so PMMG_HIP_LANE_STREAMS=1 PMMG_HIP_GROUP_LANES=8 tools/groups_only.py --no-parity" \
 "py PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so tools/groups_only.py --no-parity" \
 "tracepy tools/shard_step.py --config cfg4 --world 8 --ranks 0 --steps 10"
