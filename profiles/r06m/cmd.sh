M="PMMG_HIP_SO=parmmg_amd/libpmmg_hip_measure.so"
python3 tools/gpu_job.py --tag r06m \
 "py $M tools/groups_probe.py --rounds 3 --variants base;big_auto" \
 "py $M PMMG_HIP_GROUP_LANES=4 tools/groups_probe.py --rounds 3 --variants base;big_auto" \
 "py $M PMMG_HIP_GROUP_LANES=4 PMMG_HIP_LANE_STREAMS=1 tools/groups_probe.py --rounds 3 --variants base;big_auto" \
 "py $M PMMG_HIP_GROUP_LANES=5 PMMG_HIP_LANE_STREAMS=1 tools/groups_probe.py --rounds 3 --variants base;big_auto" \
 "py $M PMMG_HIP_GROUP_LANES=3 PMMG_HIP_LANE_STREAMS=1 tools/groups_probe.py --rounds 3 --variants base;big_auto"
