"""bench.py's groups leg alone (10 cfg2-size groups in one
pmmg_hip_locate_interp_groups call vs one call per group), for lane /
hardware-queue sweeps:

    GPU_MAX_HW_QUEUES=16 PMMG_HIP_GROUP_LANES=8 python tools/groups_only.py [--no-parity]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    args = argparse.Namespace(no_cpu_baseline=a.no_parity)
    res = bench.groups_leg(args, reps=a.reps)
    res["env"] = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "PMMG_HIP_GROUP_LANES")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
