"""Host-buffer (PCIe-inclusive) transfer of one config, as bench.py's
host_mode leg, with PMMG_HIP_VERBOSE=1 transfer timings on stderr.

    python tools/host_mode.py --config cfg4 --reps 3
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("PMMG_HIP_VERBOSE", "1")

import bench  # noqa: E402
from parmmg_amd import configs  # noqa: E402
from parmmg_amd.transfer import TransferContext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    w = configs.SHORT[a.config]
    bg, new, met, fields, pc = bench.build_workload(w, 0)
    with TransferContext(0) as ctx:
        print(bench.host_mode_timing(ctx, w, bg, met, fields, new.xyz, pc, 0, reps=a.reps), flush=True)


if __name__ == "__main__":
    main()
