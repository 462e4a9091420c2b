"""Per-wave lifetimes of k_bdy from the measurement build's PMMG_HIP_WAVETIME
records (u64 quads {start, end, longest walk in the wave, active lanes},
wall clock at 100 MHz, one block of records per call appended to
PMMG_HIP_WAVETIME_OUT).

  python tools/wave_time.py FILE --calls N
"""
import argparse

import numpy as np

TICK_US = 0.01  # wall_clock64: 100 MHz


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--calls", type=int, required=True)
    a = ap.parse_args()
    w = np.fromfile(a.path, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
    per = w.shape[0] // a.calls
    q = [0, 10, 50, 90, 99, 100]
    for c in range(a.calls):
        r = w[c * per:(c + 1) * per]
        ran = r[r[:, 0] > 0]
        if ran.shape[0] == 0:
            print(f"call {c}: no records")
            continue
        t0 = ran[:, 0].min()
        start = (ran[:, 0] - t0) * TICK_US
        end = (ran[:, 1] - t0) * TICK_US
        life = end - start
        act = ran[:, 3] > 0
        print(f"call {c}: waves {ran.shape[0]} (active {int(act.sum())}), span {end.max():.1f} us")
        for name, v in (("start", start[act]), ("end", end[act]), ("lifetime", life[act]),
                        ("steps", ran[act, 2].astype(float)), ("empty lifetime", life[~act])):
            if v.size:
                print(f"  {name:15s} " + " ".join(f"p{p}={np.percentile(v, p):8.1f}" for p in q))
        if act.sum() > 10:
            s = ran[act, 2].astype(float)
            for lo, hi in ((0, 8), (8, 12), (12, 16), (16, 24), (24, 1 << 30)):
                m = (s >= lo) & (s < hi)
                if m.any():
                    print(f"  longest walk {lo:3d}-{min(hi, 999):3d}: {int(m.sum()):6d} waves, lifetime median "
                          f"{np.median(life[act][m]):8.1f} us, max {life[act][m].max():8.1f}")


if __name__ == "__main__":
    main()
