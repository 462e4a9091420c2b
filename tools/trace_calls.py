"""Per-call view of a rocprofv3 kernel trace (kernel_trace.csv): the calls
are cut at each k_reset dispatch; prints, per kernel, the median duration and
the median gap from the previous kernel of the same queue, and the median
span of a call (first start to last end over all of its kernels).

  python tools/trace_calls.py TRACE.csv [--skip N]   (N first calls dropped: warm-up)
"""
import csv
import statistics as S
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    return n.replace("pmmg::", "").replace("void ", "")


def main() -> None:
    path = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], []
    for r in rows:
        if short(r["Kernel_Name"]) == "k_reset" and cur:
            calls.append(cur)
            cur = []
        cur.append(r)
    if cur:
        calls.append(cur)
    calls = calls[skip:]
    dur, gap = defaultdict(list), defaultdict(list)
    spans = []
    for c in calls:
        t0 = min(int(r["Start_Timestamp"]) for r in c)
        t1 = max(int(r["End_Timestamp"]) for r in c)
        spans.append((t1 - t0) / 1e3)
        last = {}
        for r in c:
            q = (r["Agent_Id"], r["Queue_Id"])
            k = short(r["Kernel_Name"])
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            dur[k].append((e - s) / 1e3)
            if q in last:
                gap[k].append((s - last[q]) / 1e3)
            last[q] = e
    print(f"{len(calls)} calls, median span {S.median(spans):.1f} us, min {min(spans):.1f} us")
    print(f"{'kernel':40s} {'n':>5s} {'med us':>8s} {'gap us':>8s}")
    order = sorted(dur, key=lambda k: -S.median(dur[k]) * len(dur[k]))
    for k in order:
        g = f"{S.median(gap[k]):8.1f}" if gap[k] else "       -"
        print(f"{k[:40]:40s} {len(dur[k]):5d} {S.median(dur[k]):8.1f} {g}")


if __name__ == "__main__":
    main()
