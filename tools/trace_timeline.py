"""One call's kernel timeline from a rocprofv3 kernel trace (kernel_trace.csv):
the calls are cut at each k_reset; prints kernel, queue, start and end in us
from the call's k_reset, for the call `--call` from the end (default 3rd last).

  python tools/trace_timeline.py TRACE.csv [--call 3] [--all]   (--all: keep the gated binning kernels)
"""
import csv
import sys


def short(n: str) -> str:
    return n.split("(")[0].replace("pmmg::", "").replace("void ", "")[:24]


def main() -> None:
    path = sys.argv[1]
    k = int(sys.argv[sys.argv.index("--call") + 1]) if "--call" in sys.argv else 3
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == "k_reset"]
    i0 = idx[-k]
    i1 = idx[-k + 1] if k > 1 else len(rows)
    t0 = int(rows[i0]["Start_Timestamp"])
    print(f"{'kernel':26s} queue  start_us   end_us")
    for r in rows[i0:i1]:
        n = short(r["Kernel_Name"])
        if "--all" not in sys.argv and (n.startswith("k_rs") or n == "k_scan_top"):
            continue
        print(f"{n:26s} q{r['Queue_Id']:4s} {(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {(int(r['End_Timestamp']) - t0) / 1e3:8.1f}")


if __name__ == "__main__":
    main()
