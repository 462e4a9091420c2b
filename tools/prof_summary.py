"""Summarise one tools/gpu_prof.sh run into profiles/<round>/:

* kernel_stats.csv       rocprofv3 --kernel-trace --stats summary (copied)
* kernels.json           per kernel: calls, average duration, VGPR/SGPR/LDS
* pmc_<workload>.json    HBM bytes per launch of every kernel from the two
                         PMC passes, corrected as MI355X_MICROARCH.md
                         prescribes (FETCH_SIZE and WRITE_SIZE are in KiB;
                         FETCH_SIZE counts half the bytes of wide reads on
                         gfx950 -> doubled)
* bench.json             the bench line of the same run

  python tools/prof_summary.py gpurun_out/r1c profiles/r01
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def per_dispatch(path):
    """counter sum per dispatch, grouped by kernel name"""
    disp = defaultdict(float)
    name = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        disp[d] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
    by = defaultdict(list)
    for d, v in disp.items():
        by[name[d]].append(v)
    return by


def short(k):
    k = k.replace("(anonymous namespace)::", "").replace("void ", "").replace("pmmg::", "")
    return k.split("(")[0]


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    bpath = os.path.join(src, "bench.json")  # optional: the bench line of the same session
    bench = {}
    if os.path.exists(bpath):
        bench = json.loads(open(bpath).read().strip().splitlines()[-1])
        json.dump(bench, open(os.path.join(dst, "bench.json"), "w"), indent=1)
    kern = {}
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
    for r in rows:
        k = short(r["Kernel_Name"])
        e = kern.setdefault(k, dict(calls=0, total_ns=0, vgpr=int(r["VGPR_Count"]), sgpr=int(r["SGPR_Count"]),
                                    lds=int(r["LDS_Block_Size"]), scratch=int(r["Scratch_Size"]),
                                    grid=int(r["Grid_Size_X"]), block=int(r["Workgroup_Size_X"])))
        e["calls"] += 1
        e["total_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for e in kern.values():
        e["avg_us"] = round(e["total_ns"] / e["calls"] / 1e3, 3)
    # volume stage span per transfer call from the trace timestamps: the walk
    # and interpolation launches of one call (chunked, on two streams, so
    # they overlap) from the first start to the last end; a call starts at
    # its k_seed_vol launch
    spans, cur = [], None
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        k = short(r["Kernel_Name"])
        if k == "k_seed_vol":
            if cur:
                spans.append(cur[1] - cur[0])
            cur = None
            continue
        if k.startswith("k_vol<") or k.startswith("k_vol_walk") or k.startswith("k_vol_interp") or k.startswith("k_vol_fused"):
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            cur = [a, b] if cur is None else [min(cur[0], a), max(cur[1], b)]
    if cur:
        spans.append(cur[1] - cur[0])
    calls = sum(1 for r in rows if short(r["Kernel_Name"]) == "k_seed_vol")
    kern_summary = {"kernels": kern, "transfer_calls": calls,
                    "k_vol_stage_span_us": round(sum(spans) / len(spans) / 1e3, 3) if spans else None,
                    "k_vol_stage_spans_us": [round(x / 1e3, 3) for x in spans]}
    json.dump(kern_summary, open(os.path.join(dst, "kernels.json"), "w"), indent=1)
    fetch = per_dispatch(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = per_dispatch(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    pmc = {"note": "bytes per launch; FETCH_SIZE/WRITE_SIZE are KiB; FETCH doubled: on gfx950 FETCH_SIZE = 64 B x "
                   "TCC_EA0_RDREQ and every read request moves a 128 B line (calibrated in profiles/r02a/calib: "
                   "streamed and gathered whole lines, 4-16 B per lane, report exactly half); counters include "
                   "Infinity-Cache hits",
           "workload": bench.get("config", {}).get("workload", os.environ.get("PMMG_PROF_WORKLOAD", "cfg4-shell100M-aniso")),
           "kernels": {}}
    ncall = max(1, len(fetch.get(next((k for k in fetch if short(k) == "k_seed_vol"), ""), [])))
    for k in set(fetch) | set(write):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        fb = 2.0 * 1024.0 * sum(f) / len(f)
        wb = 1024.0 * sum(w) / len(w)
        pmc["kernels"][short(k)] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                                    "fetch_raw_kib": sum(f) / len(f), "write_raw_kib": sum(w) / len(w),
                                    "launches_per_call": len(f) / ncall,
                                    "hbm_bytes_per_call": (2.0 * 1024.0 * sum(f) + 1024.0 * sum(w)) / ncall}
    # the volume stage: every k_vol* kernel of one call (walk + interpolation,
    # or the fused kernel)
    kv = sorted(k for k in pmc["kernels"] if k.startswith("k_vol") and "exhaust" not in k and "finish" not in k)
    if kv:
        pmc["k_vol_kernel"] = " + ".join(kv)
        # one volume stage = every launch of those kernels in one transfer call
        pmc["k_vol_hbm_bytes_per_call"] = sum(pmc["kernels"][k]["hbm_bytes_per_call"] for k in kv)
    json.dump(pmc, open(os.path.join(dst, f"pmc_{pmc['workload']}.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in pmc.items() if k != "kernels"}, indent=1))
    print("volume stage span (trace):", kern_summary["k_vol_stage_span_us"], "us over", len(spans), "calls")
    for k, e in sorted(kern.items(), key=lambda kv: -kv[1]["total_ns"]):
        print(f"{e['avg_us']:10.1f} us x{e['calls']:3d}  vgpr {e['vgpr']:3d}  {k}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
