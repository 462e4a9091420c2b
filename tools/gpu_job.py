"""One parameterised GPU job (replaces the per-run tools/gpu_r0*.sh scripts,
which now live beside their results under profiles/<run>/cmd.sh).

Runs on the GPU box as   python3 tools/gpu_job.py --tag r05b STEP [STEP ...]
with every step a string, run in order, each under its own time limit; the
job stops at the first step that fails (no retries), and every step's log
goes to gpurun_out/<tag>/.  The driver process itself never touches the GPU
(each step is a child process), so nothing is exec'ed from a GPU process.

Steps:
  pytest ARGS            python -m pytest ARGS -x -v --timeout 300 (thread method)
  sweep ARGS             tools/sweep.py ARGS (interleaved A/B of module settings)
  bench ARGS             bench.py ARGS; the JSON line -> <tag>/bench[_N].json
  pmcpy FILT CTRS ARGS   one rocprofv3 --pmc pass of python3 -u ARGS (a tools/ script), table of
                         the kernels matching FILT
  pmc CFG VARIANT CTRS   one rocprofv3 --pmc pass of tools/sweep.py (one live
                         context, one step) with counters CTRS (space separated,
                         within one pass's limits); table -> <tag>/pmc_*.txt
  trace ARGS             rocprofv3 --kernel-trace --stats of bench.py ARGS
                         (kernel_stats.csv copied to <tag>/)
  tracepy ARGS           the same of python3 -u ARGS (a tools/ script); the
                         kernel_trace.csv is copied too
  py ARGS                python3 -u ARGS (a tools/ script)
A step may start with NAME=VALUE tokens: environment variables of that step.
"""
from __future__ import annotations

import argparse
import glob
import os
import shlex
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIMITS = {"pytest": 900, "sweep": 900, "bench": 900, "pmc": 120, "trace": 900, "tracepy": 600, "py": 600}


def run(cmd: list[str], log: str, limit: int, kill_signal: str = "TERM") -> int:
    full = ["timeout", "-s", kill_signal, "-k", "10", str(limit)] + cmd
    print(f"[gpu_job] {time.strftime('%H:%M:%S')} {' '.join(shlex.quote(c) for c in cmd)} -> {log}", flush=True)
    t0 = time.time()
    with open(log, "w") as f:
        # lines go to the log as they come: the harness watches gpurun_out/ for progress
        rc = subprocess.call(full, stdout=f, stderr=subprocess.STDOUT, cwd=ROOT)
    print(f"[gpu_job] rc={rc} in {time.time() - t0:.1f}s", flush=True)
    return rc


def tail(path: str, n: int = 15) -> None:
    try:
        with open(path) as f:
            lines = f.readlines()
        sys.stdout.write("".join(lines[-n:]))
        sys.stdout.flush()
    except OSError:
        pass


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("steps", nargs="+")
    a = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out", a.tag)
    os.makedirs(out, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    counts: dict[str, int] = {}
    for step in a.steps:
        kind, _, rest = step.partition(" ")
        args = shlex.split(rest)
        # leading NAME=VALUE tokens: environment of this step only
        env = {}
        while args and "=" in args[0] and args[0].split("=")[0].isidentifier() and args[0].split("=")[0].isupper():
            k, v = args.pop(0).split("=", 1)
            env[k] = v
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        i = counts.get(kind, 0)
        counts[kind] = i + 1
        name = f"{kind}{i if i else ''}"
        log = os.path.join(out, f"{name}.log")
        if kind == "pytest":
            rc = run([sys.executable, "-u", "-m", "pytest"] + args + ["-x", "-v", "--timeout", "300",
                                                                     "--timeout-method", "thread"], log, LIMITS[kind])
        elif kind == "sweep":
            rc = run([sys.executable, "-u", "tools/sweep.py"] + args, log, LIMITS[kind])
        elif kind == "py":
            rc = run([sys.executable, "-u"] + args, log, LIMITS[kind])
        elif kind == "bench":
            rc = run([sys.executable, "-u", "bench.py"] + args, log, LIMITS[kind])
            if rc == 0:
                lines = [x for x in open(log) if x.startswith("{")]
                if lines:
                    with open(os.path.join(out, f"bench{('_' + str(i)) if i else ''}.json"), "w") as f:
                        f.write(lines[-1])
        elif kind == "pmc":
            cfg, variant, ctrs = args[0], args[1], args[2]
            d = os.path.join(out, f"{name}")
            rc = run(["rocprofv3", "--pmc"] + ctrs.split() + ["-d", os.path.join(d, "p1"), "-o", "run",
                                                              "--output-format", "csv", "--", sys.executable, "-u",
                                                              "tools/sweep.py", "--config", cfg, "--variants", variant,
                                                              "--rounds", "1", "--steps", "1"], log, LIMITS[kind],
                     kill_signal="KILL")
            if rc == 0:
                with open(os.path.join(out, f"{name}.txt"), "w") as f:
                    f.write(f"# variant {variant!r}, counters {ctrs}\n")
                    f.flush()
                    subprocess.call([sys.executable, "tools/pmc_table.py", d, "k_"], stdout=f, cwd=ROOT)
        elif kind == "pmcpy":  # pmcpy KERNEL-SUBSTRING "CTRS" SCRIPT ARGS...: one --pmc pass of a tools/ script
            filt, ctrs = args[0], args[1]
            d = os.path.join(out, f"{name}")
            rc = run(["rocprofv3", "--pmc"] + ctrs.split() + ["-d", os.path.join(d, "p1"), "-o", "run",
                                                              "--output-format", "csv", "--", sys.executable, "-u"]
                     + args[2:], log, LIMITS["pmc"], kill_signal="KILL")
            if rc == 0:
                with open(os.path.join(out, f"{name}.txt"), "w") as f:
                    f.write(f"# {' '.join(args[2:])!r}, counters {ctrs}\n")
                    f.flush()
                    subprocess.call([sys.executable, "tools/pmc_table.py", d, filt], stdout=f, cwd=ROOT)
        elif kind in ("trace", "tracepy"):
            d = os.path.join(out, name)
            prog = ["bench.py"] if kind == "trace" else []
            rc = run(["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "run", "--output-format", "csv", "--",
                      sys.executable, "-u"] + prog + args, log, LIMITS[kind])
            for p in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
                shutil.copy(p, os.path.join(out, f"{name}_kernel_stats.csv"))
            if kind == "tracepy":
                for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
                    shutil.copy(p, os.path.join(out, f"{name}_kernel_trace.csv"))
        else:
            print(f"[gpu_job] unknown step kind {kind!r}", flush=True)
            return 2
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        tail(log)
        if rc != 0:
            print(f"[gpu_job] step {name} failed (rc={rc}); stopping", flush=True)
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
