"""In-tree build of the native libraries (no cmake, no JIT cache).

* ``parmmg_amd/libpmmg_hip.so``   — the product: HIP kernels + C-ABI of
  ``include/parmmg_hip.h`` (hipcc, gfx950 only, ``-ffp-contract=off``).
* ``parmmg_amd/libpmmg_host.so``  — the product's C host layer
  (``csrc/pmmg_host.c``: group loop / point classification of
  ``PMMG_interpMetricsAndFields``), linked against libpmmg_hip.so.
* ``parmmg_amd/libpmmg_synth.so`` — synthetic-mesh generator (tests/bench).
* ``oracle/liboracle.so``         — the CPU restatement (test infrastructure).

Outputs are .so files next to their sources; they are git-ignored but travel
to the GPU box with the working tree.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "parmmg_amd")
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
ORACLE = os.path.join(ROOT, "oracle")

HIP_SO = os.path.join(PKG, "libpmmg_hip.so")
# the measurement build (-DPMMG_HIP_MEASURE: the A/B switches of tools/, never
# linked by the host layer or loaded by the tests; PMMG_HIP_SO selects it)
HIP_MEASURE_SO = os.path.join(PKG, "libpmmg_hip_measure.so")
HOST_SO = os.path.join(PKG, "libpmmg_host.so")
SYNTH_SO = os.path.join(PKG, "libpmmg_synth.so")
ORACLE_SO = os.path.join(ORACLE, "liboracle.so")
C_TEST = os.path.join(ROOT, "tests", "c", "test_c_abi")

ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP module cannot be built")


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        sys.stderr.write(proc.stdout)
        raise RuntimeError("build command failed: " + " ".join(cmd))


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build_hip(force: bool = False, measure: bool = False) -> str:
    out = HIP_MEASURE_SO if measure else HIP_SO
    src = os.path.join(CSRC, "pmmg_hip.hip")
    snap = os.path.join(CSRC, "pmmg_snapshot.hip")
    qual = os.path.join(CSRC, "pmmg_quality.hip")
    deps = [src, snap, qual, os.path.join(INC, "parmmg_hip.h"), __file__] + [
        os.path.join(CSRC, h) for h in ("pmmg_device.hpp", "pmmg_prep.hpp", "pmmg_vol.hpp", "pmmg_bdy.hpp",
                                        "pmmg_fallback.hpp", "pmmg_snapshot.hpp", "pmmg_quality.hpp",
                                        "pmmg_brick.hpp", "pmmg_sort.hpp")]
    if force or _stale(out, deps):
        # max-memory-clause scheduling: the gathers of a step issued as clauses
        # (volume kernel -4.6 % at cfg4, same registers; profiles/r02e/sweep_sched_strategy.txt)
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-mllvm", "-amdgpu-sched-strategy=max-memory-clause",
              "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
              # (r05: flowing off a lambda that a `return 0` made non-void is undefined: a host segfault)
              "-Werror=return-type"] + (["-DPMMG_HIP_MEASURE"] if measure else []) +
             [f"-I{INC}", "-o", out, src, snap, qual])
    return out


def build_host(force: bool = False) -> str:
    src = os.path.join(CSRC, "pmmg_host.c")
    shard = os.path.join(CSRC, "pmmg_shard.c")
    medit = os.path.join(CSRC, "pmmg_medit.c")
    deps = [src, shard, medit, os.path.join(CSRC, "pmmg_host.h"), os.path.join(CSRC, "pmmg_medit.h"),
            os.path.join(INC, "parmmg_hip.h"), HIP_SO, __file__]
    if force or _stale(HOST_SO, deps):
        # -fopenmp: the halo-shard builder (pmmg_shard.c) runs its passes over
        # the group's tetra on the host threads
        _run(["gcc", "-O2", "-std=c99", "-fopenmp", "-Wall", "-Wextra", "-fPIC", "-shared", f"-I{INC}", f"-I{CSRC}",
              "-o", HOST_SO, src, shard, medit, f"-L{PKG}", "-lpmmg_hip", "-Wl,-rpath,$ORIGIN"])
    return HOST_SO


def build_synth(force: bool = False) -> str:
    src = os.path.join(CSRC, "pmmg_synth.c")
    deps = [src, os.path.join(CSRC, "pmmg_synth.h"), __file__]
    if force or _stale(SYNTH_SO, deps):
        _run(["gcc", "-O2", "-std=c99", "-fopenmp", "-Wall", "-Wextra", "-fPIC", "-shared", "-o", SYNTH_SO, src,
              "-lm"])
    return SYNTH_SO


def build_oracle(force: bool = False) -> str:
    src = os.path.join(ORACLE, "pmmg_oracle.c")
    deps = [src, os.path.join(ORACLE, "pmmg_oracle.h"), __file__]
    if force or _stale(ORACLE_SO, deps):
        # -ffp-contract=off: keep the reference's rounding (no FMA contraction)
        _run(["gcc", "-O2", "-std=gnu99", "-pthread", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wextra",
              "-fPIC", "-shared", "-o", ORACLE_SO, src, "-lm", "-lpthread"])
    return ORACLE_SO


def build_c_test(force: bool = False) -> str:
    """tests/c/test_c_abi: the C-ABI driven from C, linked against both
    product libraries (rpath relative to the binary, so it runs from any copy
    of the tree)."""
    src = os.path.join(ROOT, "tests", "c", "test_c_abi.c")
    synth = os.path.join(CSRC, "pmmg_synth.c")
    deps = [src, synth, HIP_SO, HOST_SO, os.path.join(INC, "parmmg_hip.h"), os.path.join(CSRC, "pmmg_host.h"),
            os.path.join(CSRC, "pmmg_medit.h"), __file__]
    if force or _stale(C_TEST, deps):
        _run(["gcc", "-O2", "-std=c99", "-Wall", "-Wextra", f"-I{INC}", f"-I{CSRC}", "-o", C_TEST, src, synth,
              f"-L{PKG}", "-lpmmg_host", "-lpmmg_hip", "-lm", "-Wl,-rpath,$ORIGIN/../../parmmg_amd"])
    return C_TEST


def build_all(force: bool = False) -> None:
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(2) as ex:  # the two HIP builds side by side (hipcc is single-threaded)
        jobs = [ex.submit(build_hip, force), ex.submit(build_hip, force, True)]
        for j in jobs:
            j.result()
    build_host(force)
    build_synth(force)
    build_oracle(force)
    build_c_test(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built:", HIP_SO, HOST_SO, SYNTH_SO, ORACLE_SO)
