"""The C-ABI library loads and exports every symbol the headers declare; the
product path never links the oracle and has no CPU fallback (CPU only)."""
import ctypes
import os
import re
import subprocess

import pytest

from parmmg_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pmmg_[a-z0-9_]+)\s*\(", text)))


def _exports(so):
    out = subprocess.run(["nm", "-D", "--defined-only", so], stdout=subprocess.PIPE, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_hip_module_exports_the_c_abi():
    names = _declared(os.path.join(ROOT, "include", "parmmg_hip.h"))
    assert len(names) >= 12
    lib = ctypes.CDLL(build.HIP_SO)
    exp = _exports(build.HIP_SO)
    for n in names:
        assert n in exp, n
        getattr(lib, n)


def test_host_layer_exports():
    names = [n for n in _declared(os.path.join(ROOT, "parmmg_amd", "csrc", "pmmg_host.h"))]
    exp = _exports(build.HOST_SO)
    for n in names:
        assert n in exp, n


def test_hip_module_is_gfx950_code():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", build.HIP_SO], stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True).stdout
    blob = open(build.HIP_SO, "rb").read()
    assert b"gfx950" in blob, out[:200]


@pytest.mark.parametrize("so", [build.HIP_SO, build.HOST_SO])
def test_product_does_not_link_the_oracle(so):
    exp = _exports(so)
    assert not any(s.startswith("orc_") for s in exp)
    deps = subprocess.run(["readelf", "-d", so], stdout=subprocess.PIPE, text=True).stdout
    assert "oracle" not in deps


def test_no_cpu_fallback_without_gpu():
    from parmmg_amd import transfer

    if transfer.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        transfer.TransferContext(0)


def test_ctypes_structs_match_the_header(tmp_path):
    """The Python mirrors of the header's structs (pmmg_hip_stats,
    pmmg_hip_group) have the C compiler's size and field offsets: a field
    added to include/parmmg_hip.h without its mirror would shift every later
    field the bench and the tests read."""
    import ctypes
    import subprocess

    from parmmg_amd._native import HipGroup, HipStats

    checks = []
    for cname, py in (("pmmg_hip_stats", HipStats), ("pmmg_hip_group", HipGroup)):
        checks.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            checks.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "parmmg_hip.h"\nint main(void) {\n'
                   + "\n".join(checks) + "\nreturn 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    want = {}
    for line in filter(None, out):
        cname, fname, v = line.split()
        want[(cname, fname)] = int(v)
    for cname, py in (("pmmg_hip_stats", HipStats), ("pmmg_hip_group", HipGroup)):
        assert ctypes.sizeof(py) == want[(cname, "size")], cname
        for fname, _ in py._fields_:
            assert getattr(py, fname).offset == want[(cname, fname)], (cname, fname)


def test_abi_version_and_stats_size():
    """The load-time check a shim makes (include/parmmg_hip.h): the library's
    ABI version is the header's PMMG_HIP_ABI_VERSION and it writes exactly
    sizeof(pmmg_hip_stats) bytes of stats (a counter appended
    without a version let an older shim's struct be overrun)."""
    import re

    from parmmg_amd import _native

    hdr = open(os.path.join(ROOT, "include", "parmmg_hip.h")).read()
    v = int(re.search(r"#define PMMG_HIP_ABI_VERSION (\d+)", hdr).group(1))
    lib = _native.hip_lib()
    assert lib.pmmg_hip_abi_version() == v == _native.ABI_VERSION
    assert lib.pmmg_hip_stats_size() == ctypes.sizeof(_native.HipStats)
