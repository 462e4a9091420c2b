"""The drop-in boundary driven from C (tests/c/test_c_abi.c: group views,
pmmg_interp_metrics_and_fields, pmmg_copy_metrics_and_fields_point through
the C-ABI, linked against both product libraries), and the north_star's
CMake build (gfx950 only) configured, built and tested with ctest."""
import os
import shutil
import subprocess

import pytest

from parmmg_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_c_test():
    exe = build.build_c_test()
    return subprocess.run([exe, os.path.join(ROOT, "tests", "golden")], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)


def test_c_program_host_part():
    """Without a device: the host-only entry points work and the module
    refuses to run (no CPU fallback)."""
    from parmmg_amd.transfer import device_count
    if device_count() > 0:
        pytest.skip("a device is visible: covered by test_c_program_on_the_gpu")
    p = _run_c_test()
    assert p.returncode == 0, p.stdout
    assert "host-only checks passed" in p.stdout and "SKIPPED" in p.stdout


@pytest.mark.gpu
def test_c_program_on_the_gpu():
    p = _run_c_test()
    print(p.stdout)
    assert p.returncode == 0, p.stdout
    assert "host-only and device checks passed" in p.stdout
    assert "test_c_abi: carried iteration" in p.stdout
    assert "reference cube fixture (12 tetra, 24 points) transferred, 0 wrong values" in p.stdout


@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not installed")
def test_cmake_build_and_ctest(tmp_path):
    """cmake -S . -B build (gfx950 only) && cmake --build && ctest."""
    b = tmp_path / "build"
    env = dict(os.environ)
    subprocess.run(["cmake", "-S", ROOT, "-B", str(b)], check=True, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                   timeout=300, env=env)
    p = subprocess.run(["cmake", "--build", str(b), "-j", "8"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=900, env=env)
    assert p.returncode == 0, p.stdout[-3000:]
    cache = (b / "CMakeCache.txt").read_text()
    assert "CMAKE_HIP_ARCHITECTURES:STRING=gfx950" in cache
    assert (b / "libpmmg_hip.so").exists() and (b / "libpmmg_host.so").exists()
    p = subprocess.run(["ctest", "--test-dir", str(b), "--output-on-failure"], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout
