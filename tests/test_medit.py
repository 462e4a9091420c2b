"""The C Medit reader of the host library (csrc/pmmg_medit.c: the inputs of
PMMG_loadMesh_centralized / PMMG_loadAllSols_centralized, reference
src/inout_pmmg.c:488, :748) against the numpy reader, on the reference's own
libexamples fixtures (tests/golden/cube*.{mesh,sol}) and on edge cases."""
import os

import numpy as np
import pytest

from parmmg_amd import medit

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_cube_mesh_matches_numpy_reader():
    path = os.path.join(GOLD, "cube.mesh")
    a, b = medit.read_mesh_c(path), medit.read_mesh(path)
    np.testing.assert_array_equal(a["xyz"], b["xyz"])
    np.testing.assert_array_equal(a["vref"], b["vref"])
    np.testing.assert_array_equal(a["tetv"], b["tetv"])
    np.testing.assert_array_equal(a["triv"], b["triv"])
    assert a["tetv"].shape == (12, 4) and a["triv"].shape[0] == 20


@pytest.mark.parametrize("name", ["cube-met.sol", "cube-solphys.sol"])
def test_cube_sols_match_numpy_reader(name):
    path = os.path.join(GOLD, name)
    a, b = medit.read_sol_c(path), medit.read_sol(path)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_tensor_order_swap(tmp_path):
    """Medit m11 m12 m22 m13 m23 m33 -> MMG5 m11 m12 m13 m22 m23 m33."""
    p = tmp_path / "t.sol"
    p.write_text("MeshVersionFormatted 2\nDimension 3\nSolAtVertices\n2\n2 1 3\n"
                 "7 11 12 22 13 23 33\n8 1 2 3 4 5 6\nEnd\n")
    s, v = medit.read_sol_c(str(p))
    np.testing.assert_array_equal(s[:, 0], [7, 8])
    np.testing.assert_array_equal(v[0], [11, 12, 13, 22, 23, 33])
    np.testing.assert_array_equal(v[1], [1, 2, 4, 3, 5, 6])


def test_comments_and_skipped_blocks(tmp_path):
    p = tmp_path / "m.mesh"
    p.write_text("# header comment\nMeshVersionFormatted 2\nDimension\n3\nVertices\n4\n"
                 "0 0 0 1\n1 0 0 1 # trailing\n0 1 0 2\n0 0 1 3\nEdges\n1\n1 2 0\nCorners\n2\n1 2\n"
                 "Tetrahedra\n1\n1 2 3 4 7\nEnd\n")
    m = medit.read_mesh_c(str(p))
    assert m["xyz"].shape == (4, 3) and m["tetv"].tolist() == [[1, 2, 3, 4]] and m["tref"].tolist() == [7]
    np.testing.assert_array_equal(m["vref"], [1, 1, 2, 3])
    assert m["triv"].shape == (0, 3)


@pytest.mark.parametrize("text,msg", [
    ("MeshVersionFormatted 2\nDimension 3\nVertices\n2\n0 0 0 0\n", "truncated"),
    ("MeshVersionFormatted 2\nDimension 2\nVertices\n1\n0 0 0\n", "dimension"),
    ("MeshVersionFormatted 2\nDimension 3\nVertices\n1\n0 0 0 0\nTetrahedra\n1\n1 2 3 4 0\nEnd\n", "out of range"),
    ("MeshVersionFormatted 2\nDimension 3\nFancyBlock\n1\n1 2 3\n", "unknown block"),
])
def test_malformed_mesh_rejected(tmp_path, text, msg):
    p = tmp_path / "bad.mesh"
    p.write_text(text)
    with pytest.raises(ValueError, match=msg):
        medit.read_mesh_c(str(p))


def test_missing_files_rejected(tmp_path):
    with pytest.raises(ValueError, match="cannot open"):
        medit.read_mesh_c(str(tmp_path / "none.mesh"))
    with pytest.raises(ValueError, match="cannot open"):
        medit.read_mesh_c(str(tmp_path / "x.meshb"))
    p = tmp_path / "nosol.sol"
    p.write_text("MeshVersionFormatted 2\nDimension 3\nEnd\n")
    with pytest.raises(ValueError, match="no SolAtVertices"):
        medit.read_sol_c(str(p))


def test_reader_survives_corrupted_fixtures_under_asan(tmp_path):
    """tests/c/fuzz_medit.c built with ASan + UBSan against pmmg_medit.c:
    every truncation and ~8 single-byte corruptions per 3 bytes of the
    reference's cube fixtures must return 0/1 without a memory error or a
    leak."""
    import shutil
    import subprocess

    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not found")
    repo = os.path.dirname(os.path.dirname(GOLD))
    exe = tmp_path / "fuzz_medit"
    cmd = [gcc, "-O1", "-g", "-std=c99", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=all", f"-I{os.path.join(repo, 'parmmg_amd', 'csrc')}", "-o", str(exe),
           os.path.join(repo, "tests", "c", "fuzz_medit.c"), os.path.join(repo, "parmmg_amd", "csrc", "pmmg_medit.c")]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0 and "sanitize" in p.stdout:
        pytest.skip("sanitizer runtime not available: " + p.stdout[-200:])
    assert p.returncode == 0, p.stdout
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    r = subprocess.run([str(exe), os.path.join(GOLD, "cube.mesh"), os.path.join(GOLD, "cube-solphys.sol"),
                        str(tmp_path / "scratch.mesh")], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "fuzz_medit:" in r.stdout
    # an id past INT_MAX and a repeated entity block are rejected
    assert "huge vertex id accepted=0" in r.stdout, r.stdout[-500:]
    assert "repeated block accepted=0" in r.stdout, r.stdout[-500:]
    # the binary reader on binary forms of the same fixtures (scratch *.meshb:
    # every corruption goes through read_mesh_binary / read_sol_binary)
    m = medit.read_mesh_c(os.path.join(GOLD, "cube.mesh"))
    _gmf(tmp_path / "cube.meshb", 2, _mesh_blocks(m))
    cols = medit.read_sol_c(os.path.join(GOLD, "cube-solphys.sol"))
    types = [1 if c.shape[1] == 1 else (2 if c.shape[1] == 3 else 3) for c in cols]
    _gmf(tmp_path / "cube.solb", 3, [(GMF_DIM, [("i", np.array([3]))]),
                                     (GMF_SOL, [("i", np.array([cols[0].shape[0], len(types)] + types)),
                                                ("r", np.hstack(cols))])])
    r = subprocess.run([str(exe), str(tmp_path / "cube.meshb"), str(tmp_path / "cube.solb"),
                        str(tmp_path / "scratch.meshb")], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "fuzz_medit:" in r.stdout


# ---- binary .meshb / .solb (GMF layout restated from libMeshb's published
# format; libMeshb is absent from the image and the reference holds no binary
# fixture, so these files are written here and the reader is checked against
# the ASCII reading of the same data: parity unpinned)

GMF_DIM, GMF_VER, GMF_TRI, GMF_TET, GMF_END, GMF_SOL, GMF_CORNERS = 3, 4, 6, 8, 54, 62, 13


def _gmf(path, ver, blocks, big=False):
    """blocks: (code, [(dtype, array), ...]) written in order, each keyword with
    the position of the next one"""
    e = ">" if big else "<"
    real = np.dtype(e + ("f4" if ver == 1 else "f8"))
    pos = np.dtype(e + ("i8" if ver >= 3 else "i4"))
    i4 = np.dtype(e + "i4")
    out = bytearray(np.array([1, ver], i4).tobytes())
    for code, parts in blocks:
        body = b"".join(np.ascontiguousarray(a, dtype=real if k == "r" else i4).tobytes() for k, a in parts)
        head = np.array([code], i4).tobytes()
        nxt = len(out) + len(head) + pos.itemsize + len(body)
        out += head + np.array([nxt], pos).tobytes() + body
    out += np.array([GMF_END], i4).tobytes()
    path.write_bytes(bytes(out))


def _mesh_blocks(m, extra=()):
    def rows(ids, ref):
        return np.hstack([ids, ref[:, None]]).astype(np.int32)
    return [(GMF_DIM, [("i", np.array([3]))])] + list(extra) + [
        (GMF_VER, [("i", np.array([m["xyz"].shape[0]]))] + [item for i in range(m["xyz"].shape[0])
                                                              for item in (("r", m["xyz"][i]),
                                                                           ("i", m["vref"][i:i + 1]))]),
        (GMF_TET, [("i", np.array([m["tetv"].shape[0]])), ("i", rows(m["tetv"], m["tref"]))]),
        (GMF_TRI, [("i", np.array([m["triv"].shape[0]])), ("i", rows(m["triv"], m["trref"]))])]


@pytest.mark.parametrize("ver,big", [(1, False), (2, False), (3, False), (2, True), (3, True)])
def test_binary_mesh_matches_ascii(tmp_path, ver, big):
    a = medit.read_mesh_c(os.path.join(GOLD, "cube.mesh"))
    corners = (GMF_CORNERS, [("i", np.array([2, 1, 2]))])  # a block the reader skips by its position
    p = tmp_path / "cube.meshb"
    _gmf(p, ver, _mesh_blocks(a, extra=[corners]), big)
    b = medit.read_mesh_c(str(p))
    xyz = a["xyz"].astype(np.float32).astype(np.float64) if ver == 1 else a["xyz"]
    np.testing.assert_array_equal(b["xyz"], xyz)
    for k in ("vref", "tetv", "tref", "triv", "trref"):
        np.testing.assert_array_equal(b[k], a[k])


@pytest.mark.parametrize("name", ["cube-met.sol", "cube-solphys.sol"])
@pytest.mark.parametrize("ver,big", [(2, False), (3, True)])
def test_binary_sol_matches_ascii(tmp_path, name, ver, big):
    path = os.path.join(GOLD, name)
    cols = medit.read_sol_c(path)
    types = [1 if c.shape[1] == 1 else (2 if c.shape[1] == 3 else 3) for c in cols]
    # back to Medit's tensor order for the file (m11 m12 m22 m13 m23 m33)
    fileo = [c[:, [0, 1, 3, 2, 4, 5]] if c.shape[1] == 6 else c for c in cols]
    n = cols[0].shape[0]
    vals = np.hstack(fileo)
    p = tmp_path / (name + "b")
    _gmf(p, ver, [(GMF_DIM, [("i", np.array([3]))]),
                  (GMF_SOL, [("i", np.array([n, len(types)] + types)), ("r", vals)])], big)
    for x, y in zip(medit.read_sol_c(str(p)), cols):
        np.testing.assert_array_equal(x, y)


def test_binary_files_rejected(tmp_path):
    a = medit.read_mesh_c(os.path.join(GOLD, "cube.mesh"))
    p = tmp_path / "t.meshb"
    _gmf(p, 2, _mesh_blocks(a))
    raw = p.read_bytes()
    (tmp_path / "trunc.meshb").write_bytes(raw[: len(raw) // 2])
    with pytest.raises(ValueError, match="truncated|valid count"):  # a count past the end of the file
        medit.read_mesh_c(str(tmp_path / "trunc.meshb"))
    (tmp_path / "v4.meshb").write_bytes(np.array([1, 4], "<i4").tobytes() + raw[8:])
    with pytest.raises(ValueError, match="version 4"):
        medit.read_mesh_c(str(tmp_path / "v4.meshb"))
    (tmp_path / "junk.meshb").write_bytes(b"MeshVersionFormatted 2\n")
    with pytest.raises(ValueError, match="not a binary Medit"):
        medit.read_mesh_c(str(tmp_path / "junk.meshb"))
    # an unknown block whose next-keyword position points back: rejected, not looped over
    loop = np.array([1, 2, GMF_CORNERS, 8], "<i4").tobytes()
    (tmp_path / "loop.meshb").write_bytes(loop)
    with pytest.raises(ValueError, match="malformed"):
        medit.read_mesh_c(str(tmp_path / "loop.meshb"))
    (tmp_path / "d2.meshb").write_bytes(raw[:8] + np.array([GMF_DIM, 20, 2], "<i4").tobytes() + raw[20:])
    with pytest.raises(ValueError, match="dimension"):
        medit.read_mesh_c(str(tmp_path / "d2.meshb"))
