"""Background snapshot on the device (pmmg_hip_build_adjacency /
pmmg_hip_build_boundary; reference PMMG_create_oldGrp, src/grpsplit_pmmg.c:207-418,
with Mmg's MMG3D_hashTetra / MMG5_chkBdryTria / MMG3D_hashTria).

The checker is the host builder of the synthetic meshes (pmmg_synth.c: tetra
adjacency analytic from the lattice, boundary trias and their adjacency by
sorted edge matching), which restates the same Mmg conventions independently
of the GPU's bucket hashing.  Results must be bit-identical.  Mmg itself is not
in the image, so the conventions are restated, not pinned.
"""
import numpy as np
import pytest

from parity import make_case, run_gpu
from parmmg_amd import synth
from parmmg_amd.transfer import TransferContext, pack_tet8


def _snapshot(ctx, bg, use_tet8=True):
    tetv = ctx.upload(bg.tetv)
    adja, tet8 = ctx.build_adjacency(bg.np, tetv)
    if use_tet8:
        triv, adjt = ctx.build_boundary(bg.np, tet8=tet8)
    else:
        triv, adjt = ctx.build_boundary(bg.np, tetv=tetv, adja=adja)
    return tetv, adja, tet8, triv, adjt


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [(synth.CUBE, 1), (synth.CUBE, 5), (synth.SHELL, 8), (synth.SHELL, 12),
                                    (synth.CUBE, 40)])
@pytest.mark.parametrize("use_tet8", [True, False])
def test_snapshot_matches_host_builder(kind, n, use_tet8):
    bg = synth.lattice(kind, n)
    with TransferContext(0) as ctx:
        _, adja, tet8, triv, adjt = _snapshot(ctx, bg, use_tet8)
        np.testing.assert_array_equal(adja.download(), bg.adja)
        np.testing.assert_array_equal(tet8.download(), pack_tet8(bg.tetv, bg.adja))
        assert triv.shape[0] == bg.nt
        np.testing.assert_array_equal(triv.download(), bg.triv)
        np.testing.assert_array_equal(adjt.download(), bg.adjt)


@pytest.mark.gpu
def test_snapshot_of_a_shuffled_numbering():
    """Tetra order and vertex numbering are arbitrary: the adjacency of a
    permuted mesh is the permuted adjacency."""
    bg = synth.lattice(synth.SHELL, 8)
    rng = np.random.default_rng(7)
    pe = rng.permutation(bg.ne)          # new tetra j = old tetra pe[j]
    pv = rng.permutation(bg.np) + 1      # old vertex v -> new id pv[v-1]
    tetv = pv[bg.tetv[pe] - 1].astype(np.int32)
    inv = np.empty_like(pe)
    inv[pe] = np.arange(bg.ne)
    old = bg.adja[pe]
    k_old, i_old = old // 4, old % 4
    expect = np.where(old > 0, 4 * (inv[np.maximum(k_old - 1, 0)] + 1) + i_old, 0).astype(np.int32)
    with TransferContext(0) as ctx:
        adja, _ = ctx.build_adjacency(bg.np, ctx.upload(np.ascontiguousarray(tetv)), tet8=False)
        np.testing.assert_array_equal(adja.download(), expect)


def _host_adjacency(tetv):
    """MMG3D_hashTetra's result by a dictionary of sorted faces (face i opposite vertex i)."""
    faces = {}
    for k, t in enumerate(tetv.tolist()):
        for i in range(4):
            faces.setdefault(tuple(sorted(t[:i] + t[i + 1:])), []).append(4 * (k + 1) + i)
    adja = np.zeros(tetv.shape, np.int32)
    for codes in faces.values():
        if len(codes) == 2:
            a, b = codes
            adja[a // 4 - 1, a % 4], adja[b // 4 - 1, b % 4] = b, a
    return adja


@pytest.mark.gpu
def test_snapshot_of_a_high_valence_vertex():
    """A star of tetra around one vertex (vertex 1, the smallest id, in every
    tetra): its face bucket holds 3 faces per tetra, more than the match
    kernel stages in LDS for a block of vertices (kMatchCap, 768 entries), so
    that block scans its buckets in place."""
    bg = synth.lattice(synth.SHELL, 12)
    r = np.linalg.norm(bg.xyz - bg.xyz.mean(0), axis=1)
    outer = bg.triv[(r[bg.triv - 1] > np.median(r)).all(axis=1)]
    assert 3 * outer.shape[0] > 2048  # pmmg_snapshot.hip kMatchCap
    tetv = np.hstack([np.ones((outer.shape[0], 1), np.int32), outer + 1]).astype(np.int32)
    with TransferContext(0) as ctx:
        adja, tet8 = ctx.build_adjacency(bg.np + 1, ctx.upload(np.ascontiguousarray(tetv)))
        expect = _host_adjacency(tetv)
        np.testing.assert_array_equal(adja.download(), expect)
        np.testing.assert_array_equal(tet8.download(), pack_tet8(tetv, expect))
        assert (expect[:, 0] == 0).all() and (expect[:, 1:] > 0).all()  # the outer faces, the star's inner faces


_IDIR = np.array([[1, 2, 3], [0, 3, 2], [0, 1, 3], [0, 2, 1]])


def _host_tria_adjacency(triv):
    """MMG3D_hashTria's adjt: edge j (opposite local vertex j) paired only
    when exactly two trias share it"""
    edges = {}
    for t, tri in enumerate(triv.tolist()):
        for j in range(3):
            edges.setdefault(tuple(sorted((tri[(j + 1) % 3], tri[(j + 2) % 3]))), []).append(3 * (t + 1) + j)
    adjt = np.zeros(triv.shape, np.int32)
    for codes in edges.values():
        if len(codes) == 2:
            a, b = codes
            adjt[a // 3 - 1, a % 3], adjt[b // 3 - 1, b % 3] = b, a
    return adjt


@pytest.mark.gpu
@pytest.mark.parametrize("use_tet8", [True, False])
def test_snapshot_boundary_of_a_multi_material_mesh(use_tet8):
    """With tetra references the boundary trias are the faces without a
    neighbour and the interface faces seen from the larger reference
    (MMG5_chkBdryTria's rule restated in pmmg_snapshot.hip), in (tetra, face)
    order, oriented by MMG5_idir."""
    bg = synth.lattice(synth.CUBE, 6)
    cx = bg.xyz[bg.tetv - 1, 0].mean(axis=1)
    tref = (np.floor(3 * (cx - cx.min()) / np.ptp(cx) * 0.999) + 1).astype(np.int32)
    assert len(set(tref.tolist())) == 3
    nbr = np.maximum(bg.adja // 4 - 1, 0)
    keep = (bg.adja == 0) | (tref[:, None] > tref[nbr])
    k, i = np.nonzero(keep)
    expect = bg.tetv[k[:, None], _IDIR[i]].astype(np.int32)
    assert expect.shape[0] > bg.nt  # interface faces beside the outer boundary
    with TransferContext(0) as ctx:
        tetv = ctx.upload(bg.tetv)
        adja, tet8 = ctx.build_adjacency(bg.np, tetv)
        d_tref = ctx.upload(tref)
        if use_tet8:
            triv, adjt = ctx.build_boundary(bg.np, tet8=tet8, tref=d_tref)
        else:
            triv, adjt = ctx.build_boundary(bg.np, tetv=tetv, adja=adja, tref=d_tref)
        np.testing.assert_array_equal(triv.download(), expect)
        np.testing.assert_array_equal(adjt.download(), _host_tria_adjacency(expect))


@pytest.mark.gpu
def test_snapshot_rejects_invalid_connectivity():
    bg = synth.lattice(synth.CUBE, 2)
    with TransferContext(0) as ctx:
        bad = bg.tetv.copy()
        bad[3, 2] = bg.np + 5  # id out of range
        with pytest.raises(RuntimeError, match="vertex ids"):
            ctx.build_adjacency(bg.np, ctx.upload(bad))
        bad = bg.tetv.copy()
        bad[0, 1] = bad[0, 0]  # repeated id
        with pytest.raises(RuntimeError, match="vertex ids"):
            ctx.build_adjacency(bg.np, ctx.upload(bad))
        # a third tetra on an interior face: non-manifold
        k = int(np.nonzero((bg.adja > 0).all(axis=1))[0][0]) if (bg.adja > 0).all(axis=1).any() else 0
        extra = np.concatenate([bg.tetv, bg.tetv[k:k + 1, [1, 0, 2, 3]]]).astype(np.int32)
        with pytest.raises(RuntimeError, match="more than two"):
            ctx.build_adjacency(bg.np, ctx.upload(np.ascontiguousarray(extra)))


@pytest.mark.gpu
@pytest.mark.parametrize("host_mode", [True, False])
def test_failed_snapshot_drops_the_background(host_mode):
    """A background whose device snapshot fails (non-manifold: a third tetra
    on an interior face) must not stay usable: its adjacency is partly
    written.  Host mode defers the snapshot to a host thread (the failure is
    reported by the next call); every later locate_interp fails cleanly until
    a valid set_background."""
    case = make_case(kind=synth.CUBE, n_old=3, n_new=4, with_ref=False)
    bg = case["bg"]
    k = int(np.nonzero((bg.adja > 0).all(axis=1))[0][0])
    extra = np.ascontiguousarray(np.concatenate([bg.tetv, bg.tetv[k:k + 1, [1, 0, 2, 3]]]).astype(np.int32))
    q, pc = case["new"].xyz, case["pclass"]
    n = q.shape[0]
    with TransferContext(0) as ctx:
        def locate():
            mo = np.full((n, case["met"].shape[1]), np.nan)
            fo = [np.full((n, f.shape[1]), np.nan) for f in case["fields"]]
            ctx.locate_interp(q, pc, mo, fo, np.zeros(n, np.int32), np.zeros(n, np.int8))

        if host_mode:
            ctx.set_background(bg.xyz, extra, None, None, None, case["hausd"])  # snapshot deferred
            ctx.set_solutions(case["met"], case["fields"])  # uploads beside the snapshot (does not join it)
        else:
            with pytest.raises(RuntimeError, match="more than two"):
                ctx.set_background(ctx.upload(bg.xyz), ctx.upload(extra), None, None, None, case["hausd"])
        for _ in range(2):
            with pytest.raises(RuntimeError):
                locate()
        # a valid background makes the context usable again
        ctx.set_background(bg.xyz, bg.tetv, None, None, None, case["hausd"])
        ctx.set_solutions(case["met"], case["fields"])
        locate()


@pytest.mark.gpu
def test_transfer_on_device_snapshot_is_identical():
    """Locate + interpolate against the device-built background gives the
    same outputs bit for bit as against the host-built arrays."""
    case = make_case(kind=synth.SHELL, n_old=12, n_new=16, with_ref=False)
    ref = run_gpu(case)
    bg = case["bg"]
    with TransferContext(0) as ctx:
        xyz = ctx.upload(bg.xyz)
        _, _, tet8, triv, adjt = _snapshot(ctx, bg)
        ctx.set_background_tet8(xyz, tet8, triv, adjt, case["hausd"])
        met = ctx.upload(case["met"])
        fields = [ctx.upload(f) for f in case["fields"]]
        ctx.set_solutions(met, fields)
        q, pc = ctx.upload(case["new"].xyz), ctx.upload(case["pclass"])
        mo = ctx.upload(np.full((q.shape[0], case["met"].shape[1]), np.nan))
        fo = [ctx.upload(np.full((q.shape[0], f.shape[1]), np.nan)) for f in case["fields"]]
        el, hit = ctx.empty((q.shape[0],), np.int32), ctx.empty((q.shape[0],), np.int8)
        ctx.locate_interp(q, pc, mo, fo, el, hit)
        np.testing.assert_array_equal(el.download(), ref["elem"])
        np.testing.assert_array_equal(hit.download(), ref["hit"])
        np.testing.assert_array_equal(mo.download(), ref["met"])
        for a, b in zip(fo, ref["fields"]):
            np.testing.assert_array_equal(a.download(), b)


@pytest.mark.gpu
def test_snapshot_full_size_cfg3():
    """cfg3 background (20.25M tetra, 3.4M vertices): bit-exact against the
    host builder."""
    bg = synth.lattice(synth.CUBE, 150)
    with TransferContext(0) as ctx:
        _, adja, tet8, triv, adjt = _snapshot(ctx, bg)
        assert np.array_equal(adja.download(), bg.adja)
        assert np.array_equal(triv.download(), bg.triv)
        assert np.array_equal(adjt.download(), bg.adjt)


@pytest.mark.gpu
def test_outputs_in_torch_tensors():
    """Device-mode outputs may be torch tensors in HBM (the Morton-sharded
    bench all-gathers them in place): same results as numpy host mode."""
    import torch
    case = make_case(kind=synth.CUBE, n_old=6, n_new=9, with_ref=False)
    ref = run_gpu(case)
    bg = case["bg"]
    dev = torch.device("cuda", 0)
    with TransferContext(0) as ctx:
        ctx.set_background(ctx.upload(bg.xyz), ctx.upload(bg.tetv), ctx.upload(bg.adja), ctx.upload(bg.triv),
                           ctx.upload(bg.adjt), case["hausd"])
        ctx.set_solutions(ctx.upload(case["met"]), [ctx.upload(f) for f in case["fields"]])
        npn = case["new"].np
        mo = torch.full((npn, case["met"].shape[1]), float("nan"), dtype=torch.float64, device=dev)
        fo = [torch.full((npn, f.shape[1]), float("nan"), dtype=torch.float64, device=dev) for f in case["fields"]]
        el = torch.zeros(npn, dtype=torch.int32, device=dev)
        ctx.locate_interp(ctx.upload(case["new"].xyz), ctx.upload(case["pclass"]), mo, fo, el, None)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(el.cpu().numpy(), ref["elem"])
        np.testing.assert_array_equal(mo.cpu().numpy(), ref["met"])
        for a, b in zip(fo, ref["fields"]):
            np.testing.assert_array_equal(a.cpu().numpy(), b)
