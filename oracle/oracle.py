"""ctypes front-end of the CPU oracle (oracle/pmmg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline.  The product
path (parmmg_amd/) never imports it.  Parity status: see pmmg_oracle.h
("parity unpinned" at the Mmg arithmetic boundary).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liboracle.so")

MODE_FAITHFUL, MODE_FRESH = 0, 1
EPS = 1.0e-06


class _Bg(ctypes.Structure):
    _fields_ = [("np", ctypes.c_int), ("ne", ctypes.c_int), ("nt", ctypes.c_int),
                ("xyz", ctypes.c_void_p), ("tetv", ctypes.c_void_p), ("adja", ctypes.c_void_p),
                ("triv", ctypes.c_void_p), ("adjt", ctypes.c_void_p), ("hausd", ctypes.c_double),
                ("met_size", ctypes.c_int), ("met", ctypes.c_void_p), ("nfield", ctypes.c_int),
                ("field_size", ctypes.c_void_p), ("field", ctypes.c_void_p)]


class _Q(ctypes.Structure):
    _fields_ = [("np", ctypes.c_int), ("xyz", ctypes.c_void_p), ("pclass", ctypes.c_void_p),
                ("nvisit", ctypes.c_int), ("visit", ctypes.c_void_p)]


class _Out(ctypes.Structure):
    _fields_ = [("met", ctypes.c_void_p), ("field", ctypes.c_void_p), ("elem", ctypes.c_void_p),
                ("hit", ctypes.c_void_p), ("loc", ctypes.c_void_p), ("minbary", ctypes.c_void_p),
                ("steps", ctypes.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(SO)
        vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
        L.orc_interp_mesh.argtypes = [vp, vp, vp, ci, vp]
        L.orc_interp_mesh.restype = ci
        L.orc_interp_mesh_budget.argtypes = [vp, vp, vp, ci, cd, vp]
        L.orc_interp_mesh_budget.restype = ci
        L.orc_interp_mesh_mt.argtypes = [vp, vp, vp, ci, ci, cd, vp]
        L.orc_interp_mesh_mt.restype = ci
        L.orc_eval_in_element.argtypes = [vp, vp, ci, ci, ci, ci, vp, vp]
        L.orc_eval_in_element.restype = ci
        L.orc_tetra_minbary.argtypes = [vp, ci, vp]
        L.orc_tetra_minbary.restype = cd
        L.orc_tria_accepts.argtypes = [vp, ci, vp, vp]
        L.orc_tria_accepts.restype = ci
        for n in ("orc_first_accepting_tetra", "orc_closest_tetra", "orc_first_accepting_tria", "orc_closest_tria"):
            getattr(L, n).argtypes = [vp, vp]
            getattr(L, n).restype = ci
        L.orc_closest_value.argtypes = [vp, ci, vp]
        L.orc_closest_value.restype = cd
        L.orc_wedge_test.argtypes = [vp, ci, ci, vp]
        L.orc_wedge_test.restype = ci
        L.orc_cone_test.argtypes = [vp, ci, ci, vp]
        L.orc_cone_test.restype = ci
        L.orc_invmat.argtypes = [vp, vp]
        L.orc_invmat.restype = ci
        L.orc_tetra_qual.argtypes = [ci, vp, ci, vp, ci, vp, vp]
        L.orc_tetra_qual.restype = cd
        L.orc_face_wgt.argtypes = [vp, vp, ci, ci, vp]
        L.orc_face_wgt.restype = cd
        L.orc_compute_wgt_mesh.argtypes = [ci, vp, vp, vp, vp, ci, vp, ci, vp]
        L.orc_compute_wgt_mesh.restype = None
        L.orc_check_batch.argtypes = [vp, vp, vp, vp, ctypes.c_int64, vp, vp, vp, vp, vp, vp, vp, ci, cd, vp]
        L.orc_check_batch.restype = ci
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class CheckReport(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("exact", ctypes.c_int64), ("class_i", ctypes.c_int64),
                ("class_i_same", ctypes.c_int64), ("accept_fail", ctypes.c_int64), ("value_fail", ctypes.c_int64),
                ("unprocessed", ctypes.c_int64), ("skipped_written", ctypes.c_int64), ("first_fail", ctypes.c_int64),
                ("maxrel", ctypes.c_double), ("hits", ctypes.c_int64 * 16)]

    def as_dict(self) -> dict:
        d = {name: getattr(self, name) for name, _ in self._fields_ if name != "hits"}
        d["hits"] = {h: int(self.hits[h]) for h in range(16) if self.hits[h]}
        return d


class Background:
    """Holds an orc_background built from a Mesh + solutions (keeps arrays alive)."""

    def __init__(self, mesh, met, fields, hausd=0.01):
        self.mesh = mesh
        self.met = None if met is None else np.ascontiguousarray(met, np.float64)
        self.fields = [np.ascontiguousarray(f, np.float64) for f in fields]
        self._fsz = (ctypes.c_int * max(1, len(self.fields)))(*[f.shape[1] for f in self.fields])
        self._fpt = (ctypes.c_void_p * max(1, len(self.fields)))(*[_p(f) for f in self.fields])
        self.s = _Bg(mesh.np, mesh.ne, mesh.nt, _p(mesh.xyz), _p(mesh.tetv), _p(mesh.adja), _p(mesh.triv),
                     _p(mesh.adjt), float(hausd), 0 if self.met is None else self.met.shape[1], _p(self.met),
                     len(self.fields), ctypes.cast(self._fsz, ctypes.c_void_p),
                     ctypes.cast(self._fpt, ctypes.c_void_p))

    @property
    def ref(self):
        return ctypes.byref(self.s)


def run(bg: Background, xyz_new, pclass, visit, mode=MODE_FAITHFUL, budget_s: float = 0.0, threads: int = 0):
    """Sequential reference-order run.  Returns dict of per-point arrays.
    With budget_s > 0 the locate+interp phase stops after about that many
    seconds; out["nvisited"] is the number of visit entries processed.
    threads > 0: the threaded driver (visit[] split into `threads` ranges)."""
    xyz_new = np.ascontiguousarray(xyz_new, np.float64)
    pclass = np.ascontiguousarray(pclass, np.uint8)
    visit = np.ascontiguousarray(visit, np.int32)
    npn = xyz_new.shape[0]
    out = {
        "met": None if bg.met is None else np.full((npn, bg.met.shape[1]), np.nan),
        "fields": [np.full((npn, f.shape[1]), np.nan) for f in bg.fields],
        "elem": np.zeros(npn, np.int32), "hit": np.zeros(npn, np.int8), "loc": np.full(npn, -1, np.int8),
        "minbary": np.zeros(npn), "steps": np.zeros(npn, np.int32),
    }
    fpt = (ctypes.c_void_p * max(1, len(out["fields"])))(*[_p(f) for f in out["fields"]])
    o = _Out(_p(out["met"]), ctypes.cast(fpt, ctypes.c_void_p), _p(out["elem"]), _p(out["hit"]), _p(out["loc"]),
             _p(out["minbary"]), _p(out["steps"]))
    q = _Q(npn, _p(xyz_new), _p(pclass), visit.shape[0], _p(visit))
    timing = (ctypes.c_double * 2)()
    if threads > 0:
        nv = lib().orc_interp_mesh_mt(bg.ref, ctypes.byref(q), ctypes.byref(o), int(mode), int(threads),
                                      float(budget_s), timing)
    else:
        nv = lib().orc_interp_mesh_budget(bg.ref, ctypes.byref(q), ctypes.byref(o), int(mode), float(budget_s),
                                          timing)
    if nv < 0:
        raise RuntimeError("oracle run failed")
    out["nvisited"] = nv
    out["t_precompute"], out["t_locate"] = timing[0], timing[1]
    return out


def eval_in_element(bg: Background, x, is_bdy, elem, hit, loc):
    """Values the reference arithmetic gives for x evaluated in (elem, hit, loc)."""
    x = np.ascontiguousarray(x, np.float64)
    met = None if bg.met is None else np.full(bg.met.shape[1], np.nan)
    fr = [np.full(f.shape[1], np.nan) for f in bg.fields]
    fpt = (ctypes.c_void_p * max(1, len(fr)))(*[_p(f) for f in fr])
    ok = lib().orc_eval_in_element(bg.ref, _p(x), int(is_bdy), int(elem), int(hit), int(loc), _p(met),
                                   ctypes.cast(fpt, ctypes.c_void_p))
    if not ok:
        raise ValueError(f"cannot evaluate hit={hit} elem={elem}")
    return met, fr


def tetra_minbary(bg, k, x):
    return lib().orc_tetra_minbary(bg.ref, int(k), _p(np.ascontiguousarray(x, np.float64)))


def tria_accepts(bg, k, x):
    mb = ctypes.c_double()
    ok = lib().orc_tria_accepts(bg.ref, int(k), _p(np.ascontiguousarray(x, np.float64)), ctypes.byref(mb))
    return bool(ok), mb.value


def first_accepting_tetra(bg, x):
    return lib().orc_first_accepting_tetra(bg.ref, _p(np.ascontiguousarray(x, np.float64)))


def closest_tetra(bg, x):
    return lib().orc_closest_tetra(bg.ref, _p(np.ascontiguousarray(x, np.float64)))


def closest_value(bg, k, x):
    return lib().orc_closest_value(bg.ref, int(k), _p(np.ascontiguousarray(x, np.float64)))


def first_accepting_tria(bg, x):
    return lib().orc_first_accepting_tria(bg.ref, _p(np.ascontiguousarray(x, np.float64)))


def closest_tria(bg, x):
    return lib().orc_closest_tria(bg.ref, _p(np.ascontiguousarray(x, np.float64)))


def wedge_test(bg, k, l, x):
    return lib().orc_wedge_test(bg.ref, int(k), int(l), _p(np.ascontiguousarray(x, np.float64)))


def cone_test(bg, k, iloc, x):
    return lib().orc_cone_test(bg.ref, int(k), int(iloc), _p(np.ascontiguousarray(x, np.float64)))


def check_batch(bg: Background, xyz, pclass, elem, hit, met_out, fields_out, idx=None, ref=None,
                threads: int = 0, rel_tol: float = 1e-12) -> dict:
    """The parity contract of tests/parity.py::check over many points in C
    (orc_check_batch): acceptance of each point's element for its hit kind,
    values of the reference interpolator in that element (bit-exact count,
    max relative error), and with `ref` (an oracle run) class (i) identity.
    idx: 0-based points to check (default: all)."""
    xyz = np.ascontiguousarray(xyz, np.float64)
    pclass = np.ascontiguousarray(pclass, np.uint8)
    elem = np.ascontiguousarray(elem, np.int32)
    hit = np.ascontiguousarray(hit, np.int8)
    met_out = None if met_out is None else np.ascontiguousarray(met_out, np.float64)
    fo = [np.ascontiguousarray(f, np.float64) for f in fields_out]
    fpt = (ctypes.c_void_p * max(1, len(fo)))(*[_p(f) for f in fo])
    if idx is None:
        n = xyz.shape[0]
    else:
        idx = np.ascontiguousarray(idx, np.int32)
        n = idx.shape[0]
    r_elem = r_hit = r_mb = None
    if ref is not None:
        r_elem = np.ascontiguousarray(ref["elem"], np.int32)
        r_hit = np.ascontiguousarray(ref["hit"], np.int8)
        r_mb = np.ascontiguousarray(ref["minbary"], np.float64)
    rep = CheckReport()
    threads = threads or min(16, os.cpu_count() or 1)
    ok = lib().orc_check_batch(bg.ref, _p(xyz), _p(pclass), _p(idx), int(n), _p(elem), _p(hit), _p(met_out),
                               ctypes.cast(fpt, ctypes.c_void_p), _p(r_elem), _p(r_hit), _p(r_mb), int(threads),
                               float(rel_tol), ctypes.byref(rep))
    if not ok:
        raise RuntimeError("orc_check_batch failed")
    return rep.as_dict()


def invmat(m):
    m = np.ascontiguousarray(m, np.float64)
    mi = np.zeros(6)
    ok = lib().orc_invmat(_p(m), _p(mi))
    return bool(ok), mi


def tetra_qual(xyz, tetv, met=None):
    """MMG3D_tetraQual(mesh, met, 1) restated: (qual[ne], ALPHAD * min)."""
    xyz = np.ascontiguousarray(xyz, np.float64)
    tetv = np.ascontiguousarray(tetv, np.int32)
    met = None if met is None else np.ascontiguousarray(met, np.float64)
    qual = np.empty(tetv.shape[0], np.float64)
    mn = lib().orc_tetra_qual(xyz.shape[0], _p(xyz), tetv.shape[0], _p(tetv), 0 if met is None else met.shape[1],
                              _p(met), _p(qual))
    return qual, mn


def face_wgt(xyz, v, ifac, met=None):
    """PMMG_computeWgt of face ifac of the tetra with vertices v (1-based)."""
    xyz = np.ascontiguousarray(xyz, np.float64)
    v = np.ascontiguousarray(v, np.int32)
    met = None if met is None else np.ascontiguousarray(met, np.float64)
    return lib().orc_face_wgt(_p(xyz), _p(v), int(ifac), 0 if met is None else met.shape[1], _p(met))


def compute_wgt_mesh(xyz, tetv, xt, ftag, met, tag, qual):
    """PMMG_computeWgt_mesh restated: qual updated in place (a copy is returned)."""
    q = np.array(qual, np.float64, copy=True)
    xyz = np.ascontiguousarray(xyz, np.float64)
    tetv = np.ascontiguousarray(tetv, np.int32)
    xt = np.ascontiguousarray(xt, np.int32)
    ftag = np.ascontiguousarray(ftag, np.uint16)
    met = None if met is None else np.ascontiguousarray(met, np.float64)
    lib().orc_compute_wgt_mesh(tetv.shape[0], _p(tetv), _p(xt), _p(ftag), _p(xyz),
                               0 if met is None else met.shape[1], _p(met), int(tag), _p(q))
    return q
