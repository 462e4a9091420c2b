"""Python front-end of the C-ABI (include/parmmg_hip.h) and of the C host
layer (csrc/pmmg_host.h).

``TransferContext`` wraps one ``pmmg_hip_ctx``.  Host-mode calls take numpy
arrays; device-mode calls take ``DeviceArray`` handles (raw HIP allocations
made through the module itself), which is what the benchmark uses to keep
every input resident in HBM.

``interp_metrics_and_fields`` mirrors the reference driver
``PMMG_interpMetricsAndFields(parmesh, permNodGlob)``
(src/interpmesh_pmmg.c:663-741) group by group, through the C host layer.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._native import HipStats, hip_lib, host_lib

HOST, DEVICE = 0, 1
PT_SKIP, PT_VOL, PT_BDY = 0, 1, 2

HIT_NAMES = {
    0: "none", 1: "vol_walk", 2: "vol_exhaust", 3: "vol_closest", 4: "bdy_face", 5: "bdy_edge", 6: "bdy_vertex",
    7: "bdy_wedge", 8: "bdy_cone", 9: "bdy_exhaust", 10: "bdy_stale", 11: "bdy_closest",
}


def _p(a):
    if a is None:
        return None
    if isinstance(a, DeviceArray):
        return ctypes.c_void_p(a.ptr)
    if getattr(a, "is_cuda", False):  # torch tensor in HBM (e.g. an all-gather buffer)
        if not a.is_contiguous():
            raise ValueError("device tensors passed to the C-ABI must be contiguous")
        return ctypes.c_void_p(a.data_ptr())
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("arrays passed to the C-ABI must be C-contiguous")
    return a.ctypes.data_as(ctypes.c_void_p)


def _is_dev(a) -> bool:
    return isinstance(a, DeviceArray) or bool(getattr(a, "is_cuda", False))


@dataclass
class DeviceArray:
    ptr: int
    nbytes: int
    shape: tuple
    dtype: np.dtype
    ctx: "TransferContext"

    def download(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        if not self.ctx.lib.pmmg_hip_memcpy_d2h(self.ctx.h, _p(out), ctypes.c_void_p(self.ptr), self.nbytes):
            raise RuntimeError(self.ctx.error())
        return out

    def free(self) -> None:
        if self.ptr:
            self.ctx.lib.pmmg_hip_free(self.ctx.h, ctypes.c_void_p(self.ptr))
            self.ptr = 0


def device_count() -> int:
    return int(hip_lib().pmmg_hip_device_count())


def pack_tet8(tetv: np.ndarray, adja: np.ndarray) -> np.ndarray:
    """Packed tetra records {v0..v3, adja0..adja3} (include/parmmg_hip.h,
    pmmg_hip_set_background_tet8): what a host shim builds while packing
    MMG5_Tetra.v."""
    return np.ascontiguousarray(np.hstack([np.asarray(tetv, np.int32), np.asarray(adja, np.int32)]))


def pack_solutions(met, fields):
    """Packed per-vertex records of the metric and fields
    (pmmg_hip_set_solutions_packed): size-6 slots first (even columns), then
    size-3, then size-1, the record padded to an even number of doubles.
    Returns (rec, met_size, met_off, field_sizes, field_offs)."""
    slots = ([("m", met)] if met is not None else []) + [(j, f) for j, f in enumerate(fields)]
    order = sorted(slots, key=lambda s: -s[1].shape[1])  # stable: 6, 3, 1
    off, col = {}, 0
    for key, a in order:
        off[key] = col
        col += a.shape[1]
    stride = col + (col & 1)
    npt = (met if met is not None else fields[0]).shape[0]
    rec = np.zeros((npt, max(stride, 2)), np.float64)
    for key, a in slots:
        rec[:, off[key]:off[key] + a.shape[1]] = a
    msize = 0 if met is None else met.shape[1]
    return (rec, msize, off.get("m", 0), [f.shape[1] for f in fields], [off[j] for j in range(len(fields))])


class TransferContext:
    """One ``pmmg_hip_ctx`` on a HIP device."""

    def __init__(self, device: int = 0, sort: bool | None = None, scan: bool = False, fused: bool = False):
        """Volume points are located by per-query adjacency walks (default)
        or, with scan=True, by the tetra-centric scan.  sort=None picks the
        query order automatically (Morton-bin unless the numbering is
        coherent); True / False force binning / input order.  fused=True runs
        the walk and the interpolation as one kernel."""
        self.lib = hip_lib()
        opts = (0 if sort is None else (2 if sort else 1)) | (4 if scan else 0) | (8 if fused else 0)
        self.h = self.lib.pmmg_hip_create(int(device), opts)
        if not self.h:
            raise RuntimeError(f"pmmg_hip_create({device}) failed: no usable HIP device (the transfer step has "
                               "no CPU fallback)")
        self._keep: list = []

    def close(self) -> None:
        if self.h:
            self.lib.pmmg_hip_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self) -> str:
        e = self.lib.pmmg_hip_last_error(self.h)
        return e.decode() if e else ""

    def _ck(self, ok: int, what: str) -> None:
        if not ok:
            raise RuntimeError(f"{what} failed: {self.error()}")

    # ------------------------------------------------------------------ device memory
    def upload(self, a: np.ndarray) -> DeviceArray:
        a = np.ascontiguousarray(a)
        ptr = self.lib.pmmg_hip_malloc(self.h, a.nbytes)
        if not ptr:
            raise RuntimeError(self.error())
        self._ck(self.lib.pmmg_hip_memcpy_h2d(self.h, ctypes.c_void_p(ptr), _p(a), a.nbytes), "h2d")
        return DeviceArray(ptr, a.nbytes, a.shape, a.dtype, self)

    def empty(self, shape, dtype) -> DeviceArray:
        dtype = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * dtype.itemsize
        ptr = self.lib.pmmg_hip_malloc(self.h, nbytes)
        if not ptr:
            raise RuntimeError(self.error())
        return DeviceArray(ptr, nbytes, tuple(shape), dtype, self)

    # ------------------------------------------------------------------ C-ABI
    def set_background(self, xyz, tetv, adja, triv, adjt, hausd: float) -> None:
        where = DEVICE if _is_dev(xyz) else HOST
        npt, ne, nt = xyz.shape[0], tetv.shape[0], triv.shape[0]
        self._keep = [xyz, tetv, adja, triv, adjt]
        self._ck(self.lib.pmmg_hip_set_background(self.h, npt, _p(xyz), ne, _p(tetv), _p(adja), nt, _p(triv),
                                                  _p(adjt), float(hausd), where), "set_background")

    def set_background_tet8(self, xyz, tet8, triv, adjt, hausd: float) -> None:
        """Background with packed {v[4], adja[4]} tetra records (pack_tet8)."""
        where = DEVICE if _is_dev(xyz) else HOST
        npt, ne, nt = xyz.shape[0], tet8.shape[0], triv.shape[0]
        if tet8.shape[1] != 8:
            raise ValueError("tet8 must have 8 ints per tetra")
        self._keep = [xyz, tet8, triv, adjt]
        self._ck(self.lib.pmmg_hip_set_background_tet8(self.h, npt, _p(xyz), ne, _p(tet8), nt, _p(triv), _p(adjt),
                                                       float(hausd), where), "set_background_tet8")

    # ------------------------------------------------------------------ background snapshot
    def build_adjacency(self, npt: int, tetv: DeviceArray, adja: bool = True, tet8: bool = True):
        """Device-side MMG3D_hashTetra: (adja, tet8) DeviceArrays (None when not requested)."""
        ne = tetv.shape[0]
        a = self.empty((ne, 4), np.int32) if adja else None
        t = self.empty((ne, 8), np.int32) if tet8 else None
        self._ck(self.lib.pmmg_hip_build_adjacency(self.h, int(npt), ne, _p(tetv), _p(a), _p(t)), "build_adjacency")
        return a, t

    def build_boundary(self, npt: int, tet8: DeviceArray | None = None, tetv: DeviceArray | None = None,
                       adja: DeviceArray | None = None, adjt: bool = True):
        """Device-side MMG5_chkBdryTria + MMG3D_hashTria: (triv, adjt) DeviceArrays of nt rows."""
        ne = (tet8 if tet8 is not None else tetv).shape[0]
        nt = ctypes.c_int(0)
        # capacity 0: the call only counts (it fails when there are trias, with nt set)
        self.lib.pmmg_hip_build_boundary(self.h, int(npt), ne, _p(tet8), _p(tetv), _p(adja), 0, ctypes.byref(nt),
                                         None, None)
        n = nt.value
        triv = self.empty((n, 3), np.int32)
        at = self.empty((n, 3), np.int32) if adjt else None
        self._ck(self.lib.pmmg_hip_build_boundary(self.h, int(npt), ne, _p(tet8), _p(tetv), _p(adja), n,
                                                  ctypes.byref(nt), _p(triv), _p(at)), "build_boundary")
        return triv, at

    def set_solutions(self, met, fields) -> None:
        fields = list(fields)
        where = DEVICE if (_is_dev(met) or (fields and _is_dev(fields[0]))) else HOST
        msize = 0 if met is None else int(met.shape[1])
        sizes = (ctypes.c_int * max(1, len(fields)))(*[int(f.shape[1]) for f in fields])
        ptrs = (ctypes.c_void_p * max(1, len(fields)))(*[_p(f) for f in fields])
        self._sol_keep = [met, fields, sizes, ptrs]
        self._ck(self.lib.pmmg_hip_set_solutions(self.h, msize, _p(met), len(fields), sizes, ptrs, where),
                 "set_solutions")

    def set_solutions_packed(self, rec, met_size: int, met_off: int, field_sizes, field_offs) -> None:
        """Solutions as packed per-vertex records (pack_solutions)."""
        where = DEVICE if _is_dev(rec) else HOST
        nf = len(field_sizes)
        sizes = (ctypes.c_int * max(1, nf))(*[int(x) for x in field_sizes])
        offs = (ctypes.c_int * max(1, nf))(*[int(x) for x in field_offs])
        self._sol_keep = [rec, sizes, offs]
        self._ck(self.lib.pmmg_hip_set_solutions_packed(self.h, int(met_size), int(met_off), nf, sizes, offs, _p(rec),
                                                        int(rec.shape[1]), where), "set_solutions_packed")

    def locate_interp(self, xyz_new, pclass, met_out, fields_out, elem_out=None, hit_out=None,
                      sync: bool = True) -> HipStats | None:
        where = DEVICE if _is_dev(xyz_new) else HOST
        fields_out = list(fields_out)
        ptrs = (ctypes.c_void_p * max(1, len(fields_out)))(*[_p(f) for f in fields_out])
        st = HipStats()
        self._ck(self.lib.pmmg_hip_locate_interp(self.h, xyz_new.shape[0], _p(xyz_new), _p(pclass), _p(met_out),
                                                 ptrs, _p(elem_out), _p(hit_out),
                                                 ctypes.byref(st) if (sync or where == HOST) else None, where),
                 "locate_interp")
        return st if (sync or where == HOST) else None

    def tetra_qual(self, xyz, tetv, met=None, qual=None):
        """PMMG_tetraQual's MMG3D_tetraQual(mesh, met, 1) on the device
        (pmmg_hip_tetra_qual): device arrays (the metric where locate_interp
        wrote it).  Returns (qual DeviceArray [ne], ALPHAD * min quality)."""
        if not (_is_dev(xyz) and _is_dev(tetv) and (met is None or _is_dev(met))):
            raise ValueError("tetra_qual takes device arrays")
        ne = tetv.shape[0]
        qual = qual if qual is not None else self.empty((ne,), np.float64)
        mn = ctypes.c_double(0.0)
        self._ck(self.lib.pmmg_hip_tetra_qual(self.h, xyz.shape[0], _p(xyz), ne, _p(tetv),
                                              0 if met is None else int(met.shape[1]), _p(met), _p(qual),
                                              ctypes.byref(mn)), "tetra_qual")
        return qual, mn.value

    def sync(self) -> HipStats:
        st = HipStats()
        self._ck(self.lib.pmmg_hip_sync(self.h, ctypes.byref(st)), "sync")
        return st


def transfer(mesh_old, met, fields, xyz_new, pclass, hausd=0.01, device=0, sort=None, ctx=None):
    """One-shot host-mode transfer: returns (met_new, fields_new, elem, hit, stats)."""
    own = ctx is None
    ctx = ctx or TransferContext(device, sort=sort)
    try:
        ctx.set_background(mesh_old.xyz, mesh_old.tetv, mesh_old.adja, mesh_old.triv, mesh_old.adjt, hausd)
        ctx.set_solutions(met, fields)
        npn = xyz_new.shape[0]
        met_out = None if met is None else np.zeros((npn, met.shape[1]))
        f_out = [np.zeros((npn, f.shape[1])) for f in fields]
        elem = np.zeros(npn, np.int32)
        hit = np.zeros(npn, np.int8)
        st = ctx.locate_interp(np.ascontiguousarray(xyz_new), np.ascontiguousarray(pclass), met_out, f_out, elem, hit)
        return met_out, f_out, elem, hit, st
    finally:
        if own:
            ctx.close()


# ---------------------------------------------------------------- C host layer (csrc/pmmg_host.h)

class OldGroup(ctypes.Structure):
    _fields_ = [("np", ctypes.c_int), ("ne", ctypes.c_int), ("nt", ctypes.c_int),
                ("xyz", ctypes.c_void_p), ("tetv", ctypes.c_void_p), ("adja", ctypes.c_void_p),
                ("triv", ctypes.c_void_p), ("adjt", ctypes.c_void_p), ("hausd", ctypes.c_double),
                ("met_size", ctypes.c_int), ("met", ctypes.c_void_p), ("nfield", ctypes.c_int),
                ("field_size", ctypes.c_void_p), ("field", ctypes.c_void_p)]


class NewGroup(ctypes.Structure):
    _fields_ = [("np", ctypes.c_int), ("ne", ctypes.c_int), ("xyz", ctypes.c_void_p), ("tag", ctypes.c_void_p),
                ("tetv", ctypes.c_void_p), ("met", ctypes.c_void_p), ("field", ctypes.c_void_p),
                ("elem", ctypes.c_void_p), ("hit", ctypes.c_void_p)]


TAG_REQ, TAG_BDY, TAG_NUL = 1 << 2, 1 << 4, 1 << 14


def interp_metrics_and_fields(ctx: TransferContext, old_groups, new_groups, input_met: int = 1, hsiz: float = 0.0):
    """PMMG_interpMetricsAndFields over groups (src/interpmesh_pmmg.c:663-741).

    ``old_groups``: list of dicts {mesh, met, fields, hausd};
    ``new_groups``: list of dicts {xyz, tag, tetv, met, fields[, elem, hit]} whose
    ``met`` / ``fields`` arrays are filled in place.  Returns (ier, stats)."""
    lib = host_lib()
    fn = lib.pmmg_interp_metrics_and_fields
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                   ctypes.POINTER(HipStats)]
    ng = len(old_groups)
    olds = (OldGroup * ng)()
    news = (NewGroup * ng)()
    keep = []
    for i, (o, g) in enumerate(zip(old_groups, new_groups)):
        m = o["mesh"]
        fs = list(o.get("fields", []))
        fsz = (ctypes.c_int * max(1, len(fs)))(*[f.shape[1] for f in fs])
        fpt = (ctypes.c_void_p * max(1, len(fs)))(*[_p(f) for f in fs])
        met = o.get("met")
        olds[i] = OldGroup(m.np, m.ne, m.nt, _p(m.xyz), _p(m.tetv), _p(m.adja), _p(m.triv), _p(m.adjt),
                           float(o.get("hausd", 0.01)), 0 if met is None else met.shape[1], _p(met), len(fs),
                           ctypes.cast(fsz, ctypes.c_void_p), ctypes.cast(fpt, ctypes.c_void_p))
        gf = list(g.get("fields", []))
        gpt = (ctypes.c_void_p * max(1, len(gf)))(*[_p(f) for f in gf])
        news[i] = NewGroup(g["xyz"].shape[0], g["tetv"].shape[0], _p(g["xyz"]), _p(g.get("tag")), _p(g["tetv"]),
                           _p(g.get("met")), ctypes.cast(gpt, ctypes.c_void_p), _p(g.get("elem")), _p(g.get("hit")))
        keep += [fsz, fpt, gpt]
    st = HipStats()
    ier = fn(ctx.h, ng, ctypes.cast(olds, ctypes.c_void_p), ctypes.cast(news, ctypes.c_void_p), int(input_met),
             float(hsiz), ctypes.byref(st))
    return ier, st
