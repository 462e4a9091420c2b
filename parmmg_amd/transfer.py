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

from ._native import HipGroup, HipStats, hip_lib, host_lib

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

    def zero(self) -> None:
        z = np.zeros(self.nbytes, np.uint8)
        if not self.ctx.lib.pmmg_hip_memcpy_h2d(self.ctx.h, ctypes.c_void_p(self.ptr), _p(z), self.nbytes):
            raise RuntimeError(self.ctx.error())

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


def pack_solutions(met, fields) -> np.ndarray:
    """Packed per-vertex solution records [metric | field 0 | ...], stride
    rounded up to an even number of doubles (include/parmmg_hip.h,
    pmmg_hip_set_solutions_packed)."""
    cols = ([] if met is None else [np.asarray(met, np.float64)]) + [np.asarray(f, np.float64) for f in fields]
    k = sum(c.shape[1] for c in cols)
    rs = (k + 1) & ~1
    rec = np.zeros((cols[0].shape[0], rs), np.float64)
    o = 0
    for c in cols:
        rec[:, o:o + c.shape[1]] = c
        o += c.shape[1]
    return rec


class TransferContext:
    """One ``pmmg_hip_ctx`` on a HIP device."""

    def __init__(self, device: int = 0, sort: bool | None = None):
        """sort=None picks the query order on the device (Morton-bin unless
        the numbering is spatially coherent); True / False force binning /
        input order."""
        self.lib = hip_lib()
        opts = 0 if sort is None else (2 if sort else 1)
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
        """adja None: adjacency built on the device; triv None: boundary trias
        and their adjacency built on the device; adjt None (triv given): tria
        adjacency built on the device."""
        where = DEVICE if _is_dev(xyz) else HOST
        npt, ne, nt = xyz.shape[0], tetv.shape[0], (-1 if triv is None else triv.shape[0])
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
    def build_adjacency(self, npt: int, tetv: DeviceArray, adja: bool = True, tet8: bool = True, out=None):
        """Device-side MMG3D_hashTetra: (adja, tet8) DeviceArrays (None when
        not requested); out = (adja, tet8) arrays to fill instead of new ones."""
        ne = tetv.shape[0]
        a = (out[0] if out and out[0] is not None else self.empty((ne, 4), np.int32)) if adja else None
        t = (out[1] if out and out[1] is not None else self.empty((ne, 8), np.int32)) if tet8 else None
        self._ck(self.lib.pmmg_hip_build_adjacency(self.h, int(npt), ne, _p(tetv), _p(a), _p(t)), "build_adjacency")
        return a, t

    def build_boundary(self, npt: int, tet8: DeviceArray | None = None, tetv: DeviceArray | None = None,
                       adja: DeviceArray | None = None, adjt: bool = True, tref: DeviceArray | None = None):
        """Device-side MMG5_chkBdryTria + MMG3D_hashTria: (triv, adjt) DeviceArrays of nt rows
        (tref: tetra references, for interface faces of a multi-material mesh)."""
        ne = (tet8 if tet8 is not None else tetv).shape[0]
        nt = ctypes.c_int(0)
        # capacity 0: the call only counts (it fails when there are trias, with nt set)
        self.lib.pmmg_hip_build_boundary(self.h, int(npt), ne, _p(tet8), _p(tetv), _p(adja), _p(tref), 0,
                                         ctypes.byref(nt), None, None)
        n = nt.value
        triv = self.empty((n, 3), np.int32)
        at = self.empty((n, 3), np.int32) if adjt else None
        self._ck(self.lib.pmmg_hip_build_boundary(self.h, int(npt), ne, _p(tet8), _p(tetv), _p(adja), _p(tref), n,
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

    def set_solutions_packed(self, rec, met_size: int, field_sizes) -> None:
        """Packed per-vertex records (pack_solutions) in host or device memory
        (pmmg_hip_set_solutions_packed)."""
        where = DEVICE if _is_dev(rec) else HOST
        sizes = (ctypes.c_int * max(1, len(field_sizes)))(*[int(x) for x in field_sizes])
        self._sol_keep = [rec, sizes]
        self._ck(self.lib.pmmg_hip_set_solutions_packed(self.h, int(met_size), len(field_sizes), sizes, _p(rec),
                                                        where), "set_solutions_packed")

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

    def locate_interp_rec(self, xyz_new, pclass, rec_out, elem_out=None, hit_out=None,
                          sync: bool = True) -> HipStats | None:
        """pmmg_hip_locate_interp_rec: device arrays; after set_solutions_packed,
        the new points' values as records of the packed layout (rec_out
        [np_new, RS])."""
        st = HipStats()
        self._ck(self.lib.pmmg_hip_locate_interp_rec(self.h, xyz_new.shape[0], _p(xyz_new), _p(pclass), _p(rec_out),
                                                     _p(elem_out), _p(hit_out), ctypes.byref(st) if sync else None,
                                                     DEVICE), "locate_interp_rec")
        return st if sync else None

    def locate_interp_groups(self, groups, sync: bool = True) -> HipStats | None:
        """pmmg_hip_locate_interp_groups: many groups in one call, device
        arrays only.  Each group is a dict {xyz, tet8 | (tetv, adja), triv,
        adjt, hausd, met, fields, xyz_new, pclass, met_out, fields_out[,
        elem_out, hit_out]}.  sync: wait and return the summed counters;
        otherwise only enqueue (pmmg_hip_sync before reading outputs)."""
        G = (HipGroup * max(1, len(groups)))()
        keep = []
        for i, g in enumerate(groups):
            arrays = [g["xyz"], g.get("tet8"), g.get("tetv"), g.get("adja"), g["triv"], g.get("adjt"), g.get("met"),
                      g["xyz_new"], g["pclass"], g.get("met_out"), g.get("elem_out"), g.get("hit_out")]
            arrays += list(g.get("fields", [])) + list(g.get("fields_out", []))
            if not all(a is None or _is_dev(a) for a in arrays):
                raise ValueError(f"group {i}: locate_interp_groups takes device arrays")
            fs, fo = list(g.get("fields", [])), list(g.get("fields_out", []))
            fsz = (ctypes.c_int * max(1, len(fs)))(*[int(f.shape[1]) for f in fs])
            fpt = (ctypes.c_void_p * max(1, len(fs)))(*[_p(f) for f in fs])
            opt = (ctypes.c_void_p * max(1, len(fo)))(*[_p(f) for f in fo])
            keep += [fsz, fpt, opt, arrays]
            tet = g["tet8"] if g.get("tet8") is not None else g["tetv"]
            met = g.get("met")
            v = lambda a: None if a is None else _p(a).value  # noqa: E731
            G[i] = HipGroup(int(g["xyz"].shape[0]), int(tet.shape[0]), int(g["triv"].shape[0]), v(g["xyz"]),
                            v(g.get("tet8")), v(g.get("tetv")), v(g.get("adja")), v(g["triv"]), v(g.get("adjt")),
                            float(g["hausd"]), 0 if met is None else int(met.shape[1]), v(met), len(fs),
                            ctypes.cast(fsz, ctypes.c_void_p), ctypes.cast(fpt, ctypes.c_void_p),
                            int(g["xyz_new"].shape[0]), v(g["xyz_new"]), v(g["pclass"]), v(g.get("met_out")),
                            ctypes.cast(opt, ctypes.c_void_p), v(g.get("elem_out")), v(g.get("hit_out")))
        self._grp_keep = (G, keep)
        st = HipStats()
        self._ck(self.lib.pmmg_hip_locate_interp_groups(self.h, len(groups), ctypes.cast(G, ctypes.c_void_p),
                                                        ctypes.byref(st) if sync else None), "locate_interp_groups")
        return st if sync else None

    def keep(self, slot: int = 0) -> None:
        """pmmg_hip_keep: the last host-mode call's new points and written rows
        stay on the device in `slot` (the next iteration's background)."""
        self._ck(self.lib.pmmg_hip_keep(self.h, int(slot)), "keep")

    def carry_over(self, slot: int, npt: int, src=None) -> None:
        """pmmg_hip_carry_over: the next host-mode set_background /
        set_solutions take vertex i+1 from kept point src[i] (1-based, 0: from
        the host arrays; None: the identity)."""
        s = None if src is None else np.ascontiguousarray(src, np.int32)
        self._ck(self.lib.pmmg_hip_carry_over(self.h, int(slot), int(npt), _p(s)), "carry_over")

    def release_scratch(self) -> None:
        """pmmg_hip_release_scratch: free the snapshot buckets, the binning's
        scratch and the group lanes (re-allocated on demand)."""
        self._ck(self.lib.pmmg_hip_release_scratch(self.h), "release_scratch")

    def bytes_up(self, reset: bool = False) -> int:
        """host -> device bytes of host-mode calls (pmmg_hip_bytes_up)"""
        return int(self.lib.pmmg_hip_bytes_up(self.h, int(reset)))

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

    def compute_wgt_mesh(self, xyz, tetv, xt, ftag, met, tag, qual):
        """PMMG_computeWgt_mesh on the device (pmmg_hip_compute_wgt_mesh):
        device arrays; qual is updated in place for tetra with an xtetra."""
        if not all(_is_dev(a) for a in (xyz, tetv, xt, ftag, qual)) or (met is not None and not _is_dev(met)):
            raise ValueError("compute_wgt_mesh takes device arrays")
        self._ck(self.lib.pmmg_hip_compute_wgt_mesh(self.h, xyz.shape[0], _p(xyz), tetv.shape[0], _p(tetv), _p(xt),
                                                    _p(ftag), 0 if met is None else int(met.shape[1]), _p(met),
                                                    int(tag), _p(qual)), "compute_wgt_mesh")
        return qual

    def compute_wgt_faces(self, xyz, tetv, face, met, wgt=None):
        """PMMG_computeWgt of a (tetra, face) list (pmmg_hip_compute_wgt_faces)."""
        if not all(_is_dev(a) for a in (xyz, tetv, face)) or (met is not None and not _is_dev(met)):
            raise ValueError("compute_wgt_faces takes device arrays")
        nf = face.shape[0]
        wgt = wgt if wgt is not None else self.empty((nf,), np.float64)
        self._ck(self.lib.pmmg_hip_compute_wgt_faces(self.h, xyz.shape[0], _p(xyz), _p(tetv), nf, _p(face),
                                                     0 if met is None else int(met.shape[1]), _p(met), _p(wgt)),
                 "compute_wgt_faces")
        return wgt

    # ------------------------------------------------------------------ split over GPUs (RCCL)
    @staticmethod
    def comm_unique_id() -> bytes:
        """pmmg_hip_comm_unique_id: the RCCL id one rank makes and broadcasts."""
        buf = ctypes.create_string_buffer(128)
        if not hip_lib().pmmg_hip_comm_unique_id(buf):
            raise RuntimeError("pmmg_hip_comm_unique_id failed (RCCL unavailable?)")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes) -> None:
        """pmmg_hip_comm_init (collective over the nranks processes)."""
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        self._ck(self.lib.pmmg_hip_comm_init(self.h, int(nranks), int(rank), buf), "comm_init")

    def allgather_points(self, counts, rows, rows_all, elem=None, elem_all=None, hit=None, hit_all=None) -> None:
        """pmmg_hip_allgather_points: this rank's rows (device arrays / tensors,
        one per slot) and optional elem / hit gathered in rank order into
        rows_all / elem_all / hit_all on every rank."""
        cnt = np.ascontiguousarray(counts, np.int64)
        rows, rows_all = list(rows), list(rows_all)
        sizes = (ctypes.c_int * max(1, len(rows)))(*[int(r.shape[1]) for r in rows])
        rin = (ctypes.c_void_p * max(1, len(rows)))(*[_p(r) for r in rows])
        rout = (ctypes.c_void_p * max(1, len(rows_all)))(*[_p(r) for r in rows_all])
        self._ck(self.lib.pmmg_hip_allgather_points(self.h, _p(cnt), len(rows), sizes, rin, rout, _p(elem),
                                                    _p(elem_all), _p(hit), _p(hit_all)), "allgather_points")

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
                ("xyz", ctypes.c_void_p), ("tag", ctypes.c_void_p), ("tetv", ctypes.c_void_p),
                ("adja", ctypes.c_void_p), ("triv", ctypes.c_void_p), ("adjt", ctypes.c_void_p),
                ("hausd", ctypes.c_double), ("met_size", ctypes.c_int), ("met", ctypes.c_void_p),
                ("nfield", ctypes.c_int), ("field_size", ctypes.c_void_p), ("field", ctypes.c_void_p)]


class NewGroup(ctypes.Structure):
    _fields_ = [("np", ctypes.c_int), ("ne", ctypes.c_int), ("xyz", ctypes.c_void_p), ("tag", ctypes.c_void_p),
                ("tetv", ctypes.c_void_p), ("met_size", ctypes.c_int), ("met", ctypes.c_void_p),
                ("field", ctypes.c_void_p), ("elem", ctypes.c_void_p), ("hit", ctypes.c_void_p),
                ("hsiz", ctypes.c_double), ("hmin", ctypes.c_double), ("hmax", ctypes.c_double),
                ("ani", ctypes.c_int)]


TAG_REQ, TAG_BDY, TAG_NUL = 1 << 2, 1 << 4, 1 << 14


class _Groups:
    """ctypes views of old/new group dicts (keeps every array alive).

    old: {mesh, met, fields, hausd[, tag, device_adjacency, device_boundary]}
    new: {xyz, tag, tetv, met, fields[, elem, hit, hsiz, hmin, hmax, ani]}"""

    def __init__(self, old_groups, new_groups):
        ng = len(old_groups)
        self.olds = (OldGroup * ng)()
        self.news = (NewGroup * ng)()
        self.keep = []
        for i, (o, g) in enumerate(zip(old_groups, new_groups)):
            m = o["mesh"]
            fs = list(o.get("fields", []))
            fsz = (ctypes.c_int * max(1, len(fs)))(*[f.shape[1] for f in fs])
            fpt = (ctypes.c_void_p * max(1, len(fs)))(*[_p(f) for f in fs])
            met = o.get("met")
            dev_bdy = o.get("device_boundary", False)
            self.olds[i] = OldGroup(m.np, m.ne, -1 if dev_bdy else m.nt, _p(m.xyz), _p(o.get("tag")), _p(m.tetv),
                                    None if o.get("device_adjacency", False) else _p(m.adja),
                                    None if dev_bdy else _p(m.triv), None if dev_bdy else _p(m.adjt),
                                    float(o.get("hausd", 0.01)), 0 if met is None else met.shape[1], _p(met),
                                    len(fs), ctypes.cast(fsz, ctypes.c_void_p), ctypes.cast(fpt, ctypes.c_void_p))
            gf = list(g.get("fields", []))
            gpt = (ctypes.c_void_p * max(1, len(gf)))(*[_p(f) for f in gf])
            gm = g.get("met")
            self.news[i] = NewGroup(g["xyz"].shape[0], g["tetv"].shape[0], _p(g["xyz"]), _p(g.get("tag")),
                                    _p(g["tetv"]), 0 if gm is None else gm.shape[1], _p(gm),
                                    ctypes.cast(gpt, ctypes.c_void_p), _p(g.get("elem")), _p(g.get("hit")),
                                    float(g.get("hsiz", 0.0)), float(g.get("hmin", 0.0)), float(g.get("hmax", 0.0)),
                                    int(g.get("ani", 0)))
            self.keep += [fsz, fpt, gpt]


def interp_metrics_and_fields(ctx: TransferContext, old_groups, new_groups, input_met: int = 1, carry=None):
    """PMMG_interpMetricsAndFields over groups (src/interpmesh_pmmg.c:663-741)
    through the C host layer (pmmg_interp_metrics_and_fields).  The new
    groups' ``met`` / ``fields`` arrays are filled in place; per-group
    ``hsiz`` > 0 replaces the metric by a constant (MMG3D_Set_constantSize).
    carry: None (plain call), or (carried, src) for
    pmmg_interp_metrics_and_fields_carry — the new groups stay on the device,
    and with carried the old groups are the previous call's new groups (src:
    None, or per group None / the 1-based map of its vertices onto them).
    Returns (ier, stats)."""
    G = _Groups(old_groups, new_groups)
    st = HipStats()
    if carry is None:
        ier = host_lib().pmmg_interp_metrics_and_fields(ctx.h, len(old_groups), ctypes.cast(G.olds, ctypes.c_void_p),
                                                        ctypes.cast(G.news, ctypes.c_void_p), int(input_met),
                                                        ctypes.byref(st))
        return ier, st
    carried, src = carry
    maps = None
    if src is not None:
        arrs = [None if m is None else np.ascontiguousarray(m, np.int32) for m in src]
        maps = (ctypes.c_void_p * max(1, len(arrs)))(*[None if a is None else _p(a).value for a in arrs])
        G.keep.append(arrs)
    ier = host_lib().pmmg_interp_metrics_and_fields_carry(ctx.h, len(old_groups), ctypes.cast(G.olds, ctypes.c_void_p),
                                                          ctypes.cast(G.news, ctypes.c_void_p), int(input_met),
                                                          int(bool(carried)),
                                                          None if maps is None else ctypes.cast(maps, ctypes.c_void_p),
                                                          ctypes.byref(st))
    return ier, st


def copy_metrics_and_fields_point(old_group, new_group, perm_nod_glob=None, renum: int = 1, input_met: int = 1):
    """PMMG_copyMetricsAndFields_point (src/interpmesh_pmmg.c:432-446) through
    the C host layer: rows of the old group's valid MG_REQ points copied into
    the new group's arrays (through perm_nod_glob, 1-based with entry 0
    unused, when renum and a permutation are given).  Returns 1/0."""
    G = _Groups([old_group], [new_group])
    perm = None if perm_nod_glob is None else np.ascontiguousarray(perm_nod_glob, np.int32)
    return host_lib().pmmg_copy_metrics_and_fields_point(ctypes.cast(G.olds, ctypes.c_void_p),
                                                         ctypes.cast(G.news, ctypes.c_void_p), _p(perm),
                                                         int(renum), int(input_met))


def classify_points(new_group) -> np.ndarray:
    """The reference's point classification (src/interpmesh_pmmg.c:535-550)
    through the C host layer: PT_SKIP / PT_VOL / PT_BDY per new point."""
    g = dict(new_group)
    g.setdefault("fields", [])
    G = _Groups([dict(mesh=_EmptyMesh(), fields=[])], [g])
    pc = np.empty(g["xyz"].shape[0], np.uint8)
    host_lib().pmmg_classify_points(ctypes.cast(G.news, ctypes.c_void_p), _p(pc))
    return pc


def set_constant_metric(new_group) -> int:
    """MMG3D_Set_constantSize's fill through the C host layer (restated, unpinned)."""
    G = _Groups([dict(mesh=_EmptyMesh(), fields=[])], [new_group])
    return host_lib().pmmg_set_constant_metric(ctypes.cast(G.news, ctypes.c_void_p))


class _EmptyMesh:
    np = ne = nt = 0
    xyz = tetv = adja = triv = adjt = None
