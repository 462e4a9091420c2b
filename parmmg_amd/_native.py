"""ctypes bindings of the native libraries.

The product path is ``libpmmg_hip.so`` (include/parmmg_hip.h) and the C host
layer ``libpmmg_host.so``.  Loading fails loudly when a library is missing:
there is no Python or CPU fallback for the transfer step.
"""
from __future__ import annotations

import ctypes
import os

from . import build as _build

c_int, c_int64, c_double, c_void_p, c_char_p = ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p, ctypes.c_char_p
P = ctypes.POINTER


ABI_VERSION = 6  # PMMG_HIP_ABI_VERSION of include/parmmg_hip.h


class HipStats(ctypes.Structure):
    """``pmmg_hip_stats`` of include/parmmg_hip.h."""

    _fields_ = [
        ("nvol", c_int64), ("nbdy", c_int64),
        ("nvol_walk", c_int64), ("nvol_exhaust", c_int64), ("nvol_closest", c_int64), ("nvol_exact", c_int64),
        ("nbdy_face", c_int64), ("nbdy_edge", c_int64), ("nbdy_vertex", c_int64), ("nbdy_wedge", c_int64),
        ("nbdy_cone", c_int64), ("nbdy_exhaust", c_int64), ("nbdy_stale", c_int64), ("nbdy_closest", c_int64),
        ("steps_total", c_int64), ("stepmax", c_int64), ("wave_iters", c_int64), ("sorted", c_int64),
        ("ms_prepare", ctypes.c_float), ("ms_sort", ctypes.c_float), ("ms_vol", ctypes.c_float),
        ("ms_bdy", ctypes.c_float), ("ms_fallback", ctypes.c_float), ("ms_total", ctypes.c_float),
        ("ms_vol_locate", ctypes.c_float),
        ("nvol_noseed", c_int64), ("nvol_stuck", c_int64), ("nvol_limit", c_int64), ("seed_map_axes", c_int64),
        ("nbdy_fanscan", c_int64), ("reserved", c_int64 * 6),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_ if name != "reserved"}


class HipGroup(ctypes.Structure):
    """``pmmg_hip_group`` of include/parmmg_hip.h (device pointers)."""

    _fields_ = [
        ("np", c_int), ("ne", c_int), ("nt", c_int), ("xyz", c_void_p), ("tet8", c_void_p), ("tetv", c_void_p),
        ("adja", c_void_p), ("triv", c_void_p), ("adjt", c_void_p), ("hausd", c_double),
        ("met_size", c_int), ("met", c_void_p), ("nfield", c_int), ("field_size", c_void_p), ("fields", c_void_p),
        ("np_new", c_int), ("xyz_new", c_void_p), ("pclass", c_void_p), ("met_out", c_void_p),
        ("fields_out", c_void_p), ("elem_out", c_void_p), ("hit_out", c_void_p),
    ]


# C-ABI of include/parmmg_hip.h: name -> (restype, argtypes)
HIP_API = {
    "pmmg_hip_abi_version": (c_int, []),
    "pmmg_hip_stats_size": (c_int64, []),
    "pmmg_hip_create": (c_void_p, [c_int, c_int]),
    "pmmg_hip_destroy": (None, [c_void_p]),
    "pmmg_hip_set_background": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                        c_void_p, c_double, c_int]),
    "pmmg_hip_set_background_tet8": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                             c_double, c_int]),
    "pmmg_hip_set_solutions": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int]),
    "pmmg_hip_locate_interp": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, P(HipStats), c_int]),
    "pmmg_hip_sync": (c_int, [c_void_p, P(HipStats)]),
    "pmmg_hip_locate_interp_groups": (c_int, [c_void_p, c_int, c_void_p, P(HipStats)]),
    "pmmg_hip_keep": (c_int, [c_void_p, c_int]),
    "pmmg_hip_carry_over": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "pmmg_hip_bytes_up": (c_int64, [c_void_p, c_int]),
    "pmmg_hip_release_scratch": (c_int, [c_void_p]),
    "pmmg_hip_malloc": (c_void_p, [c_void_p, c_int64]),
    "pmmg_hip_free": (c_int, [c_void_p, c_void_p]),
    "pmmg_hip_build_adjacency": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "pmmg_hip_build_boundary": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                        c_void_p, c_void_p, c_void_p]),
    "pmmg_hip_set_solutions_packed": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int]),
    "pmmg_hip_compute_wgt_mesh": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                          c_void_p, c_int, c_void_p]),
    "pmmg_hip_compute_wgt_faces": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                           c_void_p]),
    "pmmg_hip_tetra_qual": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                    P(c_double)]),
    "pmmg_hip_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "pmmg_hip_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "pmmg_hip_locate_interp_rec": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_int]),
    "pmmg_hip_comm_unique_id": (c_int, [c_void_p]),
    "pmmg_hip_comm_init": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "pmmg_hip_comm_attach": (c_int, [c_void_p, c_void_p, c_int, c_int]),
    "pmmg_hip_allgather_points": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p]),
    "pmmg_hip_last_error": (c_char_p, [c_void_p]),
    "pmmg_hip_device_count": (c_int, []),
}

SYNTH_API = {
    "synth_counts": (c_int, [c_int, c_int, P(c_int64)]),
    "synth_vertices": (c_int, [c_int, c_int, c_double, ctypes.c_uint64, c_void_p, c_void_p]),
    "synth_vertices_valid": (c_int, [c_int, c_int, c_double, ctypes.c_uint64, c_void_p, c_void_p]),
    "synth_tetra": (c_int, [c_int, c_int, c_void_p, c_void_p]),
    "synth_trias": (c_int64, [c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "synth_field": (c_int, [c_int, c_int64, c_void_p, c_void_p]),
    "synth_field_size": (c_int, [c_int]),
    "synth_visit_order": (c_int64, [c_int, c_void_p, c_int, c_void_p]),
    "synth_classes": (c_int, [c_int64, c_void_p, c_int, c_void_p]),
}

_cache: dict[str, ctypes.CDLL] = {}


def _load(path: str, api: dict, what: str) -> ctypes.CDLL:
    if path in _cache:
        return _cache[path]
    if not os.path.exists(path):
        raise RuntimeError(f"{what} is not built ({path}); run `python -m parmmg_amd.build` "
                           "(there is no fallback path)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in api.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _cache[path] = lib
    return lib


def hip_lib() -> ctypes.CDLL:
    """The product HIP module (include/parmmg_hip.h)."""
    # PMMG_HIP_SO: an alternative build of the same module (A/B measurements)
    lib = _load(os.environ.get("PMMG_HIP_SO", _build.HIP_SO), HIP_API, "libpmmg_hip.so")
    # the load-time ABI check a shim makes (include/parmmg_hip.h, PMMG_HIP_ABI_VERSION)
    if lib.pmmg_hip_abi_version() != ABI_VERSION or lib.pmmg_hip_stats_size() != ctypes.sizeof(HipStats):
        raise RuntimeError(f"libpmmg_hip.so ABI {lib.pmmg_hip_abi_version()} / stats {lib.pmmg_hip_stats_size()} B, "
                           f"expected {ABI_VERSION} / {ctypes.sizeof(HipStats)} B: rebuild (python -m parmmg_amd.build)")
    return lib


def synth_lib() -> ctypes.CDLL:
    return _load(_build.SYNTH_SO, SYNTH_API, "libpmmg_synth.so")


HOST_API = {
    "pmmg_classify_points": (c_int64, [c_void_p, c_void_p]),
    "pmmg_copy_metrics_and_fields_point": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int]),
    "pmmg_set_constant_metric": (c_int, [c_void_p]),
    "pmmg_interp_metrics_and_fields": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, P(HipStats)]),
    "pmmg_interp_metrics_and_fields_carry": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                                     P(HipStats)]),
    "pmmg_max_tet_extent": (c_double, [c_int, c_void_p, c_int, c_void_p]),
    "pmmg_shard_mark": (c_int, [c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_double, c_void_p,
                                c_void_p, P(c_int64)]),
    "pmmg_shard_mark_cells": (c_int, [c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_double,
                                      c_void_p, c_void_p, c_double, c_void_p, c_void_p, P(c_int64)]),
    "pmmg_shard_fill": (c_int64, [c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p]),
    "pmmg_shard_mark_trias": (c_int64, [c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "pmmg_shard_fill_region": (c_int64, [c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmmg_shard_part_pack": (c_int64, [c_void_p, c_void_p, c_void_p, c_int64]),
    "pmmg_shard_assemble": (c_int, [c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmmg_medit_read_mesh": (c_int, [ctypes.c_char_p, c_void_p, ctypes.c_char_p, c_int]),
    "pmmg_medit_read_sol": (c_int, [ctypes.c_char_p, c_void_p, ctypes.c_char_p, c_int]),
    "pmmg_medit_free_mesh": (None, [c_void_p]),
    "pmmg_medit_free_sol": (None, [c_void_p]),
}


def host_lib() -> ctypes.CDLL:
    hip_lib()  # resolve the dependency from the same directory first
    return _load(_build.HOST_SO, HOST_API, "libpmmg_host.so")
