"""One process per GPU: rank setup, the bench's reductions and the result
all-gather of the split modes.

ParMmg runs the transfer step per group on every MPI rank with no exchange
(src/interpmesh_pmmg.c:690-730; interface points are MG_REQ and copied), so
the step itself has no collective.  Across ranks there is the bench's
barrier, the max-over-ranks of the step time and, when one group is split
over the GPUs (RCB parts or Morton ranges of its new points, bench.py
--shard halo / morton), one all-gather per output array after the step
(``allgather_rows``: every rank receives every part's located elements and
interpolated rows), all through torch.distributed ("nccl" = RCCL over xGMI
on the GPU box, "gloo" in the CPU tests).
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class RankInfo:
    rank: int
    world: int
    local: int
    backend: str | None  # None: single process, no process group

    @property
    def distributed(self) -> bool:
        return self.backend is not None


def from_env() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl") -> RankInfo:
    """Join the process group torchrun set up (no-op for WORLD_SIZE=1).
    With "nccl" the rank binds its node-local GPU first."""
    rank, world, local = from_env()
    if world <= 1:
        return RankInfo(rank, world, local, None)
    import torch
    import torch.distributed as dist

    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend)
    return RankInfo(rank, world, local, backend)


def barrier(ri: RankInfo) -> None:
    if ri.distributed:
        import torch.distributed as dist

        dist.barrier()


def _reduce(ri: RankInfo, value: float, op_name: str) -> float:
    if not ri.distributed:
        return float(value)
    import torch
    import torch.distributed as dist

    dev = f"cuda:{ri.local}" if ri.backend == "nccl" else "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=getattr(dist.ReduceOp, op_name))
    return float(t.item())


def broadcast_object(ri: RankInfo, objs: list, src: int = 0) -> None:
    """objs (a list) replaced in place by rank src's (e.g. the RCCL unique id
    of pmmg_hip_comm_init, as a shim would MPI_Bcast it)."""
    if ri.distributed:
        import torch.distributed as dist

        dist.broadcast_object_list(objs, src=src)


def max_over_ranks(ri: RankInfo, value: float) -> float:
    return _reduce(ri, value, "MAX")


def sum_over_ranks(ri: RankInfo, value: float) -> float:
    return _reduce(ri, value, "SUM")


def finalize(ri: RankInfo) -> None:
    if ri.distributed:
        import torch.distributed as dist

        dist.destroy_process_group()


def aggregate(ri: RankInfo, points_this_rank: int, elapsed_s: float, steps: int) -> dict:
    """Whole-job throughput of a weak-scaled run: points of all ranks per
    step divided by the slowest rank's step time."""
    t = max_over_ranks(ri, elapsed_s)
    pts = sum_over_ranks(ri, points_this_rank)
    return {"elapsed_s": t, "points_per_step": int(pts), "ms_per_step": t / steps * 1e3,
            "mpts_per_s": pts / (t / steps) / 1e6}


# ---------------------------------------------------------------- Morton-range sharding
#
# one transfer problem split over the GPUs of a node, each
# GPU owning a contiguous Morton range of the new points (balanced by count)
# against a replicated background; the located elements and interpolated rows
# are then collected with an all-gather (RCCL over xGMI on the GPU box, gloo
# in the CPU tests).  This is the strong-scaling alternative to the
# one-group-per-rank default above.

def _expand10(v):
    import numpy as np

    v = v.astype(np.uint32) & np.uint32(0x3FF)
    v = (v | (v << np.uint32(16))) & np.uint32(0x030000FF)
    v = (v | (v << np.uint32(8))) & np.uint32(0x0300F00F)
    v = (v | (v << np.uint32(4))) & np.uint32(0x030C30C3)
    v = (v | (v << np.uint32(2))) & np.uint32(0x09249249)
    return v


def morton_codes(xyz):
    """30-bit Morton codes of points (10 bits per axis over their bbox)."""
    import numpy as np

    lo, hi = xyz.min(axis=0), xyz.max(axis=0)
    ext = np.where(hi > lo, hi - lo, 1.0)
    q = np.clip(((xyz - lo) / ext * 1024.0).astype(np.int64), 0, 1023)
    return (_expand10(q[:, 0]) << np.uint32(2)) | (_expand10(q[:, 1]) << np.uint32(1)) | _expand10(q[:, 2])


# device cost of a surface point relative to a volume point (cfg4 on one
# MI355X: k_bdy 0.56 ms for 0.60M surface points, k_vol 3.9 ms for 19.7M
# volume points); balances the ranks' step times, not their point counts
BDY_WEIGHT = 4


def morton_shards(xyz, pclass, world: int, bdy_weight: int = BDY_WEIGHT):
    """0-based point indices of each rank: the processed points (pclass != 0)
    in Morton order (stable), cut into `world` contiguous ranges of equal
    cost (a surface point, pclass 2, counts bdy_weight volume points; with
    bdy_weight 1 the sizes differ by at most one); inside its range a rank
    keeps the input order of the points (a mesh numbering is spatially
    coherent, a Morton order is not at the scale of a wave: neighbouring
    lanes would walk from unrelated seeds).  Skipped points (MG_REQ, copied
    by the host) are in no shard."""
    import numpy as np

    idx = np.nonzero(pclass != 0)[0]
    order = idx[np.argsort(morton_codes(xyz[idx]), kind="stable")]
    if bdy_weight == 1 or len(order) == 0:
        cuts = [len(order) * r // world for r in range(world + 1)]
    else:
        cost = np.cumsum(np.where(pclass[order] == 2, bdy_weight, 1).astype(np.int64))
        total = int(cost[-1])
        cuts = [0] + [int(np.searchsorted(cost, total * r // world, side="right")) for r in range(1, world)] + \
            [len(order)]
    return [np.sort(order[cuts[r]:cuts[r + 1]]) for r in range(world)]


def rcb_shards(xyz, pclass, world: int, bdy_weight: int = BDY_WEIGHT):
    """0-based point indices of each rank by recursive coordinate bisection:
    the processed points (pclass != 0) are cut at the cost-weighted quantile
    (world_left / world of the cost, a surface point counting bdy_weight
    volume points) across the longest side of their box, recursively, so
    that every rank gets a compact box of equal cost.  A contiguous Morton
    range of a shell can cover two pieces far apart (its box up to 4x the
    volume its points fill); the halo shard around it and the seed grid over
    that box are then sparse.  Inside its part a rank keeps the input order
    of the points.  Skipped points are in no shard."""
    import numpy as np

    idx = np.nonzero(pclass != 0)[0]
    w = np.where(pclass[idx] == 2, bdy_weight, 1).astype(np.int64)
    out = [None] * world

    def cut(sel, wsel, r0, n):
        if n == 1 or len(sel) == 0:
            for r in range(r0, r0 + n):
                out[r] = np.sort(sel) if r == r0 else np.zeros(0, sel.dtype)
            return
        p = xyz[sel]
        d = int(np.argmax(p.max(axis=0) - p.min(axis=0)))
        o = np.argsort(p[:, d])  # introsort: deterministic, the same split on every rank
        cw = np.cumsum(wsel[o])
        nl = n // 2
        k = int(np.searchsorted(cw, cw[-1] * nl // n, side="right"))
        cut(sel[o[:k]], wsel[o[:k]], r0, nl)
        cut(sel[o[k:]], wsel[o[k:]], r0 + nl, n - nl)

    cut(idx, w, 0, world)
    return out


def allgather_rows(ri: RankInfo, rows, counts):
    """All-gather of per-rank row blocks (torch tensors [n_r, C], same dtype
    and C on every rank; counts[r] = n_r): padded to the largest block, one
    all_gather_into_tensor, trimmed; returns the blocks concatenated in rank
    order.  Single process: the rows themselves."""
    if not ri.distributed:
        return rows
    import torch
    import torch.distributed as dist

    m = max(counts)
    pad = torch.zeros((m,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=rows.device)
    pad[: rows.shape[0]] = rows
    out = torch.empty((ri.world * m,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=rows.device)
    dist.all_gather_into_tensor(out, pad)
    return torch.cat([out[r * m: r * m + counts[r]] for r in range(ri.world)])
