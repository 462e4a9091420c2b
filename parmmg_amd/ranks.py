"""One process per GPU: rank setup and the two reductions the bench needs.

ParMmg runs the transfer step per group on every MPI rank with no exchange
(src/interpmesh_pmmg.c:690-730; interface points are MG_REQ and copied), so
the data path has no collective.  The only cross-rank traffic is the bench's
own barrier and the max-over-ranks of the step time, done here through
torch.distributed ("nccl" = RCCL on the GPU box, "gloo" in the CPU tests).
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
