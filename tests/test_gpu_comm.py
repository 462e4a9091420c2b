"""The C-ABI collective of the split (include/parmmg_hip.h,
pmmg_hip_comm_* / pmmg_hip_allgather_points: RCCL all-gather of {element,
hit code, K doubles} per point).

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), and the
one-GPU box has one, so this is the world-1 rehearsal: a communicator made
from a unique id, the records packed, all-gathered and unpacked into the
caller's arrays.  The N > 1 path runs in bench.py --gpus N (checked there
against torch.distributed's all-gather of the same arrays)."""
import numpy as np
import pytest

from parmmg_amd.transfer import TransferContext


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 1000, 100003])
def test_allgather_points_world1(n):
    rng = np.random.default_rng(n)
    sizes = [6, 1, 3, 6]
    rows = [rng.standard_normal((n, s)) for s in sizes]
    elem = rng.integers(1, 1 << 29, n).astype(np.int32)
    hit = rng.integers(1, 12, n).astype(np.int8)
    with TransferContext(0) as ctx:
        ctx.comm_init(1, 0, ctx.comm_unique_id())
        d_rows = [ctx.upload(r) for r in rows] if n else [ctx.empty((0, s), np.float64) for s in sizes]
        d_all = [ctx.empty((n, s), np.float64) for s in sizes]
        d_e, d_h = ctx.upload(elem), ctx.upload(hit)
        d_ea, d_ha = ctx.empty((n,), np.int32), ctx.empty((n,), np.int8)
        ctx.allgather_points([n], d_rows, d_all, d_e, d_ea, d_h, d_ha)
        if n:
            for a, b in zip(d_all, rows):
                assert np.array_equal(a.download(), b)
            assert np.array_equal(d_ea.download(), elem)
            assert np.array_equal(d_ha.download(), hit)
        # without elem / hit
        ctx.allgather_points([n], d_rows[:2], d_all[:2])
        with pytest.raises(RuntimeError, match="invalid"):
            ctx.allgather_points([n], d_rows, d_all, d_e, None)  # elem without elem_all
        # a rank's invalid arguments are found before the data collective (the
        # ranks' agreement): the call fails on every rank, and the
        # communicator stays usable
        with pytest.raises(RuntimeError, match="counts"):
            ctx.allgather_points([-1], d_rows, d_all)
        ctx.allgather_points([n], d_rows[:1], d_all[:1])
        if n:
            assert np.array_equal(d_all[0].download(), rows[0])


@pytest.mark.gpu
def test_allgather_needs_a_communicator():
    with TransferContext(0) as ctx:
        a = ctx.empty((4, 1), np.float64)
        with pytest.raises(RuntimeError, match="no communicator"):
            ctx.allgather_points([4], [a], [a])
