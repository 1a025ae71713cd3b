"""Multi-GPU sharding of one large commitment (BASELINE.json configs[4]).

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).
The points of Σ c_i [tau^i]G1 are split into contiguous ranges; every rank
generates its own SRS slice [tau^(start+i)]G1 on its GPU and computes the
partial MSM of its range.  EC addition is not an RCCL reduction operator, so
the one exchange step is an all-gather of the N partial points (a few hundred
bytes over xGMI) followed by an exact fold on every rank.  The fold's affine
result is order-independent, so every rank holds the bit-exact commitment.
Since round 6 the device path exchanges projective partials (one XYZZ point,
kzgx_partial_record_words int64 words): no rank inverts its partial, and the
fold's single inversion is the step's only one.

The partial-MSM and fold callables are injected so the same driver runs
with the GPU (kzgx.Context) in bench.py and with the CPU oracle in the
gloo tests (tests/test_dist_gloo.py).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, start + count) of n items for rank; remainders go to the first ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def pack_point(xy: np.ndarray, inf: bool, w64: int) -> np.ndarray:
    out = np.zeros(2 * w64 + 1, dtype=np.int64)
    out[: 2 * w64] = np.asarray(xy, dtype=np.uint64).view(np.int64)[: 2 * w64]
    out[-1] = 1 if inf else 0
    return out


def unpack_points(buf: np.ndarray, w64: int):
    buf = np.asarray(buf, dtype=np.int64).reshape(-1, 2 * w64 + 1)
    return buf[:, : 2 * w64].view(np.uint64), buf[:, -1].astype(bool)


def sharded_commit(n: int, world: int, rank: int, w64: int,
                   partial_msm: Callable[[int, int], Tuple[np.ndarray, bool]],
                   all_gather: Callable[[np.ndarray], np.ndarray],
                   fold: Callable[[np.ndarray, np.ndarray], Tuple[np.ndarray, bool]],
                   ) -> Tuple[np.ndarray, bool]:
    """partial_msm(start, count) -> (xy, inf) of this rank's slice;
    all_gather(packed) -> (world, 2 W64 + 1) array of every rank's packed point;
    fold(points, infs) -> (xy, inf) sum of the gathered points."""
    start, count = shard_range(n, world, rank)
    if count:
        xy, inf = partial_msm(start, count)
    else:
        xy, inf = np.zeros(2 * w64, dtype=np.uint64), True
    if world == 1:  # the fold of a single partial is the partial itself
        return xy, inf
    gathered = all_gather(pack_point(xy, inf, w64))
    pts, infs = unpack_points(gathered, w64)
    return fold(pts, infs)


def sharded_commit_tensor(n: int, world: int, rank: int, w64: int,
                          partial_msm: Callable[[int, int], "object"],
                          fold: Callable[["object"], "object"],
                          dist, torch, on_phase: Optional[Callable[[str], None]] = None) -> "object":
    """Device-resident form of sharded_commit (bench.py's configs[4] step).

    partial_msm(start, count) -> this rank's partial record (a 1-D int64
    tensor on the compute device: on the GPU one projective XYZZ point,
    kzgx_msm_g1_partial_device), enqueued with no host synchronisation; the
    records are all-gathered (RCCL over xGMI on GPU, gloo on CPU) straight
    into one (world, record) tensor, and fold(records) -> the packed affine
    sum (x || y || infinity word; kzgx_g1_sum_partials_device on the GPU).
    The fold runs at every world size -- at world 1 it is the partial's
    affine conversion.  Nothing crosses to the host inside a step, and
    nothing is repacked between the phases.  on_phase(name), if given, is
    called after each phase is enqueued ("partial", "gather", "fold"), e.g.
    to record timing events on the step's stream."""
    mark = on_phase or (lambda _name: None)
    start, count = shard_range(n, world, rank)
    packed = partial_msm(start, count)
    mark("partial")
    if world == 1:  # nothing to gather: the fold is the partial's conversion
        mark("gather")
        res = fold(packed.reshape(1, -1))
        mark("fold")
        return res
    g = torch.empty((world, packed.shape[0]), dtype=packed.dtype, device=packed.device)
    backend = dist.get_backend() if hasattr(dist, "get_backend") else None
    if backend == "nccl" and hasattr(dist, "all_gather_into_tensor"):
        dist.all_gather_into_tensor(g, packed)  # RCCL: straight into the (world, W) tensor
    else:  # gloo (the one-box rehearsal, CPU tests): list form into the rows of g
        outs = list(g.unbind(0))
        dist.all_gather(outs, packed)
    mark("gather")
    res = fold(g)
    mark("fold")
    return res


def torch_all_gather(dist, device: Optional[object] = None):
    """all_gather callable over torch.distributed (RCCL on GPU, gloo on CPU)."""
    import torch

    def gather(packed: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(packed))
        if device is not None:
            t = t.to(device)
        outs = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(outs, t)
        return torch.stack(outs).cpu().numpy()

    return gather
