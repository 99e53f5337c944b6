"""Frame sharding and the histogram exchange for multi-GPU runs (one process per GPU).

The block-codec hot path has no data-path collective: intra frames are independent and,
in the open-loop sequence benchmark, so are frame pairs (f-1, f).  The one exchange is the
input of the global Huffman table: every rank histograms its own symbols
on its GPU and the ranks all-gather the int64 histograms, then sum them in rank order
(integer, hence identical on every rank and independent of arrival order).
torch.distributed is the transport (backend "nccl" = RCCL over xGMI on MI355X; "gloo" in
the CPU tests).
"""
from __future__ import annotations


def shard_range(n: int, rank: int, world: int) -> tuple:
    """Contiguous [start, stop) share of n items for `rank` (sizes differ by at most 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank must be in [0, world)")
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def shard_pairs(nframes: int, rank: int, world: int) -> tuple:
    """Frames a rank needs for its share of the nframes-1 consecutive pairs (f-1, f) of a
    sequence: returns (first_frame, stop_frame) including the one-frame halo, so the rank
    runs inter coding on frames[first:stop] and produces pairs first+1 .. stop-1."""
    s, e = shard_range(max(nframes - 1, 0), rank, world)
    if s == e:
        return s, s
    return s, e + 1


def _host_staged(t, group=None):
    """gloo (CPU rehearsals, tests) has no device-tensor collectives: stage through host."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend(group) == "gloo"


def init_single_rank(device, port=None):
    """A one-rank process group on `device` (backend "nccl" = RCCL): the collectives below then
    run through RCCL even without a second GPU (`force=True`), so the exchange's RCCL path is
    exercised on a one-GPU box.  Rendezvous on 127.0.0.1."""
    import socket

    import torch
    import torch.distributed as dist
    if port is None:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=torch.device(device))
    return dist


def _collective(group, force):
    import torch.distributed as dist
    return dist.is_initialized() and (force or dist.get_world_size(group) > 1)


def global_bounds(local_mm, group=None, force=False):
    """(min, max) over every rank of the int32 pairs local_mm = [min, max] (device tensor,
    ivc_minmax_i32's output) with one all-reduce (MAX of [-min, max] in int64).  With one
    rank the all-reduce is skipped unless `force`."""
    import torch
    import torch.distributed as dist
    v = torch.stack([-local_mm[0].to(torch.int64), local_mm[1].to(torch.int64)])
    if _collective(group, force):
        if _host_staged(v, group):
            v = v.cpu()
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=group)
    lo, hi = v.tolist()
    return -lo, hi


def global_histogram(local_hist, group=None, force=False):
    """Sum of every rank's histogram (a 1-D int64 tensor on this rank's device) via one
    all-gather; every rank receives the same result.  With one rank the all-gather is
    skipped (a copy is returned) unless `force`."""
    import torch
    import torch.distributed as dist
    if not _collective(group, force):
        return local_hist.clone()
    world = dist.get_world_size(group)
    if _host_staged(local_hist, group):
        return global_histogram(local_hist.cpu(), group, force).to(local_hist.device)
    gathered = torch.empty((world,) + tuple(local_hist.shape), dtype=local_hist.dtype,
                           device=local_hist.device)
    try:
        dist.all_gather_into_tensor(gathered, local_hist.contiguous(), group=group)
    except (RuntimeError, NotImplementedError):
        # backends without the fused form (older gloo): same exchange as a list all-gather
        parts = [torch.empty_like(local_hist) for _ in range(world)]
        dist.all_gather(parts, local_hist.contiguous(), group=group)
        gathered = torch.stack(parts)
    total = gathered[0].clone()
    for k in range(1, world):           # rank order: deterministic integer sum
        total += gathered[k]
    return total
