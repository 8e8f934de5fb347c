"""Multi-GPU sharding of the compress path (one process per GPU).

Native-mode chunks are independent, so a node shards the input into
contiguous, chunk-aligned ranges: rank r compresses chunks
[M*r/W, M*(r+1)/W) on its own GPU with no data-path collective, producing its
packages without the end chunk.  The one real exchange is the reassembly of
the .ambc body in file order:

  1. all_gather of the per-rank body sizes (8 bytes each) -> file offsets;
  2. point-to-point gather of every rank's body straight into its offset of
     the destination rank's buffer (RCCL send/recv over xGMI; the destination
     receives (W-1)/W of the body, which is per-link bound, so every peer
     streams over its own link concurrently);
  3. the destination appends the 16-byte end chunk.
  4. all_reduce(SUM) of the per-rank chunk statistics.

torch.distributed is plumbing here (backend "nccl" is RCCL on ROCm; "gloo" is
used by the CPU tests).  ``compress_fn`` maps a shard (uint8 tensor) to its
body tensor; the default runs the HIP kernels through libambc_hip.
"""
import ctypes as C

from . import _lib
from .container import MARKER_BYTES

END_CHUNK = MARKER_BYTES + b"\x00" * 12


def shard_range(n_total, chunk, world, rank):
    """Byte range [start, end) of rank's contiguous chunk-aligned shard."""
    M = (n_total + chunk - 1) // chunk
    k0, k1 = M * rank // world, M * (rank + 1) // world
    return min(k0 * chunk, n_total), min(k1 * chunk, n_total)


def hip_compress_fn(params, ctx=None, dev=0):
    """compress_fn running libambc_hip on device-resident torch tensors."""
    import torch

    ctx = ctx or _lib.default_context()

    def fn(shard):
        n = shard.numel()
        p = _lib.Params()
        C.memmove(C.addressof(p), C.addressof(params), C.sizeof(_lib.Params))
        p.flags |= _lib.FLAG_NO_END_CHUNK
        cap = ctx.lib.ambc_compress_bound(n, p.chunk_size)
        out = torch.empty(cap, dtype=torch.uint8, device=shard.device)
        olen = C.c_uint64()
        st = _lib.Stats()
        torch.cuda.synchronize(shard.device)
        _lib.check(ctx.lib.ambc_compress_device(ctx.h, dev, shard.data_ptr(), n, C.byref(p),
                                                out.data_ptr(), cap, C.byref(olen), C.byref(st),
                                                None), ctx.lib)
        return out[:olen.value], st
    return fn


def reassemble(body, dst=0, group=None, out=None):
    """Gather every rank's body (uint8 tensor, no end chunk) into file order on
    rank ``dst``.  Returns the full body tensor (with end chunk) on dst, None
    elsewhere.  ``out`` may pre-hold dst's own body at offset 0 when dst == 0."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = body.device
    size = torch.tensor([body.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    sizes = [int(s.item()) for s in sizes]
    offs = [0]
    for s in sizes:
        offs.append(offs[-1] + s)
    total = offs[-1]
    if rank == dst:
        if out is None or out.numel() < total + len(END_CHUNK):
            out = torch.empty(total + len(END_CHUNK), dtype=torch.uint8, device=dev)
        if out[offs[rank]:offs[rank] + sizes[rank]].data_ptr() != body.data_ptr():
            out[offs[rank]:offs[rank] + sizes[rank]].copy_(body)
        ops = [dist.P2POp(dist.irecv, out[offs[r]:offs[r] + sizes[r]], r, group)
               for r in range(world) if r != dst and sizes[r]]
    else:
        ops = [dist.P2POp(dist.isend, body, dst, group)] if sizes[rank] else []
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != dst:
        return None
    out[total:total + len(END_CHUNK)] = torch.tensor(list(END_CHUNK), dtype=torch.uint8,
                                                     device=dev)
    return out[:total + len(END_CHUNK)]


def reduce_stats(stats_vec, group=None):
    """all_reduce(SUM) of a per-rank stats vector (tensor)."""
    import torch.distributed as dist
    dist.all_reduce(stats_vec, op=dist.ReduceOp.SUM, group=group)
    return stats_vec


def compress_sharded(data, chunk, compress_fn, dst=0, group=None):
    """Compress ``data`` (a uint8 tensor holding the WHOLE input on every rank,
    or this rank's shard when ``data`` is a (tensor, n_total) pair) across the
    process group; returns the reassembled body on dst."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if isinstance(data, tuple):
        shard, _ = data
    else:
        s, e = shard_range(data.numel(), chunk, world, rank)
        shard = data[s:e]
    body, _ = compress_fn(shard)
    return reassemble(body, dst=dst, group=group)
