"""Multi-GPU sharding of the compress path (one process per GPU).

Native-mode chunks are independent, so a node shards the input into
contiguous, chunk-aligned ranges: rank r compresses chunks
[M*r/W, M*(r+1)/W) on its own GPU with no data-path collective, producing its
packages without the end chunk.  ``file_offsets`` (an all_gather of the 8-byte
body sizes) places every rank's packages in the file-order body; the one bulk
exchange, only when one rank must hold the whole body, is ``reassemble``:

  1. all_gather of the per-rank body sizes (8 bytes each) -> file offsets;
  2. point-to-point gather of every rank's body straight into its offset of
     the destination rank's buffer (RCCL send/recv over xGMI; the destination
     receives (W-1)/W of the body, which is per-link bound, so every peer
     streams over its own link concurrently);
  3. the destination appends the 16-byte end chunk.
  4. all_reduce(SUM) of the per-rank chunk statistics.

Decode (``decompress_sharded``) shards the other way round: every rank holds
the body, cuts it at package boundaries into W ranges of about orig_size / W
decoded bytes (``ambc_split_body``: the reference's header walk with each
package's expected length), walks and decodes only its own range on its GPU,
and the decoded ranges are gathered in file order (same variable-size P2P
gather).  A body whose packages decode to other lengths than their headers
announce (the reference's lenient paths) cannot be cut in advance: the ranks
detect it and the destination decodes the whole body itself.

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


def file_offsets(nbytes, device, group=None):
    """The body's layout across ranks: all_gather of the per-rank body sizes
    (8 bytes each) -> (this rank's byte offset in the file-order body, total).
    With it every rank's packages are addressable in place (a parallel writer
    puts rank r's bytes at its offset); only ``reassemble`` moves them."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    size = torch.tensor([int(nbytes)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    sizes = [int(x.item()) for x in sizes]
    return sum(sizes[:rank]), sum(sizes)


def gather_concat(t, dst=0, group=None, out=None, extra=0):
    """Concatenate every rank's uint8 tensor in rank order on ``dst`` (sizes by
    all_gather, payloads by point-to-point send/recv).  Returns (tensor, total)
    on dst -- the tensor has ``extra`` spare bytes after the data -- and
    (None, total) elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = t.device
    size = torch.tensor([t.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    sizes = [int(s.item()) for s in sizes]
    offs = [0]
    for s in sizes:
        offs.append(offs[-1] + s)
    total = offs[-1]
    if rank == dst:
        if out is None or out.numel() < total + extra:
            out = torch.empty(total + extra, dtype=torch.uint8, device=dev)
        mine = out[offs[rank]:offs[rank] + sizes[rank]]
        if sizes[rank] and mine.data_ptr() != t.data_ptr():
            mine.copy_(t)
        ops = [dist.P2POp(dist.irecv, out[offs[r]:offs[r] + sizes[r]], r, group)
               for r in range(world) if r != dst and sizes[r]]
    else:
        ops = [dist.P2POp(dist.isend, t, dst, group)] if sizes[rank] else []
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return (out, total) if rank == dst else (None, total)


def reassemble(body, dst=0, group=None, out=None):
    """Gather every rank's body (uint8 tensor, no end chunk) into file order on
    rank ``dst``.  Returns the full body tensor (with end chunk) on dst, None
    elsewhere.  ``out`` may pre-hold dst's own body at offset 0 when dst == 0."""
    import torch
    out, total = gather_concat(body, dst=dst, group=group, out=out, extra=len(END_CHUNK))
    if out is None:
        return None
    out[total:total + len(END_CHUNK)] = torch.tensor(list(END_CHUNK), dtype=torch.uint8,
                                                     device=out.device)
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


def _registered_array(registered):
    reg = (C.c_uint64 * 4)()
    for t in registered:
        reg[t >> 6] |= 1 << (t & 63)
    return reg


def split_body(body, orig_size, nparts, registered=(1, 2, 3, 4, 5, 6, 7, 9, 255), lib=None):
    """[(body_start, body_end, out_start, out_end)] * nparts: the body cut at
    package boundaries into ranges of about orig_size / nparts decoded bytes
    (ambc_split_body, host code).  Raises ValueError on a marker mismatch, as
    the reference's decode does."""
    import numpy as np
    lib = lib or _lib.load()
    bo = (C.c_uint64 * (nparts + 1))()
    oo = (C.c_uint64 * (nparts + 1))()
    arr = np.frombuffer(body, dtype=np.uint8)
    rc = lib.ambc_split_body(arr.ctypes.data if len(arr) else None, len(arr), orig_size,
                             _registered_array(registered), nparts, bo, oo)
    if rc == _lib.AMBC_E_MARKER:
        raise ValueError("Marker mismatch in chunk header.")
    _lib.check(rc, lib)
    return [(bo[r], bo[r + 1], oo[r], oo[r + 1]) for r in range(nparts)]


def hip_decode_fn(ctx=None, dev=0, registered=(1, 2, 3, 4, 5, 6, 7, 9, 255)):
    """decode_fn running libambc_hip: (body bytes, orig) -> (device uint8 tensor
    of orig bytes, bytes the packages produced before the final pad/truncate)."""
    import numpy as np
    import torch

    ctx = ctx or _lib.default_context()
    reg = _registered_array(registered)

    def fn(body, orig):
        arr = np.frombuffer(body, dtype=np.uint8)
        out = torch.empty(max(orig, 1), dtype=torch.uint8,
                          device=torch.device("cuda", ctx.devices[dev]))
        st = _lib.Stats()
        torch.cuda.synchronize(out.device)
        rc = ctx.lib.ambc_decompress_device(ctx.h, dev, arr.ctypes.data if len(arr) else None,
                                            len(arr), orig, reg, out.data_ptr(), C.byref(st))
        if rc == _lib.AMBC_E_MARKER:
            raise ValueError("Marker mismatch in chunk header.")
        _lib.check(rc, ctx.lib)
        return out[:orig], int(st.payload_bytes)
    return fn


def decompress_sharded(body, orig_size, decode_fn, dst=0, group=None,
                       registered=(1, 2, 3, 4, 5, 6, 7, 9, 255), split=None, device=None):
    """Decode an .ambc body (bytes, held by every rank) across the process group.
    ``decode_fn(sub_body, orig)`` returns (uint8 tensor of orig bytes, bytes the
    packages produced before the final pad/truncate).  Returns the decoded
    tensor (orig_size bytes) on dst, None elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = split or split_body(body, orig_size, world, registered)
    nonempty = [r for r in range(world) if parts[r][1] > parts[r][0]]
    last = nonempty[-1] if nonempty else world - 1
    b0, b1, o0, o1 = parts[rank]
    mv = memoryview(body)
    if b1 > b0:
        out, produced = decode_fn(mv[b0:b1], o1 - o0)
    else:
        out, produced = None, 0
    # a range before the last must decode to exactly the bytes its headers announce
    ok = rank >= last or produced == o1 - o0
    if device is None:
        device = (torch.device("cuda", torch.cuda.current_device())
                  if dist.get_backend(group) == "nccl" else torch.device("cpu"))
    dev = out.device if out is not None else torch.device(device)
    if out is None:
        out = torch.empty(0, dtype=torch.uint8, device=dev)
    flags = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(world)]
    dist.all_gather(flags, torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev),
                    group=group)
    if all(int(f.item()) for f in flags):
        res, _ = gather_concat(out, dst=dst, group=group)
        return res[:orig_size] if res is not None else None
    # lenient package lengths: the destination decodes the whole body
    if rank != dst:
        return None
    res, _ = decode_fn(mv, orig_size)
    return res
