"""Multi-GPU sharding of the compress and decompress paths,
torch-free: every exchange runs inside libambc_hip over RCCL.

Native-mode chunks are independent, so a node shards the input into
contiguous, chunk-aligned ranges: rank r of W compresses chunks
[M*r/W, M*(r+1)/W) (``shard_range``) on its own GPU.  ``compress_shard`` is
``ambc_compress_shard``:

  1. the shard's packages, with no collective on the data path (the last rank
     appends the 16-byte end chunk);
  2. AllGather of the per-rank body sizes -> every rank's file-order offset;
  3. AllReduce(SUM) of the chunk statistics (the stats dict);
  4. reference mode: AllReduce(MIN) of the first chunk without a winner -- the
     reference's remainder-raw rule (adaptive_compressor.py:586-588) is global,
     so the rank holding that chunk writes ONE raw chunk header for the rest of
     the file and every later rank contributes its shard's bytes verbatim;
  5. ``root=0``: grouped ncclSend/ncclRecv of every body straight into its
     offset on rank 0 (each peer streams over its own xGMI link); ``root=-1``
     leaves the packages in place for a parallel writer.

``decompress_shard`` (``ambc_decompress_shard``) shards the other way round:
every rank holds the body, ``ambc_split_body`` cuts it at package boundaries
into W ranges of about orig_size / W decoded bytes, each rank decodes its range
into HBM, and the ranges gather on rank 0 in file order.  A body whose packages
decode to other lengths than their headers announce (the reference's lenient
paths) is detected by all ranks (AllReduce MIN of a flag) and decoded whole by
rank 0 -- the result is always the sequential decode.

Process groups come from ``ambc.comm.GpuGroup`` (one process per GPU, RCCL
unique id over a TCP rendezvous).  In one process, a ``Context`` over several
devices runs the same shards on one host thread per device through
``ambc_compress_batch`` / ``ambc_decompress_multi``.
"""
import ctypes as C

from . import _lib
from .container import MARKER_BYTES

END_CHUNK = MARKER_BYTES + b"\x00" * 12
DEFAULT_REGISTERED = (1, 2, 3, 4, 5, 6, 7, 9, 255)


def shard_range(n_total, chunk, world, rank, lib=None):
    """Byte range [start, end) of rank's contiguous chunk-aligned shard
    (ambc_shard_range, host code)."""
    lib = lib or _lib.load()
    b, e = C.c_uint64(), C.c_uint64()
    _lib.check(lib.ambc_shard_range(n_total, chunk, world, rank, C.byref(b), C.byref(e)), lib)
    return b.value, e.value


def registered_array(registered=DEFAULT_REGISTERED):
    reg = (C.c_uint64 * 4)()
    for t in registered:
        reg[t >> 6] |= 1 << (t & 63)
    return reg


def compress_shard(group, d_shard, n_total, params, d_out, out_cap, root=-1):
    """This rank's shard (device pointer / DeviceBuffer holding input bytes
    ``shard_range(...)``) of an n_total-byte input -> (ShardInfo, Stats).
    ``group`` is a GpuGroup (or a one-device Context: one rank)."""
    ctx = getattr(group, "ctx", group)
    info, st = _lib.ShardInfo(), _lib.Stats()
    with ctx.lock:
        rc = ctx.lib.ambc_compress_shard(ctx.h, int(d_shard), n_total, C.byref(params), int(d_out), out_cap,
                                         root, C.byref(info), C.byref(st))
    if rc == _lib.AMBC_E_RANGE:
        import struct
        raise struct.error("argument out of range")
    _lib.check(rc, ctx.lib)
    return info, st


def gather(group, d_src, nbytes, d_dst=None, dst_cap=0):
    """Every rank's nbytes at d_src into file order in rank 0's d_dst ->
    (this rank's offset, total)."""
    ctx = getattr(group, "ctx", group)
    off, tot = C.c_uint64(), C.c_uint64()
    with ctx.lock:
        _lib.check(ctx.lib.ambc_comm_gather(ctx.h, int(d_src), nbytes, int(d_dst) if d_dst else None, dst_cap,
                                            C.byref(off), C.byref(tot)), ctx.lib)
    return off.value, tot.value


def split_body(body, orig_size, nparts, registered=DEFAULT_REGISTERED, lib=None):
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
                             registered_array(registered), nparts, bo, oo)
    if rc == _lib.AMBC_E_MARKER:
        raise ValueError("Marker mismatch in chunk header.")
    _lib.check(rc, lib)
    return [(bo[r], bo[r + 1], oo[r], oo[r + 1]) for r in range(nparts)]


def decompress_shard(group, body, orig_size, d_out, out_cap, root=0, registered=DEFAULT_REGISTERED):
    """Decode an .ambc body (bytes, held by every rank) across the group into
    device memory -> (ShardInfo, Stats).  root 0: rank 0's d_out receives all
    orig_size bytes."""
    import numpy as np
    ctx = getattr(group, "ctx", group)
    arr = np.frombuffer(body, dtype=np.uint8)
    info, st = _lib.ShardInfo(), _lib.Stats()
    with ctx.lock:
        rc = ctx.lib.ambc_decompress_shard(ctx.h, arr.ctypes.data if len(arr) else None, len(arr), orig_size,
                                           registered_array(registered), int(d_out), out_cap, root,
                                           C.byref(info), C.byref(st))
    if rc == _lib.AMBC_E_MARKER:
        raise ValueError("Marker mismatch in chunk header.")
    _lib.check(rc, ctx.lib)
    return info, st


def decompress_multi(ctx, body, orig_size, registered=DEFAULT_REGISTERED):
    """In-process decode over every device of ctx (one host thread each)."""
    import numpy as np
    arr = np.frombuffer(body, dtype=np.uint8)
    out = bytearray(max(orig_size, 1))
    st = _lib.Stats()
    with ctx.lock:
        rc = ctx.lib.ambc_decompress_multi(ctx.h, arr.ctypes.data if len(arr) else None, len(arr), orig_size,
                                           registered_array(registered), _lib.addr(out), C.byref(st))
    if rc == _lib.AMBC_E_MARKER:
        raise ValueError("Marker mismatch in chunk header.")
    _lib.check(rc, ctx.lib)
    return bytes(out[:orig_size])
