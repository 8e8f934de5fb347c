"""World-size-2 (gloo, CPU) coverage of the multi-GPU path: contiguous
chunk-aligned shards compressed independently, reassembled in file order on
rank 0 via all_gather(sizes) + send/recv; must equal the single-process body.
The per-shard compressor here is the CPU oracle (test infrastructure); on the
GPU box the same reassembly runs over RCCL with the HIP compressor."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, chunk, seed, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "adaptive-compression_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ambc.distributed import compress_sharded, shard_range
    from oracle import oracle as orc

    data = torch.frombuffer(bytearray(orc.synth(n, seed)), dtype=torch.uint8)

    def fn(shard):
        body, st = orc.compress_body(bytes(shard.numpy()),
                                     orc.make_params(chunk, "native", (1, 3, 4, 9),
                                                     n_total=shard.numel()))
        return torch.frombuffer(bytearray(body[:-16]), dtype=torch.uint8), st

    s, e = shard_range(n, chunk, world, rank)
    assert s % chunk == 0
    out = compress_sharded(data, chunk, fn)
    if rank == 0:
        q.put(bytes(out.numpy()))
    # in place: every rank's packages are the file-order body's bytes at its offset
    from ambc.distributed import file_offsets
    mine, _ = fn(data[s:e])
    off, total = file_offsets(mine.numel(), torch.device("cpu"))
    ref, _ = orc.compress_body(bytes(data.numpy()), orc.make_params(chunk, "native", (1, 3, 4, 9),
                                                                    n_total=n))
    assert total + 16 == len(ref)
    assert ref[off:off + mine.numel()] == bytes(mine.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,chunk", [(2, 1 << 20, 4096), (2, 300001, 1024), (3, 77777, 4096),
                                           (4, 4096 * 5 + 7, 4096)])
def test_sharded_reassembly_equals_single_process(world, n, chunk):
    from oracle import oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, chunk, 42, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = orc.synth(n, 42)
    ref, _ = orc.compress_body(data, orc.make_params(chunk, "native", (1, 3, 4, 9), n_total=n))
    assert got == ref


def test_shard_ranges_cover_input():
    from ambc.distributed import shard_range
    for n, chunk, world in ((10 ** 6, 4096, 8), (4096, 4096, 8), (1, 16, 3), (4 << 30, 8192, 8)):
        prev = 0
        for r in range(world):
            s, e = shard_range(n, chunk, world, r)
            assert s == prev and (s % chunk == 0 or s == n)
            prev = e
        assert prev == n


# ---------------------------------------------------------------------------
# sharded decode: split at package boundaries, per-rank decode, file-order gather
# ---------------------------------------------------------------------------
def _dec_worker(rank, world, port, body, orig, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "adaptive-compression_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ambc.distributed import decompress_sharded
    from oracle import oracle as orc

    def fn(sub, n):
        out, produced = orc.decompress_body(bytes(sub), n, return_produced=True)
        return torch.frombuffer(bytearray(out), dtype=torch.uint8) if out else \
            torch.empty(0, dtype=torch.uint8), produced

    out = decompress_sharded(body, orig, fn)
    if rank == 0:
        q.put(bytes(out.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _run_dec(world, body, orig):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dec_worker, args=(r, world, port, body, orig, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world,n,chunk", [(2, 1 << 20, 4096), (3, 300001, 1024), (4, 9000, 4096)])
def test_sharded_decode_equals_single_process(world, n, chunk):
    from oracle import oracle as orc
    data = orc.synth(n, 7)
    body, _ = orc.compress_body(data, orc.make_params(chunk, "native", (1, 3, 4, 9), n_total=n))
    assert _run_dec(world, body, n) == data


def test_sharded_decode_lenient_bodies_fall_back():
    """Packages that decode to other lengths than announced (unregistered id,
    short Delta) and a truncated final package: the split cannot be trusted, the
    destination decodes alone -- the result still equals the sequential decode."""
    import struct
    from oracle import oracle as orc
    pk = []
    huff = orc.huff_encode(b"aaab" * 8)   # 32 symbols; announced orig 60 -> decodes short
    for t, payload, orig in ((3, huff, 60), (255, b"a" * 100, 100), (4, b"\x05" * 30, 60),
                             (77, b"xyz" * 10, 50), (255, b"b" * 200, 200), (1, b"\x07\x05", 5),
                             (255, b"c" * 90, 90)):
        pk.append(b"\xff\xff\x00\x00" + bytes([t, 0]) + struct.pack("<III", len(payload), orig,
                                                                     len(payload)) + payload)
    body = b"".join(pk) + b"\xff\xff\x00\x00" + bytes(12)
    orig = 505
    ref = orc.decompress_body(body, orig)
    assert orc.decompress_body(pk[0], 60, return_produced=True)[1] == 32   # the short package
    assert _run_dec(2, body, orig) == ref


def test_split_body_ranges():
    from ambc.distributed import split_body
    from oracle import oracle as orc
    n, chunk = 100000, 4096
    data = orc.synth(n, 3)
    body, _ = orc.compress_body(data, orc.make_params(chunk, "native", (1, 3, 4, 9), n_total=n))
    for parts in (1, 2, 5, 8, 40):
        sp = split_body(body, n, parts)
        assert sp[0][0] == 0 and sp[0][2] == 0 and sp[-1][1] == len(body) and sp[-1][3] == n
        for (b0, b1, o0, o1), (c0, _, p0, _) in zip(sp, sp[1:]):
            assert b1 == c0 and o1 == p0 and b0 <= b1 and o0 <= o1
        for b0, b1, o0, o1 in sp:
            if b1 > b0:
                assert body[b0:b0 + 4] == b"\xff\xff\x00\x00"
                assert orc.decompress_body(body[b0:b1], o1 - o0) == data[o0:o1]
    with pytest.raises(ValueError):
        split_body(b"\x00" * 40, 10, 2)
