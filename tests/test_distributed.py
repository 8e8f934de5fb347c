"""World-size 2-4 CPU coverage of the multi-GPU path's host side, torch-free:

* ``ambc.comm.HostGroup`` -- the TCP rendezvous that carries the RCCL unique id
  and the bench's control messages -- in real separate processes;
* the shard layout of ``ambc_shard_range`` (library host code): every rank
  compresses its contiguous chunk-aligned shard independently (the CPU oracle
  stands in for the GPU here), the sizes are all-gathered into file offsets,
  and the concatenation in rank order equals the single-process body;
* ``ambc_split_body`` (library host code): each rank decodes its package range
  and the ranges concatenate to the input.

On the GPU box the same layout runs inside libambc_hip over RCCL
(tests/test_gpu_distributed.py).
"""
import multiprocessing as mp
import os
import socket
import struct

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _paths():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "adaptive-compression_amd")]


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def _group_worker(rank, world, port, q):
    _paths()
    from ambc.comm import HostGroup
    g = HostGroup(rank, world, "127.0.0.1", port, timeout=60)
    parts = g.allgather(bytes([rank]) * (rank + 1))
    assert parts == [bytes([r]) * (r + 1) for r in range(world)]
    uid = g.broadcast(os.urandom(128) if rank == 0 else b"")
    assert len(uid) == 128
    ids = g.allgather(uid)
    assert all(x == uid for x in ids)
    t = g.allgather_obj([rank * 1.5, 7])
    assert [x[0] for x in t] == [r * 1.5 for r in range(world)]
    g.barrier()
    if rank == 0:
        q.put("ok")
    g.close()


@pytest.mark.parametrize("world", [2, 4])
def test_host_group_rendezvous(world):
    assert _run(_group_worker, world) == "ok"


def _compress_worker(rank, world, port, q, n, chunk, seed):
    _paths()
    from ambc.comm import HostGroup
    from ambc.distributed import shard_range
    from oracle import oracle as orc
    g = HostGroup(rank, world, "127.0.0.1", port, timeout=60)
    data = orc.synth(n, seed)
    s, e = shard_range(n, chunk, world, rank)
    assert s % chunk == 0
    body, _ = orc.compress_body(data[s:e], orc.make_params(chunk, "native", (1, 3, 4, 9), n_total=e - s))
    mine = body if rank == world - 1 else body[:-16]     # only the last rank ends the body
    sizes = [struct.unpack("<Q", x)[0] for x in g.allgather(struct.pack("<Q", len(mine)))]
    off = sum(sizes[:rank])
    ref, _ = orc.compress_body(data, orc.make_params(chunk, "native", (1, 3, 4, 9), n_total=n))
    assert sum(sizes) == len(ref)
    assert ref[off:off + len(mine)] == mine          # in place at its file offset
    parts = g.allgather(mine)
    if rank == 0:
        q.put(b"".join(parts))
    g.close()


@pytest.mark.parametrize("world,n,chunk", [(2, 1 << 20, 4096), (2, 300001, 1024), (3, 77777, 4096),
                                           (4, 4096 * 5 + 7, 4096)])
def test_sharded_layout_equals_single_process(world, n, chunk):
    from oracle import oracle as orc
    got = _run(_compress_worker, world, n, chunk, 42)
    data = orc.synth(n, 42)
    ref, _ = orc.compress_body(data, orc.make_params(chunk, "native", (1, 3, 4, 9), n_total=n))
    assert got == ref


def test_shard_ranges_cover_input():
    from ambc.distributed import shard_range
    for n, chunk, world in ((10 ** 6, 4096, 8), (4096, 4096, 8), (1, 16, 3), (4 << 30, 8192, 8),
                            (32 << 30, 8192, 8)):
        prev = 0
        M = (n + chunk - 1) // chunk
        for r in range(world):
            s, e = shard_range(n, chunk, world, r)
            assert s == prev and (s % chunk == 0 or s == n)
            assert s == min(M * r // world * chunk, n)
            prev = e
        assert prev == n


def _dec_worker(rank, world, port, q, body, orig):
    _paths()
    from ambc.comm import HostGroup
    from ambc.distributed import split_body
    from oracle import oracle as orc
    g = HostGroup(rank, world, "127.0.0.1", port, timeout=60)
    b0, b1, o0, o1 = split_body(body, orig, world)[rank]
    out = orc.decompress_body(body[b0:b1], o1 - o0) if b1 > b0 else b""
    parts = g.allgather(out)
    if rank == 0:
        q.put(b"".join(parts))
    g.close()


@pytest.mark.parametrize("world,n,chunk", [(2, 1 << 20, 4096), (3, 300001, 1024), (4, 9000, 4096)])
def test_sharded_decode_equals_single_process(world, n, chunk):
    from oracle import oracle as orc
    data = orc.synth(n, 7)
    body, _ = orc.compress_body(data, orc.make_params(chunk, "native", (1, 3, 4, 9), n_total=n))
    assert _run(_dec_worker, world, body, n) == data


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


def test_bench_rejects_mismatched_world(tmp_path):
    """bench.py --gpus 2 under a launcher that started one rank must fail fast,
    before any GPU call (a silent 1-GPU measurement is the bug this guards)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
