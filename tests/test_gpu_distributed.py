"""GPU coverage of the multi-GPU path, through the C-ABI only:

* compress: a ctx listing GPU 0 several times runs that many shards on one host
  thread each (ambc_compress_batch -> the sharded path of ambc_shard.cpp: the
  same size AllGather / stats AllReduce / reference-mode AllReduce(MIN) code as
  RCCL, over host memory because RCCL admits one rank per device); the body
  must equal the single-device body and the CPU oracle's, in native mode at
  chunks 4096 / 8192 (C4's eligibility) and in reference mode with the
  remainder-raw chunk starting in every shard;
* RCCL itself: a one-rank communicator (ncclCommInitRank) under
  ambc_compress_shard / ambc_decompress_shard / ambc_comm_gather;
* decode: the body split at package boundaries (ambc_split_body), every range
  decoded into device memory, and the in-process multi-shard decode incl. the
  whole-body fallback for lenient package lengths;
* two processes on two GPUs over RCCL, when the box has them.
"""
import ctypes as C
import os
import socket
import struct
import subprocess
import sys

import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _body(n, chunk, methods, seed, mode="native"):
    data = orc.synth(n, seed)
    # id 5 in native mode: the GPU's "ambc-deflate v1" (reference mode: zlib-9's bytes)
    body, _ = orc.compress_body(data, orc.make_params(chunk, mode, methods, n_total=n,
                                                      deflate="gd" if mode == "native" else "zlib"))
    return data, body


def _ctx(devs):
    from ambc import _lib
    return _lib.Context(devs)


def _compress(ctx, data, chunk, methods, mode="native"):
    from ambc import AdaptiveCompressor
    from ambc import _lib
    comp = AdaptiveCompressor(chunk_size=chunk, mode=mode, methods=methods)
    p, keep = comp._params(len(data))
    cap = ctx.lib.ambc_compress_bound(len(data), chunk)
    out = bytearray(cap)
    olen = C.c_uint64()
    st = _lib.Stats()
    rc = ctx.lib.ambc_compress_batch(ctx.h, _lib.addr(data), len(data), C.byref(p), _lib.addr(out), cap,
                                     C.byref(olen), C.byref(st))
    _lib.check(rc, ctx.lib)
    del keep
    return bytes(out[:olen.value]), st


@pytest.mark.parametrize("shards,n,chunk,methods", [
    (2, (1 << 22) + 123, 4096, (1, 3, 4, 9)),
    (3, (1 << 21) + 4096 * 3, 8192, (1, 3, 4, 9)),     # C4's chunk: Huffman + LZ4 eligible
    (4, 1 << 21, 4096, (1, 2, 3, 4)),                  # the byte-pinned set, Dictionary on the GPU
    (8, 3 << 20, 8192, (1, 3, 4, 9)),
    (5, 4096 * 5 + 17, 4096, (1, 3, 4, 9)),            # one chunk per shard, ragged tail
])
def test_sharded_compress_equals_single_device(hip_lib, shards, n, chunk, methods):
    data, ref = _body(n, chunk, methods + (255,), 31)
    one = _ctx([0])
    single, st1 = _compress(one, data, chunk, methods)
    multi = _ctx([0] * shards)
    got, st = _compress(multi, data, chunk, methods)
    assert single == ref
    assert got == ref
    assert st.total_chunks == st1.total_chunks and st.compressed_chunks == st1.compressed_chunks
    assert list(st.method_usage) == list(st1.method_usage)
    assert st.payload_bytes == st1.payload_bytes and st.bytes_saved == st1.bytes_saved
    multi.close()
    one.close()


def _ref_mode_input(chunk, nchunks, raw_at):
    """zero chunks (RLE wins) with one random chunk (nothing beats raw) at raw_at."""
    parts = []
    for k in range(nchunks):
        parts.append(orc.random_bytes(chunk, 1000 + k) if k == raw_at else bytes([k % 7]) * chunk)
    return b"".join(parts) + b"\x03" * 100      # ragged tail


@pytest.mark.parametrize("shards,raw_at", [(3, 1), (3, 9), (3, 17), (3, None), (4, 0), (2, 23)])
def test_sharded_reference_mode_remainder(hip_lib, shards, raw_at):
    """The reference's remainder-raw rule across shards: AllReduce(MIN) of the
    first no-winner chunk; its rank writes one raw header for the rest of the
    file, later ranks contribute their bytes verbatim."""
    chunk, nchunks = 1024, 24
    data = _ref_mode_input(chunk, nchunks, raw_at if raw_at is not None else -1)
    ref, _ = orc.compress_body(data, orc.make_params(chunk, "reference", (1, 3, 4, 255), n_total=len(data)))
    multi = _ctx([0] * shards)
    got, st = _compress(multi, data, chunk, (1, 3, 4), mode="reference")
    assert got == ref
    expect_total = (raw_at + 1) if raw_at is not None else nchunks + 1
    assert st.total_chunks == expect_total
    assert st.raw_chunks == (1 if raw_at is not None else 0)
    multi.close()


@pytest.mark.parametrize("shards,n,chunk,methods,slab", [
    (3, (5 << 20) + 333, 4096, (1, 3, 4, 9), 1 << 20),      # 6 slabs over 3 devices, ragged tail
    (2, (3 << 20) + 8192 * 5, 8192, (1, 3, 4, 9), 1 << 19),  # C4's chunk
    (4, (1 << 20) + 77, 4096, (1, 3, 4, 5), 300000),         # a slab that is not a chunk multiple, id 5
    (3, 700000, 1024, (1, 2, 3, 4), 1 << 18),                # the last round leaves a device idle
])
def test_multi_device_slab_pipeline_equals_single_device(hip_lib, shards, n, chunk, methods, slab):
    """Host-fed native compress over several devices: chunk-aligned slabs dealt
    round-robin, H2D / compress / D2H overlapped per device, every slab's body
    written at the file offset of a per-round AllGather of sizes -- the body and
    stats equal the single-device call and the oracle."""
    data, ref = _body(n, chunk, methods + (255,), 57)
    one = _ctx([0])
    single, st1 = _compress(one, data, chunk, methods)
    os.environ["AMBC_SLAB_BYTES"] = str(slab)
    try:
        multi = _ctx([0] * shards)
        got, st = _compress(multi, data, chunk, methods)
    finally:
        del os.environ["AMBC_SLAB_BYTES"]
    assert (single == ref) is True and (got == ref) is True   # (no byte diff of megabytes on failure)
    assert st.total_chunks == st1.total_chunks and st.compressed_chunks == st1.compressed_chunks
    assert list(st.method_usage) == list(st1.method_usage)
    assert st.payload_bytes == st1.payload_bytes and st.bytes_saved == st1.bytes_saved
    # a buffer too small for the body: every device fails at the same round, none hangs
    from ambc import _lib
    os.environ["AMBC_SLAB_BYTES"] = str(slab)
    try:
        p, keep = __import__("ambc").AdaptiveCompressor(chunk_size=chunk, methods=methods)._params(n)
        small = bytearray(len(ref) // 2)
        olen = C.c_uint64()
        rc = multi.lib.ambc_compress_batch(multi.h, _lib.addr(data), n, C.byref(p), _lib.addr(small),
                                           len(small), C.byref(olen), None)
    finally:
        del os.environ["AMBC_SLAB_BYTES"]
    assert rc == _lib.AMBC_E_CAPACITY
    multi.close()
    one.close()


def test_sharded_compress_reports_capacity_consistently(hip_lib):
    """A too-small host buffer fails on every shard without hanging the others."""
    from ambc import AdaptiveCompressor
    from ambc import _lib
    data = orc.synth(1 << 20, 4)
    multi = _ctx([0, 0, 0])
    p, keep = AdaptiveCompressor(chunk_size=4096, methods=(1, 3, 4, 9))._params(len(data))
    out = bytearray(1000)
    olen = C.c_uint64()
    rc = multi.lib.ambc_compress_batch(multi.h, _lib.addr(data), len(data), C.byref(p), _lib.addr(out), 1000,
                                       C.byref(olen), None)
    assert rc == _lib.AMBC_E_CAPACITY
    multi.close()


# ---------------------------------------------------------------------------
# RCCL with one rank (the box has one GPU: RCCL refuses two ranks on a device)
# ---------------------------------------------------------------------------
@pytest.fixture
def rccl_group(hip_lib):
    from ambc.comm import GpuGroup, HostGroup
    g = GpuGroup(rank=0, world=1, local_rank=0, host=HostGroup(0, 1), rccl=True)
    yield g
    g.close()


def test_rccl_one_rank_compress_shard(rccl_group):
    from ambc import AdaptiveCompressor
    from ambc import _lib
    from ambc.distributed import compress_shard, decompress_shard, gather
    ctx = rccl_group.ctx
    nr, rk = C.c_int(), C.c_int()
    _lib.check(ctx.lib.ambc_comm_size(ctx.h, C.byref(nr), C.byref(rk)), ctx.lib)
    assert (nr.value, rk.value) == (1, 0)
    n, chunk = (3 << 20) + 999, 4096
    data, ref = _body(n, chunk, (1, 3, 4, 9, 255), 77)
    p, keep = AdaptiveCompressor(chunk_size=chunk, methods=(1, 3, 4, 9))._params(n)
    d_in = _lib.DeviceBuffer(ctx, n + 64)
    d_in.upload(data)
    cap = ctx.lib.ambc_compress_bound(n, chunk)
    d_out = _lib.DeviceBuffer(ctx, cap + 64)
    info, st = compress_shard(rccl_group, d_in, n, p, d_out, cap, root=0)
    assert (info.offset, info.local_len, info.total) == (0, len(ref), len(ref))
    assert bytes(d_out.download(info.total)) == ref
    # the RCCL gather of one rank is a copy into rank 0's buffer
    d_all = _lib.DeviceBuffer(ctx, cap + 64)
    off, tot = gather(rccl_group, d_out, info.total, d_all, cap + 64)
    assert (off, tot) == (0, len(ref))
    assert bytes(d_all.download(tot)) == ref
    # sharded decode back into device memory
    d_dec = _lib.DeviceBuffer(ctx, n + 64)
    dinfo, _ = decompress_shard(rccl_group, ref, n, d_dec, n + 64, root=0)
    assert dinfo.total == n
    assert bytes(d_dec.download(n)) == data
    # collectives of one rank
    v = (C.c_uint64 * 3)(5, 7, 9)
    _lib.check(ctx.lib.ambc_comm_allreduce_u64(ctx.h, v, 3, _lib.OP_MIN), ctx.lib)
    assert list(v) == [5, 7, 9]
    rccl_group.barrier()
    for b in (d_in, d_out, d_all, d_dec):
        b.free()


# ---------------------------------------------------------------------------
# decode: split ranges, device output, in-process shards
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n,chunk,methods,parts", [
    ((1 << 22) + 123, 4096, (1, 3, 4, 9), 8),
    (1 << 21, 1024, (1, 3, 4, 9), 3),
    ((1 << 21) + 77, 4096, (1, 3, 5), 8),        # C5 method set (zlib-9 DEFLATE chunks)
])
def test_split_ranges_decode_on_device(hip_lib, n, chunk, methods, parts):
    from ambc import _lib
    from ambc.distributed import registered_array, split_body
    data, body = _body(n, chunk, methods, 11)
    ctx = _ctx([0])
    got = bytearray()
    for b0, b1, o0, o1 in split_body(body, n, parts):
        if b1 == b0:
            continue
        d = _lib.DeviceBuffer(ctx, o1 - o0 + 64)
        st = _lib.Stats()
        sub = body[b0:b1]
        _lib.check(ctx.lib.ambc_decompress_device(ctx.h, 0, _lib.addr(sub), len(sub), o1 - o0,
                                                  registered_array(), d.ptr, C.byref(st)), ctx.lib)
        assert st.payload_bytes == o1 - o0
        got += d.download(o1 - o0)
        d.free()
    assert bytes(got) == data
    ctx.close()


def test_device_decode_rejects_host_codec_packages(hip_lib):
    """ids 6/7 (bz2 / lzma) are host codecs: the device-output call says so."""
    import bz2
    from ambc import _lib
    from ambc.distributed import registered_array
    payload = bz2.compress(b"q" * 500)
    body = b"\xff\xff\x00\x00" + bytes([6, 0]) + struct.pack("<III", 500, 500, len(payload)) + \
        payload + b"\xff\xff\x00\x00" + bytes(12)
    ctx = _ctx([0])
    d = _lib.DeviceBuffer(ctx, 600)
    rc = ctx.lib.ambc_decompress_device(ctx.h, 0, _lib.addr(body), len(body), 500, registered_array(),
                                        d.ptr, None)
    assert rc == _lib.AMBC_E_HOSTCODEC
    d.free()
    ctx.close()


@pytest.mark.parametrize("shards,n,chunk", [(2, (1 << 21) + 5, 4096), (3, 300001, 1024), (8, 9000, 4096)])
def test_decompress_multi_equals_input(hip_lib, shards, n, chunk):
    from ambc.distributed import decompress_multi
    data, body = _body(n, chunk, (1, 3, 4, 9, 255), 5)
    ctx = _ctx([0] * shards)
    assert decompress_multi(ctx, body, n) == data
    ctx.close()


def test_decompress_multi_lenient_body_falls_back(hip_lib):
    """Packages that decode to other lengths than announced (short Huffman,
    unregistered id, short Delta): the ranks agree on the whole-body fallback,
    and the result equals the sequential decode."""
    from ambc.distributed import decompress_multi
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
    ctx = _ctx([0, 0])
    assert decompress_multi(ctx, body, orig) == ref
    ctx.close()


# ---------------------------------------------------------------------------
# two processes, two GPUs, RCCL (skipped on a one-GPU box)
# ---------------------------------------------------------------------------
def _ngpus(lib):
    n = C.c_int(0)
    lib.ambc_device_count(C.byref(n))
    return n.value


def test_two_rank_rccl_bench(hip_lib):
    if _ngpus(hip_lib) < 2:
        pytest.skip("one GPU on this box: RCCL admits one rank per device")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.close()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--size", str(256 << 20), "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["round_trip_bit_exact"] is True
    assert line["config"]["reassembly_to_rank0"]["rank0_prefix_equal"] is True


def test_inprocess_rccl_devices(hip_lib):
    """A ctx over every GPU of the box: ncclCommInitAll communicators (no host
    transport), the slab pipeline in native mode, contiguous shards with the
    remainder exchange in reference mode, and the split decode -- all equal to
    the single-device results.  Skips on a one-GPU box."""
    ng = _ngpus(hip_lib)
    if ng < 2:
        pytest.skip("one GPU on this box")
    from ambc.distributed import decompress_multi
    assert "AMBC_LOCAL_TRANSPORT" not in os.environ
    devs = list(range(min(ng, 8)))
    n, chunk = (24 << 20) + 999, 4096
    data, ref = _body(n, chunk, (1, 3, 4, 9, 255), 61)
    multi = _ctx(devs)
    os.environ["AMBC_SLAB_BYTES"] = str(2 << 20)
    try:
        got, st = _compress(multi, data, chunk, (1, 3, 4, 9))
    finally:
        del os.environ["AMBC_SLAB_BYTES"]
    assert got == ref
    rdata = _ref_mode_input(1024, 24 * len(devs), 29)
    rref, _ = orc.compress_body(rdata, orc.make_params(1024, "reference", (1, 3, 4, 255), n_total=len(rdata)))
    rgot, _ = _compress(multi, rdata, 1024, (1, 3, 4), mode="reference")
    assert rgot == rref
    assert decompress_multi(multi, ref, n) == data
    multi.close()


def test_rccl_multi_rank_shards(hip_lib):
    """One process per GPU over RCCL (ambc_comm_init_rank; AMBC_LOCAL_TRANSPORT
    unset): compress_shard / decompress_shard / the xGMI gather in native mode
    (chunks 4096 and 8192) and reference mode, rank 0's body equal to the oracle
    and its decode equal to the input (tests/rccl_shard_worker.py).  Skips on a
    one-GPU box."""
    ng = _ngpus(hip_lib)
    if ng < 2:
        pytest.skip("one GPU on this box: RCCL admits one rank per device")
    import json
    world = min(ng, 8)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k != "AMBC_LOCAL_TRANSPORT"}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world))
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "rccl_shard_worker.py")],
                                      env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for pr in procs:
            o, e = pr.communicate(timeout=240)
            outs.append((pr.returncode, o, e))
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    for rc, o, e in outs:
        assert rc == 0, e[-2000:]
        line = json.loads(o.strip().splitlines()[-1])
        assert line["ok"] is True


@pytest.mark.parametrize("fail_rank", [0, 1, 2])
def test_sharded_reference_mode_failure_leaves_together(hip_lib, fail_rank):
    """A rank that fails after the pre-flight (ambc_test_inject_failure injects it)
    still joins the reference mode's remainder exchange and the size exchange:
    every rank returns an error, none waits for it, and the ctx works afterwards."""
    from ambc import _lib
    chunk, nchunks = 1024, 24
    data = _ref_mode_input(chunk, nchunks, 9)
    multi = _ctx([0] * 3)
    multi.lib.ambc_test_inject_failure(fail_rank)
    try:
        with pytest.raises(_lib.AmbcError):
            _compress(multi, data, chunk, (1, 3, 4), mode="reference")
    finally:
        multi.lib.ambc_test_inject_failure(-1)
    ref, _ = orc.compress_body(data, orc.make_params(chunk, "reference", (1, 3, 4, 255), n_total=len(data)))
    got, _ = _compress(multi, data, chunk, (1, 3, 4), mode="reference")
    assert got == ref
    multi.close()
