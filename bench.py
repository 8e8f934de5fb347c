#!/usr/bin/env python3
"""Benchmark of the MI355X compress path (BASELINE.json metric).  No PyTorch:
device memory, synthetic input, RCCL and timing all go through libambc_hip.

A step = one device-resident compress of the whole per-GPU input (configs[1]:
4 GiB "ambc-mixed v1" synthetic mixed-entropy bytes, chunk 4096, native mode,
GPU methods {RLE, Huffman, Delta, LZ4}) into a device-resident .ambc body.

With N > 1 ranks (one process per GPU) the input is ONE stream of N x 4 GiB and
rank r compresses its contiguous chunk shard (ambc_compress_shard; weak
scaling: the chunks are independent, so the data path has no collective); a
step ends with the RCCL AllGather of the body sizes (every rank's file offset)
and AllReduce(SUM) of the statistics.  Gathering the whole body onto rank 0
over xGMI (grouped ncclSend/ncclRecv) is timed separately, after the timed
steps ("reassembly_to_rank0").  value = input bytes of all ranks / time (GB/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3-1024|c3-16384|c4]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N`` without a launcher starts the N rank processes itself (before any
GPU call) and exits with the worst exit code.
"""
import argparse
import ctypes as C
import glob
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd")]

METRIC = ("compress GB/s + ratio, 4 GiB synthetic mixed-entropy @ chunk=4096; "
          "decompress round-trip bit-exact")
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)
GiB = 1 << 30
# BASELINE.json configs (per-GPU input, chunk): c4 = 32 GiB over 8 GPUs at chunk 8192
CONFIGS = {"c2": (4 * GiB, 4096), "c3-1024": (4 * GiB, 1024), "c3-16384": (4 * GiB, 16384),
           "c4": (4 * GiB, 8192)}
LZ4_NOTE = ("id 9 bytes are this project's 'ambc-lz4 greedy v2' LZ4 frames (valid LZ4, decodable by any "
            "LZ4 frame decoder), not python-lz4's HC-9 output, which is absent here and unpinned")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="BASELINE.json config preset (sets --size and --chunk)")
    ap.add_argument("--size", type=int, default=4 * GiB, help="input bytes per GPU")
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--mode", default="native", choices=["native", "reference"])
    ap.add_argument("--methods", default="1,3,4,9")
    ap.add_argument("--seed", type=int, default=20250418)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--py-seconds", type=float, default=12.0,
                    help="budget of the single-core pure-Python restatement leg")
    ap.add_argument("--no-e2e", action="store_true", help="skip the pinned host-to-host leg")
    ap.add_argument("--alt-methods", default="1,3,4;1,3,4,5;1,2,3,4;1,3,4,5z",
                    help="';'-separated method sets reported beside the headline ('' to skip): "
                         "1,3,4 = the reference's per-chunk GPU-routable set (BASELINE.md's CPU row); "
                         "1,3,4,5 = every package decodable by the stdlib-only reference; "
                         "a trailing z = id 5 as zlib.compress(data, 9)'s own bytes; "
                         "1,2,3,4 = the reference's own bytes (byte-pinned set)")
    ap.add_argument("--walk-bytes", type=int, default=256 << 20,
                    help="multi-size walk leg (the reference's eight candidates) on this prefix; 0: skip")
    ap.add_argument("--walk-methods", default="1,3,4,9;1,2,3,4,5")
    ap.add_argument("--ref-walk-bytes", type=int, default=64 << 20,
                    help="the reference's default compress() path (AdaptiveCompressor.like_reference(): "
                         "eight candidates, {1,2,3,4,5}, id 5 as zlib-9's bytes) on this many bytes; 0: skip")
    ap.add_argument("--ref-walk-check-bytes", type=int, default=4 << 20,
                    help="prefix on which the cpu_baseline leg times the oracle's reference walk and "
                         "compares its body with the GPU's")
    ap.add_argument("--ref-full-walk-bytes", type=int, default=16 << 20,
                    help="the reference's default compress() path with its whole stdlib method set "
                         "(like_reference(full_set=True): {1..7}, bz2 / LZMA scored on host threads) "
                         "on this many bytes; 0: skip")
    ap.add_argument("--ref-full-walk-check-bytes", type=int, default=1 << 20,
                    help="prefix on which that leg's body is compared with the oracle's reference loop")
    ap.add_argument("--api-bytes", type=int, default=256 << 20,
                    help="input size of the AdaptiveCompressor.compress(path, path) leg (0: skip)")
    a = ap.parse_args()
    if a.config:
        a.size, a.chunk = CONFIGS[a.config]
    return a


def spawn_ranks(n):
    """bench.py --gpus N without a launcher: N child processes, one per GPU,
    each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set.  This process
    never touches the GPU."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc]
    return bad[0] if bad else 0


def make_params(args, methods, n):
    from ambc import _lib
    from ambc.compressor import entropy_terms
    from ambc.registry import METHOD_CHUNK_PREFS, method_mask
    p = _lib.Params()
    p.chunk_size = args.chunk
    p.mode = _lib.MODE_REFERENCE if args.mode == "reference" else _lib.MODE_NATIVE
    p.method_mask = method_mask(methods)
    p.flags = _lib.FLAG_INPUT_PADDED      # (the device inputs below carry 64 bytes of slack)
    for i in range(16):
        lo, hi = METHOD_CHUNK_PREFS.get(i, (1, 0))
        p.pref_min[i], p.pref_max[i] = lo, min(hi, 0xFFFFFFFF)
    keep = [entropy_terms(args.chunk)]
    p.ent_full = keep[0].ctypes.data
    if n % args.chunk:
        keep.append(entropy_terms(n % args.chunk))
        p.ent_tail = keep[1].ctypes.data
    p._keep = keep
    return p


def cpu_baseline(args, threads, methods):
    """The CPU restatements of the oracle on bounded prefixes of the same
    stream, on the host: the C/OpenMP port on the box's CPU share, and the
    pure-Python restatement on one core.  The reference
    itself is pure Python and cannot be on the GPU box (BASELINE.md §2 has its
    numbers: 1.00 MB/s for {1,3,4} at chunk 4096 in the survey container)."""
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    from oracle import oracle as orc
    from oracle import pyref
    probe = 16 << 20
    data = orc.synth(probe, args.seed)
    p = orc.make_params(args.chunk, "native", methods, n_total=probe)
    t = time.time()
    orc.compress_body(data, p, nthreads=threads)
    rate = probe / max(time.time() - t, 1e-6)
    n = int(min(args.size, max(probe, rate * args.cpu_seconds)))
    n -= n % args.chunk
    data = orc.synth(n, args.seed)
    p = orc.make_params(args.chunk, "native", methods, n_total=n)
    t = time.time()
    body, _ = orc.compress_body(data, p, nthreads=threads)
    dt = time.time() - t
    del data
    # the reference's algorithm in CPython on one core: {1,3,4} (BASELINE.md §2's row)
    py_set = [m for m in (1, 3, 4)]
    pn = 1 << 20
    pdata = orc.synth(pn, args.seed)
    t = time.time()
    pbody = pyref.compress_body_native(pdata, args.chunk, py_set)
    prate = pn / max(time.time() - t, 1e-6)
    pn2 = int(min(64 << 20, max(pn, prate * args.py_seconds)))
    pn2 -= pn2 % args.chunk
    if pn2 > pn:
        pdata = orc.synth(pn2, args.seed)
        t = time.time()
        pbody = pyref.compress_body_native(pdata, args.chunk, py_set)
        prate = pn2 / max(time.time() - t, 1e-6)
    else:
        pn2 = pn
    same = pbody == orc.compress_body(pdata, orc.make_params(args.chunk, "native", py_set + [255],
                                                             n_total=pn2))[0]
    return {"value": round(n / dt / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "os_cpu_count": os.cpu_count(),
            "cores_note": "the box's CPU share for one GPU (OMP_NUM_THREADS); os_cpu_count is the whole host",
            "sample": f"first {n} bytes (seed {args.seed}) of the same stream, chunk {args.chunk}, methods "
                      f"{methods}, oracle/ambc_oracle.c OpenMP restatement, {dt:.1f} s wall, "
                      f"ratio {len(body) / n:.4f}",
            "python_single_core": {
                "value": round(prate / 1e9, 7), "unit": "GB/s", "cores": 1, "kind": "port",
                "sample": f"first {pn2} bytes of the same stream, chunk {args.chunk}, methods {py_set} "
                          f"(the reference's {{1,3,4,255}} set), oracle/pyref.py pure-Python restatement of "
                          f"adaptive_compressor.py:537-700, body identical to the C port: {same}",
                "extrapolated_4GiB_s": round((4 * GiB) / prate, 1)}}


def e2e_leg(lib, ctx, d_in, body_len, n, p, d_out, reps=3):
    """T_e2e: page-locked host input -> page-locked host body through
    ambc_compress_batch (slab pipeline: H2D, compress and D2H overlapped).  The
    body must equal the device-resident one byte for byte."""
    from ambc import _lib
    cap = lib.ambc_compress_bound(n, p.chunk_size)
    h_in = lib.ambc_host_alloc(n)
    h_out = lib.ambc_host_alloc(cap)
    if not h_in or not h_out:
        return None
    try:
        _lib.check(lib.ambc_memcpy_d2h(ctx.h, 0, h_in, int(d_in), n), lib)
        olen = C.c_uint64()
        st = _lib.Stats()
        u8p = C.POINTER(C.c_uint8)
        ts = []
        for i in range(reps + 1):
            t = time.perf_counter()
            _lib.check(lib.ambc_compress_batch(ctx.h, C.cast(h_in, u8p), n, C.byref(p),
                                               C.cast(h_out, u8p), cap, C.byref(olen),
                                               C.byref(st)), lib)
            if i:
                ts.append(time.perf_counter() - t)
        same = olen.value == body_len and device_equals_host(ctx, h_out, body_len, d_out)
        ts.sort()
        return {"GBps": round(n / ts[len(ts) // 2] / 1e9, 3), "ms": round(ts[len(ts) // 2] * 1e3, 3),
                "reps": reps, "host_buffers": "pinned (ambc_host_alloc)", "body_equal_device": same,
                "kernel_ms": round(st.kernel_ns / 1e6, 3)}
    finally:
        lib.ambc_host_free(h_in)
        lib.ambc_host_free(h_out)


def device_equals_host(ctx, host, n, d_ref):
    """host bytes (object or address) == n bytes at device pointer d_ref (uploaded, compared on the device)."""
    from ambc import _lib
    tmp = _lib.DeviceBuffer(ctx, n + 64)
    try:
        src = host if isinstance(host, int) else _lib.addr(host)
        _lib.check(ctx.lib.ambc_memcpy_h2d(ctx.h, 0, tmp.ptr, src, n), ctx.lib)
        eq = C.c_int(0)
        _lib.check(ctx.lib.ambc_device_equal(ctx.h, 0, tmp.ptr, int(d_ref), n, C.byref(eq)), ctx.lib)
        return bool(eq.value)
    finally:
        tmp.free()


def api_leg(nbytes, chunk, mode, methods, seed):
    """T_api: AdaptiveCompressor.compress(path, path) wall time on a
    file of the same stream (file read, MD5, compress, file write included),
    then decompress(path, path) with its MD5 check."""
    import tempfile
    from ambc import AdaptiveCompressor
    from ambc import _lib
    data = bytearray(nbytes)
    _lib.load().ambc_synth_fill(_lib.addr(data), nbytes, seed)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        src, dst, back = (os.path.join(td, x) for x in ("in.bin", "out.ambc", "back.bin"))
        with open(src, "wb") as f:
            f.write(data)
        comp = AdaptiveCompressor(chunk_size=chunk, mode=mode, methods=methods)
        comp.compress(src, dst)                       # warm-up
        t = time.perf_counter()
        stats = comp.compress(src, dst)
        tc = time.perf_counter() - t
        t = time.perf_counter()
        comp.decompress(dst, back)
        td_ = time.perf_counter() - t
        with open(back, "rb") as f:
            ok = f.read() == data
    return {"bytes": nbytes, "compress_GBps": round(nbytes / tc / 1e9, 3),
            "decompress_GBps": round(nbytes / td_ / 1e9, 3), "round_trip_bit_exact": ok,
            "ratio": round(stats["compressed_size"] / nbytes, 5) if "compressed_size" in stats else None}


def alt_leg(lib, ctx, d_in, n, args, methods, steps, zlib9=False):
    """The same input under another method set (device-resident, same clock
    discipline as the headline), its ratio and a bit-exact decode.  zlib9: id 5
    as zlib.compress(data, 9)'s own bytes (AMBC_FLAG_ZLIB9); the id-5 packages
    of a 16 MiB prefix are compared with Python's zlib.compress(chunk, 9)."""
    from ambc import _lib, AdaptiveCompressor
    p = make_params(args, methods, n)
    if zlib9:
        p.flags |= _lib.FLAG_ZLIB9
    cap = lib.ambc_compress_bound(n, args.chunk)
    d_out = _lib.DeviceBuffer(ctx, cap + 64)
    olen = C.c_uint64()
    st = _lib.Stats()
    enc = []

    def once():
        _lib.check(lib.ambc_compress_device(ctx.h, 0, d_in.ptr, n, C.byref(p), d_out.ptr,
                                            cap, C.byref(olen), C.byref(st), None), lib)
        e = C.c_uint64()
        lib.ambc_last_kernel_times(ctx.h, 0, C.byref(e), None, None)
        enc.append(e.value)

    try:
        once()
        enc.clear()
        lib.ambc_synchronize(ctx.h, 0)
        t0 = time.perf_counter()
        for _ in range(steps):
            once()
        lib.ambc_synchronize(ctx.h, 0)
        dt = (time.perf_counter() - t0) / steps
        body = bytes(d_out.download(olen.value))
        usage = {i: int(st.method_usage[i]) for i in range(256) if st.method_usage[i]}
    finally:
        d_out.free()
    comp = AdaptiveCompressor(chunk_size=args.chunk, mode=args.mode, methods=methods)
    back = comp._adaptive_decompress(body, n)
    ok = device_equals_host(ctx, back, n, d_in)
    del back
    t = time.perf_counter()                     # (the second call: the main leg's host_api_GBps)
    back = comp._adaptive_decompress(body, n)
    dwall = time.perf_counter() - t
    ok = ok and device_equals_host(ctx, back, n, d_in)
    del back
    ds = comp._last_device_stats
    z9 = None
    if zlib9:
        import zlib
        pre = d_in.download(min(n, 16 << 20))
        pos = off = checked = same = 0
        while pos + 18 <= len(body) and body[pos + 4] != 0 and off + args.chunk <= len(pre):
            orig = int.from_bytes(body[pos + 10:pos + 14], "little")
            clen = int.from_bytes(body[pos + 14:pos + 18], "little")
            if body[pos + 4] == 5:
                checked += 1
                same += body[pos + 18:pos + 18 + clen] == zlib.compress(bytes(pre[off:off + orig]), 9)
            pos += 18 + clen
            off += orig
        z9 = {"id5_encoder": "zlib.compress(data, 9) bytes (AMBC_FLAG_ZLIB9)",
              "id5_packages_checked_vs_python_zlib": checked, "identical": same,
              "zlib_version": zlib.ZLIB_RUNTIME_VERSION}
    return {"methods": methods, **({"zlib9": z9} if z9 else {}),
            "GBps": round(n / dt / 1e9, 3), "ms_per_step": round(dt * 1e3, 3),
            "steps": steps, "ratio": round(olen.value / n, 5), "method_usage": usage,
            "kernels_ms": round(sum(enc) / len(enc) / 1e6, 3), "round_trip_bit_exact": ok,
            "decode": {"kernel_ms": round(ds.kernel_ns / 1e6, 3), "host_zlib_ms": round(ds.host_codec_ns / 1e6, 3),
                       "header_walk_ms": round(ds.walk_ns / 1e6, 3), "host_api_GBps": round(n / dwall / 1e9, 3)}}


def ref_walk_leg(ctx, nbytes, full_set=False, check_bytes=0):
    """The reference's own default compress() path at the reference's bytes:
    AdaptiveCompressor.like_reference() -- the eight CHUNK_SIZE_CANDIDATES walk
    (adaptive_compressor.py:61-62,537-590), id 5 as zlib.compress(chunk, 9)'s own
    bytes (advanced_compression.py:76-81) at every size -- host bytes in and out,
    second call timed, bit-exact decode.  full_set=False: its GPU-encodable
    stdlib codecs {1,2,3,4,5} (ids 6 / 7 left out); full_set=True: the reference's
    whole default set {1..7} (adaptive_compressor.py:129-176, compression_fix.py:
    60-125), bz2 / LZMA scored on host threads beside the device, and the body of
    a check_bytes prefix compared with the oracle's restatement of the reference
    loop with the same stdlib calls.  Input: multisize_bench's mixed segments (on
    the headline's stream the walk stores the rest raw at the first random byte
    run)."""
    from ambc import AdaptiveCompressor
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from multisize_bench import mixed
    data = mixed(nbytes, 7)
    comp = AdaptiveCompressor.like_reference(full_set=full_set)
    comp._adaptive_compress(data)
    t = time.perf_counter()
    body = comp._adaptive_compress(data)
    dt = time.perf_counter() - t
    steps, ev, wns, ens = C.c_uint32(), C.c_uint64(), C.c_uint64(), C.c_uint64()
    ctx.lib.ambc_last_multisize_info(comp._ctx().h, C.byref(steps), C.byref(ev), C.byref(wns), C.byref(ens))
    cs = dict(comp.chunk_stats)                  # (the timed call's: the check below compresses again)
    ok = comp._adaptive_decompress(body, nbytes) == data
    ids = [m.type_id for m in comp.compression_methods]
    check = None
    if full_set and check_bytes:
        from oracle import oracle as orc
        pre = data[:check_bytes]
        t = time.perf_counter()
        ref, _ = orc.compress_body_multisize(pre, comp.CHUNK_SIZE_CANDIDATES, tuple(ids), deflate="zlib",
                                             reference_set=True)
        dto = time.perf_counter() - t
        check = {"bytes": check_bytes, "gpu_body_equals_oracle": comp._adaptive_compress(pre) == ref,
                 "oracle_seconds": round(dto, 3), "oracle_GBps_1core": round(check_bytes / dto / 1e9, 6)}
    path = ("AdaptiveCompressor.like_reference(full_set=True): the reference's default compress() walk with "
            "its whole stdlib method set {1,2,3,4,5,6,7} (bz2 / LZMA scored on host threads)" if full_set else
            "AdaptiveCompressor.like_reference(): the reference's default compress() walk restricted to its "
            "GPU-encodable stdlib codecs {1,2,3,4,5} (ids 6 / 7 left out: like_reference_full_walk has them)")
    return {"path": path, **({"oracle_check": check} if check else {}),
            "methods": ids, "deflate": comp.deflate,
            "candidates": comp.CHUNK_SIZE_CANDIDATES, "bytes": nbytes,
            "input": "runs / text / skewed random, 8-64 KiB segments (scripts/multisize_bench.py mixed, seed 7)",
            "GBps": round(nbytes / dt / 1e9, 3), "seconds": round(dt, 4), "ratio": round(len(body) / nbytes, 5),
            "packages": cs["total_chunks"], "method_usage": cs["method_usage"],
            "walk_rounds": steps.value, "chunk_encodes": ev.value,
            "walk_ms": round(wns.value / 1e6, 2), "final_encode_ms": round(ens.value / 1e6, 2),
            "round_trip_bit_exact": ok}


def cpu_baseline_ref_walk(nbytes):
    """cpu_baseline leg of the like_reference() walk: the oracle's restatement of the
    reference's walk (oracle.compress_body_multisize with the system zlib at level
    9 -- one host core, the reference is single-threaded) timed on a bounded prefix
    of the same input, and its body compared with the GPU's body of that prefix."""
    from ambc import AdaptiveCompressor
    from oracle import oracle as orc
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from multisize_bench import mixed
    data = mixed(nbytes, 7)
    comp = AdaptiveCompressor.like_reference()
    body = comp._adaptive_compress(data)
    t = time.perf_counter()
    ref, _ = orc.compress_body_multisize(data, comp.CHUNK_SIZE_CANDIDATES, (1, 2, 3, 4, 5, 255), deflate="zlib")
    dt = time.perf_counter() - t
    return {"value": round(nbytes / dt / 1e9, 5), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"first {nbytes} bytes of the like_reference leg's input, oracle walk (C restatement, "
                      "system zlib level 9)", "seconds": round(dt, 3),
            "gpu_body_equals_oracle": ref == body}


def walk_leg(ctx, nbytes, methods):
    """The reference's default API path: _adaptive_compress with its eight
    CHUNK_SIZE_CANDIDATES (the multi-size walk, ambc_compress_multisize), host
    bytes in and out (upload, walk, final encode, body copy back); the second call
    is timed; bit-exact decode.  Input: runs, text and skewed-random segments of
    8-64 KiB (scripts/multisize_bench.py) -- on the headline's stream the
    reference's walk stops at its first incompressible position and stores the
    rest raw (its remainder rule, adaptive_compressor.py:586-588), which would
    time almost nothing."""
    from ambc import AdaptiveCompressor
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from multisize_bench import mixed
    data = mixed(nbytes, 7)
    comp = AdaptiveCompressor(methods=methods)
    comp.CHUNK_SIZE_CANDIDATES = list(comp.REFERENCE_CHUNK_SIZE_CANDIDATES)
    comp._adaptive_compress(data)
    t = time.perf_counter()
    body = comp._adaptive_compress(data)
    dt = time.perf_counter() - t
    steps, ev, wns, ens = C.c_uint32(), C.c_uint64(), C.c_uint64(), C.c_uint64()
    ctx.lib.ambc_last_multisize_info(comp._ctx().h, C.byref(steps), C.byref(ev), C.byref(wns), C.byref(ens))
    ok = comp._adaptive_decompress(body, nbytes) == data
    return {"methods": methods, "candidates": comp.CHUNK_SIZE_CANDIDATES, "bytes": nbytes,
            "input": "runs / text / skewed random, 8-64 KiB segments (scripts/multisize_bench.py mixed, seed 7)",
            "GBps": round(nbytes / dt / 1e9, 3), "seconds": round(dt, 4), "ratio": round(len(body) / nbytes, 5),
            "packages": comp.chunk_stats["total_chunks"], "walk_rounds": steps.value, "chunk_encodes": ev.value,
            "walk_ms": round(wns.value / 1e6, 2), "final_encode_ms": round(ens.value / 1e6, 2),
            "round_trip_bit_exact": ok}


def percentile(xs, q):
    """Linear-interpolated percentile of a small sample (rank 0's own step times)."""
    v = sorted(xs)
    if not v:
        return 0.0
    k = (len(v) - 1) * q / 100.0
    lo = int(k)
    hi = min(lo + 1, len(v) - 1)
    return v[lo] + (v[hi] - v[lo]) * (k - lo)


def pmc_traffic(workload):
    """HBM bytes per k_encode launch from a committed rocprofv3 --pmc summary
    (scripts/pmc_summary.py), if one exists for this workload (newest round wins)."""
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json"))):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and d.get("hbm_bytes_per_launch"):
            d["_file"] = f
            best = d
    return best


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    from ambc import _lib
    from ambc.comm import GpuGroup, env_ranks
    from ambc.distributed import gather, shard_range
    rank, world, local = env_ranks()
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU "
            f"(torch.distributed.run --nproc-per-node {args.gpus}) or run bench.py --gpus N alone")
        sys.exit(2)
    lib = _lib.load()
    ndev = C.c_int(0)
    if lib.ambc_device_count(C.byref(ndev)) != 0 or ndev.value <= local:
        log(f"bench.py: rank {rank} needs GPU {local}, {ndev.value} visible")
        sys.exit(3)
    group = GpuGroup(rank, world, local)
    ctx = group.ctx
    n = args.size
    n_total = n * world
    methods = [int(x) for x in args.methods.split(",")]
    p = make_params(args, methods, n_total if world > 1 else n)
    b0, b1 = (0, n) if world == 1 else shard_range(n_total, args.chunk, world, rank)
    sn = b1 - b0
    # this rank's bytes [b0, b1) of ONE n_total-byte stream
    d_in = _lib.DeviceBuffer(ctx, sn + 64)
    _lib.check(lib.ambc_synth_device_range(ctx.h, 0, d_in.ptr, n_total, b0, b1, args.seed), lib)
    cap = lib.ambc_compress_bound(sn, args.chunk)
    d_out = _lib.DeviceBuffer(ctx, cap + 64)
    olen = C.c_uint64()
    st = _lib.Stats()
    info = _lib.ShardInfo()
    enc_ns = []
    launches = [1]      # k_encode launches per call (pipelined segments)

    def step():
        if world == 1:
            _lib.check(lib.ambc_compress_device(ctx.h, 0, d_in.ptr, n, C.byref(p), d_out.ptr, cap,
                                                C.byref(olen), C.byref(st), None), lib)
        else:
            _lib.check(lib.ambc_compress_shard(ctx.h, d_in.ptr, n_total, C.byref(p), d_out.ptr, cap, -1,
                                               C.byref(info), C.byref(st)), lib)
            olen.value = info.local_len
        e = C.c_uint64()
        lib.ambc_last_kernel_times(ctx.h, 0, C.byref(e), None, None)
        nl = C.c_uint32()
        lib.ambc_last_encode_launches(ctx.h, 0, C.byref(nl))
        enc_ns.append(e.value / max(1, nl.value))     # per k_encode launch
        launches[0] = max(1, nl.value)

    for _ in range(args.warmup):
        step()
    enc_ns.clear()
    group.barrier()
    t0 = time.perf_counter()
    step_s = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        step()                      # the library call returns after its stream has drained
        step_s.append(time.perf_counter() - ts)
    group.barrier()
    dt = time.perf_counter() - t0
    body_len = olen.value
    body_total = body_len if world == 1 else info.total
    if world > 1:
        dt = max(x[0] for x in group.host.allgather_obj([dt]))

    reasm = shard_check = None
    if world > 1:
        # the whole body onto rank 0 in file order (grouped send/recv over xGMI), outside the timed steps
        d_all = _lib.DeviceBuffer(ctx, (body_total if rank == 0 else 0) + 64)
        group.barrier()
        tr = time.perf_counter()
        _, tot = gather(group, d_out.ptr, body_len, d_all.ptr if rank == 0 else None,
                        body_total + 64 if rank == 0 else 0)
        group.barrier()
        tr = max(x[0] for x in group.host.allgather_obj([time.perf_counter() - tr]))
        same = True
        if rank == 0:       # rank 0's own packages lead the gathered body
            eq = C.c_int(0)
            _lib.check(lib.ambc_device_equal(ctx.h, 0, d_all.ptr, d_out.ptr, body_len, C.byref(eq)), lib)
            same = bool(eq.value) and tot == body_total
        d_all.free()
        reasm = {"ms": round(tr * 1e3, 3), "body_bytes": int(body_total),
                 "GBps_into_rank0": round(body_total / tr / 1e9, 3), "rank0_prefix_equal": same}
        if not args.no_verify:
            # every rank decodes its own packages (the file-order body is their concatenation)
            from ambc import AdaptiveCompressor
            comp = AdaptiveCompressor(chunk_size=args.chunk, mode=args.mode, methods=methods)
            back = comp._adaptive_decompress(bytes(d_out.download(body_len)), sn)
            ok = device_equals_host(ctx, back, sn, d_in)
            oks = group.host.allgather_obj([1.0 if ok else 0.0])
            shard_check = all(x[0] == 1.0 for x in oks)

    verified = decode = None
    if not args.no_verify and world == 1:
        # bit-exact round trip of the last step's body (outside the timed region)
        body_host = bytes(d_out.download(body_len))
        from ambc import AdaptiveCompressor
        comp = AdaptiveCompressor(chunk_size=args.chunk, mode=args.mode, methods=methods)
        t = time.perf_counter()
        back = comp._adaptive_decompress(body_host, n)
        dcold = time.perf_counter() - t                 # first call: + pinned staging setup
        verified = device_equals_host(ctx, back, n, d_in)
        del back
        t = time.perf_counter()
        back = comp._adaptive_decompress(body_host, n)
        dwall = time.perf_counter() - t
        verified = verified and device_equals_host(ctx, back, n, d_in)
        del back
        ds = comp._last_device_stats
        decode = {"kernel_ms": round(ds.kernel_ns / 1e6, 3), "header_walk_ms": round(ds.walk_ns / 1e6, 3),
                  "h2d_ms": round(ds.h2d_ns / 1e6, 3), "d2h_ms": round(ds.d2h_ns / 1e6, 3),
                  "kernel_GBps": round(n / max(ds.kernel_ns, 1), 3),
                  "host_api_GBps": round(n / dwall / 1e9, 3),
                  "host_api_GBps_first_call": round(n / dcold / 1e9, 3),
                  "process": "torch-free (bench.py imports no torch)"}
        log(f"round trip bit-exact: {verified}; decode {decode}")
    elif shard_check is not None:
        verified = shard_check

    e2e = api = None
    alts = []
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e = e2e_leg(lib, ctx, d_in.ptr, body_len, n, p, d_out.ptr)
        log(f"e2e: {e2e}")
    if rank == 0 and world == 1 and args.alt_methods:
        for ms in args.alt_methods.split(";"):
            if ms.strip():
                z = ms.strip().endswith("z")   # "...z": id 5 as zlib-9's own bytes
                alt = alt_leg(lib, ctx, d_in, n, args, [int(x) for x in ms.strip().rstrip("z").split(",")],
                              max(2, args.steps // 2), zlib9=z)
                log(f"alt: {alt}")
                alts.append(alt)
    walks = []
    if rank == 0 and world == 1 and args.walk_bytes:
        for ms in args.walk_methods.split(";"):
            if ms.strip():
                w = walk_leg(ctx, args.walk_bytes, [int(x) for x in ms.split(",")])
                log(f"walk: {w}")
                walks.append(w)
    ref_walk = ref_full = None
    if rank == 0 and world == 1 and args.ref_walk_bytes:
        ref_walk = ref_walk_leg(ctx, args.ref_walk_bytes)
        log(f"like_reference walk: {ref_walk}")
    if rank == 0 and world == 1 and args.ref_full_walk_bytes:
        ref_full = ref_walk_leg(ctx, args.ref_full_walk_bytes, full_set=True,
                                check_bytes=args.ref_full_walk_check_bytes)
        log(f"like_reference full walk: {ref_full}")
    if rank == 0 and world == 1 and args.api_bytes:
        api = api_leg(args.api_bytes, args.chunk, args.mode, methods, args.seed)
        log(f"api: {api}")

    if rank == 0:
        total_in = n_total * args.steps
        value = total_in / dt / 1e9
        enc_avg = sum(enc_ns) / max(1, len(enc_ns))
        # read input once + write body once, per launch (a call = launches[0] equal segments)
        algo_bytes = (sn + body_len) / launches[0]
        achieved = algo_bytes / (enc_avg * 1e-9) / 1e9 if enc_avg else 0.0
        workload = f"ambc-mixed-v1 {n >> 30} GiB/GPU chunk={args.chunk} {args.mode}"
        pmc = pmc_traffic(workload)
        result = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": workload, "config": args.config or "c2",
                       "input_bytes_per_gpu": n, "input_bytes_total": n_total,
                       "chunk_size": args.chunk, "mode": args.mode, "methods": methods, "seed": args.seed,
                       "ratio": round(body_total / n_total, 5),
                       "parallelism": f"chunk-shard dp{world} (RCCL)" if world > 1 else "single GPU",
                       "round_trip_bit_exact": verified, "decode": decode,
                       "lz4_bytes": LZ4_NOTE if 9 in methods else None,
                       "reassembly_to_rank0": reasm,
                       "step_ms_p50": round(percentile(step_s, 50) * 1e3, 3),
                       "step_ms_p90": round(percentile(step_s, 90) * 1e3, 3),
                       "e2e_pinned_host": e2e, "api_file": api, "alt_method_sets": alts,
                       "multisize_walk": walks, "like_reference_walk": ref_walk,
                       "like_reference_full_walk": ref_full},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                         "traffic_source": os.path.relpath(pmc["_file"], REPO) if pmc and "_file" in pmc else None,
                         "kernel": "k_encode", "kernel_ms": round(enc_avg * 1e-6, 3),
                         "algorithmic_bytes_per_launch": round(algo_bytes),
                         "launches_per_step": launches[0]},
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
            result["cpu_baseline"] = cpu_baseline(args, threads, methods)
            if ref_walk is not None and args.ref_walk_check_bytes:
                result["cpu_baseline"]["like_reference_walk"] = cpu_baseline_ref_walk(args.ref_walk_check_bytes)
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    d_in.free()
    d_out.free()
    group.barrier()
    group.close()


if __name__ == "__main__":
    main()
