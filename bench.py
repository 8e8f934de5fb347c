#!/usr/bin/env python3
"""Benchmark of the MI355X compress path (BASELINE.json metric).

A step = one device-resident compress of the whole per-GPU input (configs[1]:
4 GiB "ambc-mixed v1" synthetic mixed-entropy bytes, chunk 4096, native mode,
GPU methods {RLE, Huffman, Delta, LZ4}) into a device-resident .ambc body;
with N > 1 ranks every rank compresses its own 4 GiB shard (weak scaling; the
chunks are independent, so there is no data-path collective) and the step ends
with the all_gather of the 8-byte body sizes that gives every rank its offset in
the file-order body (ambc.distributed.file_offsets).  Gathering the whole body
onto rank 0 over RCCL/xGMI (ambc.distributed.reassemble) is timed separately,
after the timed steps ("reassembly_to_rank0").  value = input bytes of all
ranks / time (GB/s, 1e9).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
"""
import argparse
import ctypes as C
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd")]

METRIC = ("compress GB/s + ratio, 4 GiB synthetic mixed-entropy @ chunk=4096; "
          "decompress round-trip bit-exact")
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=4 << 30, help="input bytes per GPU")
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--mode", default="native", choices=["native", "reference"])
    ap.add_argument("--methods", default="1,3,4,9")
    ap.add_argument("--seed", type=int, default=20250418)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-e2e", action="store_true", help="skip the pinned host-to-host leg")
    ap.add_argument("--alt-methods", default="1,3,4,5",
                    help="second method set reported beside the headline ('' to skip): "
                         "1,3,4,5 = RLE/Huffman/Delta/DEFLATE (every package decodable by the "
                         "stdlib-only reference)")
    ap.add_argument("--api-bytes", type=int, default=256 << 20,
                    help="input size of the AdaptiveCompressor.compress(path, path) leg (0: skip)")
    return ap.parse_args()


def cpu_baseline(args, threads):
    """The CPU restatement (oracle, "port") on a bounded prefix of the same
    workload, on the host cores; the reference itself is pure Python and is
    not present on the GPU box (BASELINE.md §2-3 has its numbers)."""
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    from oracle import oracle as orc
    probe = 16 << 20
    data = orc.synth(probe, args.seed)
    p = orc.make_params(args.chunk, "native", [int(x) for x in args.methods.split(",")],
                        n_total=probe)
    t = time.time()
    orc.compress_body(data, p, nthreads=threads)
    rate = probe / max(time.time() - t, 1e-6)
    n = int(min(args.size, max(probe, rate * args.cpu_seconds)))
    n -= n % args.chunk
    data = orc.synth(n, args.seed)
    p = orc.make_params(args.chunk, "native", [int(x) for x in args.methods.split(",")],
                        n_total=n)
    t = time.time()
    body, _ = orc.compress_body(data, p, nthreads=threads)
    dt = time.time() - t
    # the reference is single-threaded by construction: the same port on one core
    n1 = min(probe, n)
    p1 = orc.make_params(args.chunk, "native", [int(x) for x in args.methods.split(",")],
                         n_total=n1)
    t = time.time()
    orc.compress_body(data[:n1], p1, nthreads=1)
    dt1 = time.time() - t
    return {"value": round(n / dt / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"first {n} bytes (seed {args.seed}) of the same stream, chunk "
                      f"{args.chunk}, oracle/ambc_oracle.c OpenMP restatement, "
                      f"{dt:.1f} s wall, ratio {len(body) / n:.4f}",
            "single_core": {"value": round(n1 / dt1 / 1e9, 4), "unit": "GB/s", "cores": 1,
                            "sample": f"first {n1} bytes, same port, one thread, {dt1:.1f} s"}}


def e2e_leg(lib, ctx, d_in, d_out, body_len, n, p, reps=3):
    """T_e2e: page-locked host input -> page-locked host body through
    ambc_compress_batch (slab pipeline: H2D, compress and D2H overlapped).  The
    body must equal the device-resident one byte for byte."""
    import numpy as np
    import torch
    from ambc import _lib
    cap = lib.ambc_compress_bound(n, p.chunk_size)
    h_in = lib.ambc_host_alloc(n)
    h_out = lib.ambc_host_alloc(cap)
    if not h_in or not h_out:
        return None
    try:
        _lib.check(lib.ambc_memcpy_d2h(ctx.h, 0, h_in, d_in.data_ptr(), n), lib)
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
        got = np.ctypeslib.as_array((C.c_uint8 * olen.value).from_address(h_out))
        same = olen.value == body_len and bool(
            torch.equal(torch.from_numpy(got).to(d_out.device), d_out[:body_len]))
        ts.sort()
        return {"GBps": round(n / ts[len(ts) // 2] / 1e9, 3), "ms": round(ts[len(ts) // 2] * 1e3, 3),
                "reps": reps, "host_buffers": "pinned (ambc_host_alloc)", "body_equal_device": same,
                "kernel_ms": round(st.kernel_ns / 1e6, 3)}
    finally:
        lib.ambc_host_free(h_in)
        lib.ambc_host_free(h_out)


def api_leg(nbytes, chunk, mode, methods, seed):
    """T_api: AdaptiveCompressor.compress(path, path) wall time on a
    file of the same stream (file read, MD5, compress, file write included),
    then decompress(path, path) with its MD5 check."""
    import tempfile
    from ambc import AdaptiveCompressor
    from oracle import synth
    data = synth.generate(nbytes, seed)
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


def alt_leg(lib, ctx, d_in, n, args, methods, steps):
    """The same input under another method set (device-resident, same clock
    discipline as the headline), its ratio and a bit-exact decode."""
    import torch
    from ambc import _lib, AdaptiveCompressor
    from ambc.compressor import entropy_terms
    from ambc.registry import METHOD_CHUNK_PREFS, method_mask
    p = _lib.Params()
    p.chunk_size = args.chunk
    p.mode = _lib.MODE_REFERENCE if args.mode == "reference" else _lib.MODE_NATIVE
    p.method_mask = method_mask(methods)
    for i in range(16):
        lo, hi = METHOD_CHUNK_PREFS.get(i, (1, 0))
        p.pref_min[i], p.pref_max[i] = lo, min(hi, 0xFFFFFFFF)
    tabs = [entropy_terms(args.chunk)]
    p.ent_full = tabs[0].ctypes.data
    if n % args.chunk:
        tabs.append(entropy_terms(n % args.chunk))
        p.ent_tail = tabs[1].ctypes.data
    cap = lib.ambc_compress_bound(n, args.chunk)
    d_out = torch.empty(cap + 64, dtype=torch.uint8, device=d_in.device)
    olen = C.c_uint64()
    st = _lib.Stats()
    enc = []

    def once():
        _lib.check(lib.ambc_compress_device(ctx.h, 0, d_in.data_ptr(), n, C.byref(p), d_out.data_ptr(),
                                            cap, C.byref(olen), C.byref(st), None), lib)
        e = C.c_uint64()
        lib.ambc_last_kernel_times(ctx.h, 0, C.byref(e), None, None)
        enc.append(e.value)

    once()
    enc.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        once()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    body = d_out[:olen.value].cpu().numpy().tobytes()
    comp = AdaptiveCompressor(chunk_size=args.chunk, mode=args.mode, methods=methods)
    t = time.perf_counter()
    back = comp._adaptive_decompress(body, n)
    dwall = time.perf_counter() - t
    ok = equals_device(back, d_in)
    ds = comp._last_device_stats
    usage = {i: int(st.method_usage[i]) for i in range(256) if st.method_usage[i]}
    return {"methods": methods, "GBps": round(n / dt / 1e9, 3), "ms_per_step": round(dt * 1e3, 3),
            "steps": steps, "ratio": round(olen.value / n, 5), "method_usage": usage,
            "kernels_ms": round(sum(enc) / len(enc) / 1e6, 3), "round_trip_bit_exact": ok,
            "decode": {"kernel_ms": round(ds.kernel_ns / 1e6, 3), "host_zlib_ms": round(ds.host_codec_ns / 1e6, 3),
                       "header_walk_ms": round(ds.walk_ns / 1e6, 3), "host_api_GBps": round(n / dwall / 1e9, 3)}}


def equals_device(host_bytes, d_ref):
    """host_bytes == the device tensor d_ref, compared on the device (no 4 GiB
    host temporaries that would fragment the memory the next decode faults in)."""
    import warnings

    import torch
    if len(host_bytes) != d_ref.numel():
        return False
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")               # read-only buffer: we only read it
        h = torch.frombuffer(host_bytes, dtype=torch.uint8)
    return bool(torch.equal(h.to(d_ref.device), d_ref))


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
    (scripts/pmc_summary.py), if one exists for this workload."""
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json"))):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and d.get("hbm_bytes_per_launch"):
            best = d
    return best


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    from ambc import _lib
    from ambc.compressor import entropy_terms
    from ambc.registry import METHOD_CHUNK_PREFS, method_mask

    ctx = _lib.Context([local])
    lib = ctx.lib
    n = args.size
    methods = [int(x) for x in args.methods.split(",")]
    p = _lib.Params()
    p.chunk_size = args.chunk
    p.mode = _lib.MODE_REFERENCE if args.mode == "reference" else _lib.MODE_NATIVE
    p.method_mask = method_mask(methods)
    for i in range(16):
        lo, hi = METHOD_CHUNK_PREFS.get(i, (1, 0))
        p.pref_min[i], p.pref_max[i] = lo, min(hi, 0xFFFFFFFF)
    tabs = [entropy_terms(args.chunk)]
    p.ent_full = tabs[0].ctypes.data
    if n % args.chunk:
        tabs.append(entropy_terms(n % args.chunk))
        p.ent_tail = tabs[1].ctypes.data
    if world > 1:
        p.flags |= _lib.FLAG_NO_END_CHUNK

    d_in = torch.empty(n, dtype=torch.uint8, device=dev)
    _lib.check(lib.ambc_synth_device(ctx.h, 0, d_in.data_ptr(), n, args.seed + rank), lib)
    cap = lib.ambc_compress_bound(n, args.chunk)
    # rank 0 compresses straight into the front of the reassembly buffer
    out_cap = cap * (world if rank == 0 and world > 1 else 1) + 64
    d_out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    olen = C.c_uint64()
    st = _lib.Stats()
    enc_ns = []
    launches = [1]      # k_encode launches per call (pipelined segments)

    def step():
        _lib.check(lib.ambc_compress_device(ctx.h, 0, d_in.data_ptr(), n, C.byref(p),
                                            d_out.data_ptr(), cap, C.byref(olen), C.byref(st),
                                            None), lib)
        e = C.c_uint64()
        lib.ambc_last_kernel_times(ctx.h, 0, C.byref(e), None, None)
        nl = C.c_uint32()
        lib.ambc_last_encode_launches(ctx.h, 0, C.byref(nl))
        enc_ns.append(e.value / max(1, nl.value))     # per k_encode launch
        launches[0] = max(1, nl.value)
        if world > 1:
            from ambc.distributed import file_offsets
            file_offsets(olen.value, dev)

    for _ in range(args.warmup):
        step()
    enc_ns.clear()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_s = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        step()                      # the library call returns after its stream has drained
        step_s.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    body_len = olen.value
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt, float(body_len)], dtype=torch.float64, device=dev)
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        dt = float(tmax[0].item())
        body_total = float(tsum[1].item()) + 16
    else:
        body_total = float(body_len)

    reasm = None
    if world > 1:
        # the whole body onto rank 0 in file order (P2P over xGMI), outside the timed steps
        from ambc.distributed import reassemble
        torch.distributed.barrier()
        torch.cuda.synchronize()
        tr = time.perf_counter()
        reassemble(d_out[:body_len], dst=0, out=d_out if rank == 0 else None)
        torch.cuda.synchronize()
        tr = time.perf_counter() - tr
        tt = torch.tensor([tr], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        reasm = {"ms": round(tt.item() * 1e3, 3), "body_bytes": int(body_total),
                 "GBps_into_rank0": round(body_total / tt.item() / 1e9, 3)}

    verified = None
    decode = None
    if not args.no_verify and rank == 0:
        # bit-exact round trip of the last step's body (outside the timed region)
        body_host = d_out[:body_len if world == 1 else body_len].cpu().numpy().tobytes()
        if world > 1:
            body_host += b"\xff\xff" + b"\x00" * 14
        from ambc import AdaptiveCompressor
        comp = AdaptiveCompressor(chunk_size=args.chunk, mode=args.mode, methods=methods)
        t = time.perf_counter()
        back = comp._adaptive_decompress(body_host, n)
        dcold = time.perf_counter() - t                 # first call: + pinned staging setup
        verified = equals_device(back, d_in)
        del back
        t = time.perf_counter()
        back = comp._adaptive_decompress(body_host, n)
        dwall = time.perf_counter() - t
        verified = verified and equals_device(back, d_in)
        ds = comp._last_device_stats
        decode = {"kernel_ms": round(ds.kernel_ns / 1e6, 3), "header_walk_ms": round(ds.walk_ns / 1e6, 3),
                  "h2d_ms": round(ds.h2d_ns / 1e6, 3), "d2h_ms": round(ds.d2h_ns / 1e6, 3),
                  "kernel_GBps": round(n / max(ds.kernel_ns, 1), 3),
                  "host_api_GBps": round(n / dwall / 1e9, 3),
                  "host_api_GBps_first_call": round(n / dcold / 1e9, 3)}
        log(f"round trip bit-exact: {verified}; decode {decode}")

    e2e = api = None
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e = e2e_leg(lib, ctx, d_in, d_out, body_len, n, p)
        log(f"e2e: {e2e}")
    alt = None
    if rank == 0 and world == 1 and args.alt_methods:
        alt = alt_leg(lib, ctx, d_in, n, args, [int(x) for x in args.alt_methods.split(",")], args.steps)
        log(f"alt: {alt}")
    if rank == 0 and world == 1 and args.api_bytes:
        api = api_leg(args.api_bytes, args.chunk, args.mode, methods, args.seed)
        log(f"api: {api}")

    result = None
    if rank == 0:
        total_in = n * world * args.steps
        value = total_in / dt / 1e9
        enc_avg = sum(enc_ns) / max(1, len(enc_ns))
        # read input once + write body once, per launch (a call = launches[0] equal segments)
        algo_bytes = (n + body_len) / launches[0]
        achieved = algo_bytes / (enc_avg * 1e-9) / 1e9 if enc_avg else 0.0
        workload = f"ambc-mixed-v1 {n >> 30} GiB/GPU chunk={args.chunk} {args.mode}"
        pmc = pmc_traffic(workload)
        result = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": workload, "input_bytes_per_gpu": n, "chunk_size": args.chunk,
                       "mode": args.mode, "methods": methods, "seed": args.seed,
                       "ratio": round(body_total / (n * world), 5),
                       "parallelism": f"chunk-shard dp{world}" if world > 1 else "single GPU",
                       "round_trip_bit_exact": verified, "decode": decode,
                       "reassembly_to_rank0": reasm,
                       "step_ms_p50": round(percentile(step_s, 50) * 1e3, 3),
                       "step_ms_p90": round(percentile(step_s, 90) * 1e3, 3),
                       "e2e_pinned_host": e2e, "api_file": api, "alt_method_set": alt},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                         "kernel": "k_encode", "kernel_ms": round(enc_avg * 1e-6, 3),
                         "algorithmic_bytes_per_launch": round(algo_bytes),
                         "launches_per_step": launches[0]},
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
            result["cpu_baseline"] = cpu_baseline(args, threads)
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
