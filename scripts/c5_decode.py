"""decode-only path.

A 4 GiB "ambc-mixed v1" stream is compressed on the host by the CPU restatement
(oracle/ambc_oracle.c, OpenMP, native mode, methods {1, 3, 5, 255}: RLE,
Huffman, zlib-9 DEFLATE, raw -- byte-identical to the reference on the golden
files), then decoded through the library (GPU kernels for ids 1/3/255 and the
GPU inflate for id 5) and compared bit-exactly with the input.

    python scripts/c5_decode.py [--size BYTES] [--chunk C] [--reps R]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        scripts/c5_decode.py ...          # decode at N GPUs; no torch is imported

Measurement harness, not product: the oracle only PRODUCES the C5 input body
(the config asks for an .ambc written by the CPU reference); what is timed is
the library's decode.

With N ranks (one per GPU, RCCL), rank 0 produces the body once and shares it
through a file; every rank cuts the body at package boundaries
(ambc_split_body), decodes its range into device memory and the ranges are
gathered on rank 0 in file order over xGMI.  Timed: split + walk + H2D +
kernels + gather, max over ranks.  Prints one JSON line (rank 0).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd")]


def distributed(args):
    """N ranks, one per GPU, torch-free: ambc.comm.GpuGroup (RCCL) +
    ambc_decompress_shard (split, per-rank decode into HBM, grouped send/recv
    gather onto rank 0)."""
    import tempfile

    from ambc import _lib
    from ambc.comm import GpuGroup
    from ambc.distributed import decompress_shard
    from oracle import oracle as orc

    g = GpuGroup()
    rank, world = g.rank, g.world
    n = args.size
    lib = g.lib
    path = os.path.join(tempfile.gettempdir(), f"c5_body_{os.environ.get('MASTER_PORT', '0')}.bin")
    info = {}
    if rank == 0:
        data = np.empty(n, dtype=np.uint8)
        lib.ambc_synth_fill(data.ctypes.data_as(C.POINTER(C.c_uint8)), n, args.seed)
        raw = data.tobytes()
        del data
        t = time.perf_counter()
        body, st = orc.compress_body(raw, orc.make_params(args.chunk, "native", (1, 3, 5), n_total=n),
                                     nthreads=args.threads)
        info = {"t_cpu": time.perf_counter() - t, "len": len(body),
                "usage": {i: int(st.method_usage[i]) for i in range(256) if st.method_usage[i]}}
        with open(path, "wb") as f:
            f.write(body)
    info = json.loads(g.host.broadcast(json.dumps(info).encode()))
    if rank != 0:
        with open(path, "rb") as f:
            body = f.read()
    d_out = _lib.DeviceBuffer(g.ctx, (n if rank == 0 else n // world + (64 << 20)) + 64)
    best = None
    for _ in range(args.reps):
        g.barrier()
        t = time.perf_counter()
        decompress_shard(g, body, n, d_out, d_out.nbytes, root=0)
        g.barrier()
        dt = max(x[0] for x in g.host.allgather_obj([time.perf_counter() - t]))
        best = dt if best is None else min(best, dt)
    if rank == 0:
        data = np.empty(n, dtype=np.uint8)
        lib.ambc_synth_fill(data.ctypes.data_as(C.POINTER(C.c_uint8)), n, args.seed)
        eq = C.c_int(0)
        ref = _lib.DeviceBuffer(g.ctx, n + 64)
        ref.upload(data)
        _lib.check(lib.ambc_device_equal(g.ctx.h, 0, ref.ptr, d_out.ptr, n, C.byref(eq)), lib)
        ok = bool(eq.value)
        ref.free()
        os.unlink(path)
        print(json.dumps({
            "config": "C5 decode-only", "n_gpus": world, "input_bytes": n, "chunk_size": args.chunk,
            "body_bytes": info["len"], "ratio": round(info["len"] / n, 5),
            "method_usage": info["usage"],
            "producer": f"oracle/ambc_oracle.c OpenMP ({args.threads} threads), {info['t_cpu']:.1f} s",
            "decode_GBps": round(n / best / 1e9, 3), "decode_ms": round(best * 1e3, 1),
            "timed": "split + per-rank header walk + H2D + kernels + RCCL file-order gather on rank 0 "
                     "(device-resident output), max over ranks",
            "bit_exact": ok}), flush=True)
    d_out.free()
    g.barrier()
    g.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4 << 30)
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=20250418)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return distributed(args)
    from ambc import AdaptiveCompressor, _lib
    from oracle import oracle as orc
    n = args.size
    lib = _lib.load()
    data = np.empty(n, dtype=np.uint8)
    lib.ambc_synth_fill(data.ctypes.data_as(C.POINTER(C.c_uint8)), n, args.seed)
    raw = data.tobytes()
    del data
    p = orc.make_params(args.chunk, "native", (1, 3, 5), n_total=n)
    t = time.perf_counter()
    body, st = orc.compress_body(raw, p, nthreads=args.threads)
    t_cpu = time.perf_counter() - t
    usage = {i: int(st.method_usage[i]) for i in range(256) if st.method_usage[i]}
    print(f"oracle body {len(body)} B in {t_cpu:.1f} s, usage {usage}", file=sys.stderr, flush=True)
    comp = AdaptiveCompressor(chunk_size=args.chunk, methods=(1, 3, 4, 9))
    best = None
    out = None
    for _ in range(args.reps):
        out = None                      # free the previous output outside the timed call
        t = time.perf_counter()
        out = comp._adaptive_decompress(body, n)
        dt = time.perf_counter() - t
        ds = comp._last_device_stats
        rec = (dt, ds.kernel_ns, ds.walk_ns, ds.h2d_ns, ds.d2h_ns, ds.host_codec_ns)
        best = rec if best is None or dt < best[0] else best
    ok = out == raw
    dt, kern, walk, h2d, d2h, hostc = best
    print(json.dumps({
        "config": "C5 decode-only", "input_bytes": n, "chunk_size": args.chunk,
        "body_bytes": len(body), "ratio": round(len(body) / n, 5), "method_usage": usage,
        "producer": f"oracle/ambc_oracle.c OpenMP ({args.threads} threads), {t_cpu:.1f} s",
        "decode_GBps": round(n / dt / 1e9, 3), "decode_ms": round(dt * 1e3, 1),
        "kernel_ms": round(kern / 1e6, 3), "header_walk_ms": round(walk / 1e6, 3),
        "h2d_ms": round(h2d / 1e6, 3), "d2h_ms": round(d2h / 1e6, 3),
        "host_zlib_ms": round(hostc / 1e6, 3), "host_zlib_threads": int(os.environ.get(
            "AMBC_HOST_THREADS", min(16, os.cpu_count() or 1))),
        "bit_exact": ok}), flush=True)


if __name__ == "__main__":
    main()
