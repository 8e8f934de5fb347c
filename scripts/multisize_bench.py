"""Time the reference's multi-size walk (REFERENCE_CHUNK_SIZE_CANDIDATES) on the
GPU (ambc_compress_multisize) and check the body against the oracle's walk.

    python scripts/multisize_bench.py [MiB ...]      (default: 32 256)
    MS_SETS="mixed:1,3,4,5;mixed:1,2,3,4,5,9" python scripts/multisize_bench.py 32
    MS_MODE=reference ...   (id 5 as zlib-9's bytes: AdaptiveCompressor.like_reference()'s walk)

Input: runs, text-like bytes and skewed random bytes in 8-64 KiB segments, so
every position compresses and the walk never ends in the remainder-raw rule."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "adaptive-compression_amd"))
import numpy as np  # noqa: E402
import ambc  # noqa: E402


def mixed(n, seed):
    rng = np.random.default_rng(seed)
    out, have = [], 0
    while have < n:
        m = int(rng.integers(8, 65)) << 10
        kind = int(rng.integers(3))
        if kind == 0:
            seg = np.repeat(rng.integers(0, 256, m // 256 + 1, dtype=np.uint8), 256)[:m]
        elif kind == 1:
            seg = rng.choice(np.frombuffer(b"etaoin shrdlu,.ETAOIN", np.uint8), m)
        else:
            seg = np.minimum(rng.geometric(0.08, m), 255).astype(np.uint8)
        out.append(seg.tobytes())
        have += m
    return b"".join(out)[:n]


def text(n, seed):
    """homogeneous text: the largest size wins almost everywhere"""
    rng = np.random.default_rng(seed)
    return rng.choice(np.frombuffer(b"etaoin shrdlu,.ETAOIN", np.uint8), n).tobytes()


def main():
    sizes = [float(x) for x in sys.argv[1:]] or [32, 256]
    sets = (("mixed", (1, 3, 4, 9)), ("mixed", (1, 2, 3, 4)), ("text", (1, 3, 4, 9)))
    if os.environ.get("MS_SETS"):
        sets = [(k, tuple(int(x) for x in m.split(","))) for k, m in
                (e.split(":") for e in os.environ["MS_SETS"].split(";"))]
    for kind, methods in sets:
        for mib in sizes:
            data = (mixed if kind == "mixed" else text)(int(mib * (1 << 20)), 7)
            comp = ambc.AdaptiveCompressor(methods=methods, mode=os.environ.get("MS_MODE", "native"))
            comp.CHUNK_SIZE_CANDIDATES = list(comp.REFERENCE_CHUNK_SIZE_CANDIDATES)
            comp._adaptive_compress(data[:1 << 20])            # warm
            t = time.perf_counter()
            body = comp._adaptive_compress(data)
            dt = time.perf_counter() - t
            steps, ev, wns, ens = C.c_uint32(), C.c_uint64(), C.c_uint64(), C.c_uint64()
            lib = ambc._lib.load()
            lib.ambc_last_multisize_info(ambc._lib.default_context().h, C.byref(steps), C.byref(ev), C.byref(wns),
                                         C.byref(ens))
            rec = {"input": kind, "MiB": mib, "methods": list(methods), "deflate": comp.deflate,
                   "seconds": round(dt, 4),
                   "GBps": round(len(data) / dt / 1e9, 3), "ratio": round(len(body) / len(data), 5),
                   "chunks": comp.chunk_stats["total_chunks"], "walk_steps": steps.value,
                   "chunk_encodes": ev.value, "walk_ms": round(wns.value / 1e6, 2),
                   "final_encode_ms": round(ens.value / 1e6, 2)}
            if mib <= 32:
                from oracle import oracle as orc
                t = time.perf_counter()
                ref, _ = orc.compress_body_multisize(data, comp.CHUNK_SIZE_CANDIDATES, tuple(methods) + (255,),
                                                     deflate="zlib" if comp.deflate == "zlib9" else "gd")
                rec["oracle_seconds"] = round(time.perf_counter() - t, 2)
                rec["body_equals_oracle"] = ref == body
            rec["round_trip"] = comp._adaptive_decompress(body, len(data)) == data
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
