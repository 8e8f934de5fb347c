"""Time the reference's multi-size walk (REFERENCE_CHUNK_SIZE_CANDIDATES) on the
GPU with and without the look-ahead runs, and check both bodies are equal.
Usage: python scripts/multisize_bench.py [MiB]"""
import os, sys, time
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "adaptive-compression_amd"))
import numpy as np  # noqa: E402
import ambc  # noqa: E402


def mixed(n, seed):
    """runs, text-like bytes and skewed random bytes in 8-64 KiB segments: every
    position compresses, so the walk never ends in the remainder-raw rule"""
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
mib = float(sys.argv[1]) if len(sys.argv) > 1 else 4
data = mixed(int(mib * (1 << 20)), 7)
res = {}
for la, rb in ((True, 16 << 20), (True, 4 << 20), (True, 64 << 20), (True, 16 << 20), (False, 0)):
    comp = ambc.AdaptiveCompressor(methods=(1, 3, 4, 9))
    comp.CHUNK_SIZE_CANDIDATES = list(comp.REFERENCE_CHUNK_SIZE_CANDIDATES)
    comp.MULTISIZE_LOOKAHEAD = la
    if rb:
        comp.MULTISIZE_RUN_BYTES = rb
    comp._adaptive_compress(data[:4 << 20])            # warm
    t = time.perf_counter()
    body = comp._adaptive_compress(data)
    dt = time.perf_counter() - t
    res[(la, rb)] = body
    print(f"lookahead={la} run={rb >> 20} MiB {len(data)/2**20:.1f} MiB {dt*1e3:.1f} ms "
          f"{len(data)/dt/1e6:.2f} MB/s ratio {len(body)/len(data):.4f} "
          f"chunks {comp.chunk_stats['total_chunks']}", flush=True)
assert len(set(res.values())) == 1, "look-ahead changed the body"
print("bodies equal")
