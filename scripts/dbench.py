"""k_decode cost per input class: compress each class (scripts/kbench.py's
inputs) with the GPU, then decode it through ambc_decompress_ex and report the
kernel / header-walk / copy times.

    python scripts/dbench.py [--size BYTES] [--chunk C] [--reps R]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd"), os.path.join(REPO, "scripts")]

from kbench import make_inputs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256 << 20)
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--methods", default="1,3,4,9")
    args = ap.parse_args()
    from ambc import AdaptiveCompressor
    comp = AdaptiveCompressor(chunk_size=args.chunk, methods=[int(x) for x in args.methods.split(",")])
    for name, a in make_inputs(args.size).items():
        data = a.tobytes()
        body = comp._adaptive_compress(data)
        usage = {k: v for k, v in comp.chunk_stats["method_usage"].items() if v}
        best = None
        for _ in range(args.reps):
            back = comp._adaptive_decompress(body, len(data))
            ds = comp._last_device_stats
            t = (ds.kernel_ns, ds.walk_ns, ds.h2d_ns, ds.d2h_ns)
            best = t if best is None or t[0] < best[0] else best
        assert back == data, name
        print(json.dumps({"class": name, "usage": usage, "ratio": round(len(body) / len(data), 4),
                          "kernel_ms": best[0] / 1e6, "walk_ms": best[1] / 1e6,
                          "h2d_ms": best[2] / 1e6, "d2h_ms": best[3] / 1e6,
                          "kernel_GBps": round(len(data) / best[0], 2)}), flush=True)


if __name__ == "__main__":
    main()
