"""Repeat the bench's decode leg (AdaptiveCompressor._adaptive_decompress of a
device-compressed 4 GiB body) to see its spread:
python scripts/decode_leg.py [reps] [--methods 1,3,4]"""
import ctypes as C
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd")]
from ambc import AdaptiveCompressor, _lib  # noqa: E402

n = 4 << 30
args = [a for a in sys.argv[1:]]
methods = (1, 3, 4, 9)
if "--methods" in args:
    i = args.index("--methods")
    methods = tuple(int(x) for x in args[i + 1].split(","))
    del args[i:i + 2]
reps = int(args[0]) if args else 3
lib = _lib.load()
data = np.empty(n, dtype=np.uint8)
lib.ambc_synth_fill(data.ctypes.data_as(C.POINTER(C.c_uint8)), n, 20250418)
raw = data.tobytes()
del data
comp = AdaptiveCompressor(chunk_size=4096, methods=methods)
body = comp._adaptive_compress(raw)
for _ in range(reps):
    t = time.perf_counter()
    out = comp._adaptive_decompress(body, n)
    dt = time.perf_counter() - t
    ds = comp._last_device_stats
    print(f"decode {n / dt / 1e9:.2f} GB/s  walk {ds.walk_ns / 1e6:.1f} h2d {ds.h2d_ns / 1e6:.1f} "
          f"kern {ds.kernel_ns / 1e6:.1f} d2h {ds.d2h_ns / 1e6:.1f} total {dt * 1e3:.1f} ms ok={out == raw}",
          flush=True)
    del out
