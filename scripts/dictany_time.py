"""Time DictionaryCompression(window, lookahead).compress on the k_da_* path
(the plugin outside k_dict's domain) on synthetic mixed bytes; check the
body's round trip through the GPU decoder.  One JSON line per case."""
import json
import sys
import time

import random

sys.path.insert(0, "adaptive-compression_amd")
from ambc.methods import DictionaryCompression  # noqa: E402


def _mixed(n, seed):
    """runs, words and random bytes (tests/test_gpu_dictany.py's generator)"""
    rnd = random.Random(seed)
    words = [b"compress", b"the ", b"adaptive", b"chunk ", b"window", b"of ", b"GPU", b"\n"]
    out = bytearray()
    while len(out) < n:
        r = rnd.random()
        if r < 0.45:
            out += b"".join(rnd.choice(words) for _ in range(rnd.randrange(5, 80)))
        elif r < 0.7:
            out += bytes([rnd.randrange(256)]) * rnd.randrange(3, 700)
        else:
            out += rnd.randbytes(rnd.randrange(10, 400))
    return bytes(out[:n])

for n, w, lk in ((64 << 20, 4096, 32), (16 << 20, 32768, 32), (16 << 20, 4096, 255)):
    d = _mixed(n, 11)
    m = DictionaryCompression(window_size=w, lookahead_size=lk)
    m.compress(d[:1 << 20])
    t = time.perf_counter()
    enc = m.compress(d)
    dt = time.perf_counter() - t
    ok = DictionaryCompression().decompress(enc, n) == d
    print(json.dumps({"bytes": n, "window": w, "lookahead": lk, "seconds": round(dt, 4),
                      "MBps": round(n / dt / 1e6, 1), "ratio": round(len(enc) / n, 4),
                      "round_trip": ok}), flush=True)
