"""Time the single-call plugins past the batched kernels' domain: Dictionary
(window, lookahead) on k_da_*, RLE / Huffman / Delta / LZ4 on ambc_encode_any
(64 MiB of synthetic mixed bytes; each body round-trips through the GPU
decoder).  One JSON line per case.  Times include the host-device copies."""
import json
import sys
import time

import random

sys.path.insert(0, "adaptive-compression_amd")
from ambc.methods import (DeltaCompression, DictionaryCompression, HuffmanCompression,  # noqa: E402
                          LZ4Compression, RLECompression)


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

# the other plugins past one chunk (ambc_encode_any)
d = _mixed(64 << 20, 12)
d = bytes(b if b < 250 else 32 for b in d[:1 << 20]) * 64      # <= 250 distinct bytes: Huffman encodes
for name, m in (("rle", RLECompression()), ("huffman", HuffmanCompression()), ("delta", DeltaCompression()),
                ("lz4", LZ4Compression())):
    m.compress(d[:1 << 20])
    t = time.perf_counter()
    enc = m.compress(d)
    dt = time.perf_counter() - t
    t = time.perf_counter()
    su = m.should_use(d)
    ds = time.perf_counter() - t
    ok = m.decompress(enc, len(d)) == d
    print(json.dumps({"plugin": name, "bytes": len(d), "seconds": round(dt, 4), "MBps": round(len(d) / dt / 1e6, 1),
                      "ratio": round(len(enc) / len(d), 4), "should_use": su, "should_use_seconds": round(ds, 4),
                      "round_trip": ok}), flush=True)
