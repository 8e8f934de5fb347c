"""Debug: per-lane segments of k_decode_huff for one failing payload (AMBC_HUFF_DEBUG)."""
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd"), "/tmp"]
from ambc import AdaptiveCompressor  # noqa: E402
from oracle import oracle as orc  # noqa: E402

rng = np.random.default_rng(61)
words = [b"alpha", b"beta", b"gamma", b"delta", b"eps", b"zeta", b"eta", b"theta"]
comp = AdaptiveCompressor()
for n in (1000, 4096, 6000):
    text = b" ".join(words[i] for i in rng.integers(0, len(words), n // 4))[:n]
    if n != 6000:
        continue
    p = orc.huff_encode(text)
    o = 2000
    body = b"\xff\xff\x00\x00" + bytes((3, 0)) + struct.pack("<III", o, o, len(p)) + p
    want = orc.decompress_body(body, o)
    os.environ["AMBC_HUFF_DEBUG"] = "1"
    got = comp._adaptive_decompress(body, o)
    bad = next((i for i in range(len(want)) if got[i] != want[i]), -1)
    print(f"n={n} plen={len(p)} orig={o}: first mismatch {bad}", flush=True)
    print("want", want[:40])
    print("got ", got[:40])
    open(os.path.join(REPO, "gpurun_out/r6hd/payload.bin"), "wb").write(p)
