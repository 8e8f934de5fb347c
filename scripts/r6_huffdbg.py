"""Debug: one text payload's Huffman decode on the GPU against the oracle, for
several orig values, through the current routing (AMBC_HUFF_ROUTE as set)."""
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd")]
from ambc import AdaptiveCompressor  # noqa: E402
from oracle import oracle as orc  # noqa: E402

rng = np.random.default_rng(61)
words = [b"alpha", b"beta", b"gamma", b"delta", b"eps", b"zeta", b"eta", b"theta"]
comp = AdaptiveCompressor()
for n in (1000, 4096, 6000, 8192, 12000):
    text = b" ".join(words[i] for i in rng.integers(0, len(words), n // 4))[:n]
    p = orc.huff_encode(text)
    for o in (n, 2000, 3000, 4000, 4096, 1000, 500, 100):
        if o > n:
            continue
        body = b"\xff\xff\x00\x00" + bytes((3, 0)) + struct.pack("<III", o, o, len(p)) + p
        want = orc.decompress_body(body, o)
        got = comp._adaptive_decompress(body, o)
        bad = next((i for i in range(len(want)) if got[i] != want[i]), -1)
        print(f"n={n} plen={len(p)} orig={o}: first mismatch {bad}", flush=True)
