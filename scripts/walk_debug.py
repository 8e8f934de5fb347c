"""Debug aid: one crafted body of tests/test_gpu_walk.py through the device walk
with AMBC_WALK_TRACE (per-piece state on stderr), compared with the oracle."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd"), os.path.join(REPO, "tests")]

from oracle import oracle as orc  # noqa: E402
import test_gpu_walk as tw  # noqa: E402

piece = int(sys.argv[1]) if len(sys.argv) > 1 else 64
nparts = int(sys.argv[2]) if len(sys.argv) > 2 else 60
parts, orig = tw._crafted(np.random.default_rng(piece))
parts = parts[:nparts]
body = b"".join(parts) + tw.END
orig = sum(orc.decompress_body(p + tw.END, 0, return_produced=True)[1] for p in parts)
want = orc.decompress_body(body, orig)
print("body", len(body), "orig", orig, "starts", [sum(len(p) for p in parts[:k]) for k in range(len(parts) + 1)][:12],
      flush=True)
os.environ.update(AMBC_DEVWALK_MIN="0", AMBC_WALK_PIECE=str(piece), AMBC_WALK_TRACE="1")
comp = tw._comp()
try:
    got = comp._adaptive_decompress(body, orig)
    print("equal", got == want, flush=True)
except ValueError as e:
    print("raised", e, flush=True)
