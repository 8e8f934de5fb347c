"""k_encode cost breakdown: device time per input class x method set.

    python scripts/kbench.py [--size BYTES] [--chunk C]

Input classes are built from the "ambc-mixed v1" generator's segments: all
zero-run, all random, all ASCII, and the mixed stream itself."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd")]

from ambc import _lib  # noqa: E402
from ambc.compressor import entropy_terms  # noqa: E402
from ambc.registry import METHOD_CHUNK_PREFS, method_mask  # noqa: E402


def make_inputs(n, seed=20250418):
    from oracle import synth
    big = np.frombuffer(synth.generate(min(3 * n, 1 << 30) + (1 << 20), seed), dtype=np.uint8)
    cls = {0: [], 1: [], 2: []}
    for pos, L, typ, _ in synth.segments(len(big), seed):
        cls[typ].append(big[pos:pos + L])
    out = {}
    for typ, name in ((0, "zero"), (1, "random"), (2, "ascii")):
        a = np.concatenate(cls[typ])
        reps = -(-n // len(a))
        out[name] = np.ascontiguousarray(np.tile(a, reps)[:n])
    out["mixed"] = np.ascontiguousarray(big[:n])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256 << 20)
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--inputs", default="zero,random,ascii,mixed")
    ap.add_argument("--flags", type=int, default=0, help="ambc_params.flags (2 = AMBC_FLAG_ZLIB9)")
    ap.add_argument("--msets", default="-;1;3;9;1,3,4,9",
                    help="method sets, ';'-separated ('-' = none)")
    args = ap.parse_args()
    ctx = _lib.Context()
    lib = ctx.lib
    n = args.size
    d_in = lib.ambc_device_alloc(ctx.h, 0, n + 64)   # + the slack AMBC_FLAG_INPUT_PADDED promises
    cap = lib.ambc_compress_bound(n, args.chunk)
    d_out = lib.ambc_device_alloc(ctx.h, 0, cap)
    tab = entropy_terms(args.chunk)
    res = []
    inputs = make_inputs(n)
    for name, arr in inputs.items():
        if name not in args.inputs.split(","):
            continue
        _lib.check(lib.ambc_memcpy_h2d(ctx.h, 0, d_in, arr.ctypes.data, n), lib)
        msets = [() if m == "-" else tuple(int(x) for x in m.split(",")) for m in args.msets.split(";")]
        for mset in msets:
            p = _lib.Params()
            p.chunk_size = args.chunk
            p.flags = args.flags | _lib.FLAG_INPUT_PADDED
            p.method_mask = method_mask(mset)
            for i in range(16):
                lo, hi = METHOD_CHUNK_PREFS.get(i, (1, 0))
                p.pref_min[i], p.pref_max[i] = lo, hi
            p.ent_full = tab.ctypes.data
            olen = C.c_uint64()
            st = _lib.Stats()
            ts = []
            for _ in range(args.reps):
                _lib.check(lib.ambc_compress_device(ctx.h, 0, d_in, n, C.byref(p), d_out, cap,
                                                    C.byref(olen), C.byref(st), None), lib)
                e = C.c_uint64()
                lib.ambc_last_kernel_times(ctx.h, 0, C.byref(e), None, None)
                ts.append(e.value / 1e6)
            ms = min(ts)
            r = {"input": name, "methods": list(mset), "encode_ms": round(ms, 3),
                 "GBps": round(n / ms / 1e6, 1), "ratio": round(olen.value / n, 4),
                 "usage": {k: int(st.method_usage[k]) for k in (1, 2, 3, 5, 9) if st.method_usage[k]}}
            res.append(r)
            print(json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    lib.ambc_device_free(ctx.h, 0, d_in)
    lib.ambc_device_free(ctx.h, 0, d_out)


if __name__ == "__main__":
    t = time.time()
    main()
    print("elapsed", time.time() - t, file=sys.stderr)
