"""Phase cycles of the zlib-9 parse (AMBC_STAMPS build) on the multi-size walk's
mixed input and the synthetic classes, per chunk size: native mode, methods {5}
with id 5 as zlib-9's bytes.
    AMBC_STAMPS=1 AMBC_LIB=adaptive-compression_amd/ambc/libambc_hip_stamps.so python scripts/z9_stamps_ms.py"""
import ctypes as C
import os
import sys
import time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd"), os.path.join(REPO, "scripts")]
from ambc import _lib  # noqa: E402
from ambc.compressor import entropy_terms  # noqa: E402
from ambc.registry import METHOD_CHUNK_PREFS, method_mask  # noqa: E402
from multisize_bench import mixed  # noqa: E402
import kbench  # noqa: E402

ctx = _lib.Context()
lib = ctx.lib
n = int(os.environ.get("Z9_BYTES", 32 << 20))
inputs = {"ms_mixed": mixed(n, 7)}
for k, v in kbench.make_inputs(n).items():
    if k in ("ascii", "mixed"):
        inputs["synth_" + k] = v.tobytes()
d_in = lib.ambc_device_alloc(ctx.h, 0, n + 64)
for C_ in [int(x) for x in os.environ.get("Z9_CHUNKS", "4096,16384,65536").split(",")]:
    cap = lib.ambc_compress_bound(n, C_)
    d_out = lib.ambc_device_alloc(ctx.h, 0, cap)
    tab = entropy_terms(C_)
    for name, data in inputs.items():
        _lib.check(lib.ambc_memcpy_h2d(ctx.h, 0, d_in, _lib.addr(data), n), lib)
        p = _lib.Params()
        p.chunk_size = C_
        p.flags = _lib.FLAG_ZLIB9 | _lib.FLAG_INPUT_PADDED
        p.method_mask = method_mask((5,))
        for i in range(16):
            lo, hi = METHOD_CHUNK_PREFS.get(i, (1, 0))
            p.pref_min[i], p.pref_max[i] = lo, hi
        p.ent_full = tab.ctypes.data
        olen, st = C.c_uint64(), _lib.Stats()
        print(f"== {name} chunk {C_}", file=sys.stderr, flush=True)
        t = time.perf_counter()
        _lib.check(lib.ambc_compress_device(ctx.h, 0, d_in, n, C.byref(p), d_out, cap, C.byref(olen),
                                            C.byref(st), None), lib)
        e = C.c_uint64()
        lib.ambc_last_kernel_times(ctx.h, 0, C.byref(e), None, None)
        print(f"{name} chunk {C_}: encode {e.value / 1e6:.2f} ms, ratio {olen.value / n:.4f}", file=sys.stderr, flush=True)
    lib.ambc_device_free(ctx.h, 0, d_out)
