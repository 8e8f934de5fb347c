"""Step-by-step GPU bring-up probe: each C-ABI path on a tiny input, printing
(and flushing) before and after every call so a hang is pinned to one step."""
import ctypes as C
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd")]

from ambc import _lib  # noqa: E402
from ambc.compressor import entropy_terms  # noqa: E402
from ambc.registry import METHOD_CHUNK_PREFS  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def say(*a):
    print(f"[{time.time():.2f}]", *a, flush=True)


def analyze(ctx, data, chunk, mask, flags_force=False):
    n = len(data)
    M = (n + chunk - 1) // chunk
    p = _lib.Params()
    p.chunk_size = chunk
    p.method_mask = mask
    for i in range(16):
        lo, hi = METHOD_CHUNK_PREFS.get(i, (1, 0))
        p.pref_min[i], p.pref_max[i] = lo, hi
    tf = entropy_terms(chunk)
    p.ent_full = tf.ctypes.data
    ids = (C.c_uint8 * M)()
    pl = (C.c_uint32 * M)()
    su = (C.c_uint8 * M)()
    rc = ctx.lib.ambc_analyze(ctx.h, _lib.addr(data), n, C.byref(p), C.addressof(ids),
                              C.addressof(pl), C.addressof(su))
    return rc, list(ids), list(pl), list(su)


def main():
    which = sys.argv[1:] or ["all"]
    say("load")
    lib = _lib.load()
    n = C.c_int()
    say("device_count rc", lib.ambc_device_count(C.byref(n)), n.value)
    ctx = _lib.Context()
    say("ctx ok")
    mixed = orc.synth(1 << 18, 20250418)
    cases = {"zeros": bytes(4096), "ascii": mixed[70000 - 2000:70000 + 2096],
             "random": mixed[40000:44096], "mixed64": mixed[:65536]}
    for name, d in (cases.items() if "skip" not in which else []):
        for mname, mask in (("rle", 1 << 1), ("huff", 1 << 3), ("lz4", 1 << 9),
                            ("all", (1 << 1) | (1 << 3) | (1 << 4) | (1 << 9))):
            if "all" not in which and mname not in which:
                continue
            say("analyze", name, mname, "...")
            rc, ids, pl, su = analyze(ctx, d, 4096, mask)
            p = orc.make_params(4096, "native", [m for m in (1, 3, 4, 9) if mask >> m & 1],
                                n_total=len(d))
            oids, opl = orc.decide_all(d, p)
            say("   rc", rc, "ids", ids[:8], "pl", pl[:8], "oracle", oids[:8], opl[:8],
                "OK" if (ids, pl) == (oids, opl) else "MISMATCH")
    say("compress_batch 256 KiB ...")
    from ambc import AdaptiveCompressor
    comp = AdaptiveCompressor(chunk_size=4096)
    body = comp._adaptive_compress(mixed)
    ref, _ = orc.compress_body(mixed, orc.make_params(4096, "native", (1, 3, 4, 9),
                                                      n_total=len(mixed)))
    say("   body", len(body), "oracle", len(ref), "equal", body == ref)
    say("decompress ...")
    back = comp._adaptive_decompress(body, len(mixed))
    say("   roundtrip", back == mixed)


if __name__ == "__main__":
    main()
