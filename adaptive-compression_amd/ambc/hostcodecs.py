"""Host-scored methods of the multi-size walk: the reference's library codecs
that have no GPU encoder -- BZIP2 (id 6), LZMA (id 7) and ZStandard (id 8),
advanced_compression.py:112-261 -- evaluated on host threads beside the device's
encoders.

ambc_compress_multisize_ex calls ``eval`` once per walk round with the (position,
size) pairs the round evaluates (while the device encodes the same pairs) and
``emit`` once per package of the final body that a host codec won.  Per pair the
answer is the reference's per-size method loop restricted to these codecs
(adaptive_compressor.py:559-579): prefs range, ``should_use``, ``compress``, the
strict minimum of len + 18 below the chunk's own length, ids ascending; the
library then joins it with the GPU's winner in id order.  bz2 / lzma release the
GIL while they compress, so a thread pool runs the pairs in parallel.

Each round's (pair, codec) evaluations go to the pool as separate tasks, the
costliest first (LZMA, then bz2, larger chunks first), so that a round's host
time is about max(largest task, total / threads) rather than a pair's serial
sum; the pair's answer is then joined in id order exactly as the loop would.

Memory: an LZMA encoder with the reference's 16 MiB dictionary holds about
190 MiB of state; methods.py keeps as many as its memory budget allows (a
quarter of the host's memory, at most 8 GiB: 32 on a large host) and a call
waits for a free one, so the rest of the pool keeps bz2 / zstd busy meanwhile;
close() ends the idle encoders, so nothing stays resident after the walk.
"""
import ctypes as C
import os
from concurrent.futures import ThreadPoolExecutor

EVAL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_uint32,
                      C.POINTER(C.c_uint8), C.POINTER(C.c_uint32))
EMIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint8, C.POINTER(C.c_uint8), C.c_uint32)


class HostCodecs(C.Structure):
    """ambc_host_codecs (include/ambc.h)"""
    _fields_ = [("eval", EVAL_FN), ("emit", EMIT_FN), ("user", C.c_void_p)]


class HostScorer:
    """One walk's host codecs over ``data`` (bytes); ``methods``: CompressionMethod
    instances of the host-scored ids; ``prefs``: method_chunk_prefs."""

    CACHE_BYTES = 256 << 20          # payloads kept from eval for emit (beyond: recomputed)

    def __init__(self, data, methods, prefs, workers=None):
        self.data = data
        self.methods = sorted(methods, key=lambda m: m.type_id)
        self.prefs = prefs
        self.cache = {}
        self.cached = 0
        self.error = None
        env = os.environ.get("AMBC_HOST_CODEC_THREADS")
        self.pool = ThreadPoolExecutor(workers or (int(env) if env else min(32, os.cpu_count() or 4)))
        # the callbacks must outlive the call: keep them on the instance
        self._eval_cb = EVAL_FN(self._eval)
        self._emit_cb = EMIT_FN(self._emit)
        self.struct = HostCodecs(self._eval_cb, self._emit_cb, None)

    def close(self):
        self.pool.shutdown(wait=True)
        self.cache.clear()
        from .methods import _XZEncoders
        _XZEncoders.release()

    def _eligible(self, m, size):
        lo, hi = self.prefs.get(m.type_id, (1, 999999999))
        return lo <= size <= hi

    def _one(self, m, pos, size):
        """method m at data[pos:pos+size]: its payload, or None (should_use false, or it raised)"""
        chunk = self.data[pos:pos + size]
        if not m.should_use(chunk):
            return None
        try:
            return m.compress(chunk)
        except Exception:  # noqa: BLE001 -- the reference's loop skips a raising method
            return None

    def _join(self, size, outs):
        """the reference's per-size loop over the host codecs (adaptive_compressor.py:
        559-579): ids ascending, strict minimum below len + 18 < size"""
        win, wl, pay = 0, size - 18, None
        for m in self.methods:
            c = outs.get(m.type_id)
            if c is not None and len(c) < wl:
                win, wl, pay = m.type_id, len(c), c
        return win, pay

    def best(self, pos, size):
        """(id, payload) of the host codecs' winner at data[pos:pos+size], or (0, None)."""
        outs = {m.type_id: self._one(m, pos, size) for m in self.methods if self._eligible(m, size)}
        return self._join(size, outs)

    @staticmethod
    def _cost(m, size):
        return (0 if m.type_id == 7 else 1 if m.type_id == 6 else 2, -size)

    def _eval(self, _user, pos, size, count, out_id, out_len):
        try:
            pairs = [(int(pos[i]), int(size[i])) for i in range(count)]
            tasks = [(i, m) for i, (_p, sz) in enumerate(pairs) for m in self.methods if self._eligible(m, sz)]
            tasks.sort(key=lambda t: self._cost(t[1], pairs[t[0]][1]))
            futs = [(i, m.type_id, self.pool.submit(self._one, m, *pairs[i])) for i, m in tasks]
            outs = [dict() for _ in pairs]
            for i, mid, f in futs:
                outs[i][mid] = f.result()
            for i, (_p, sz) in enumerate(pairs):
                w, pay = self._join(sz, outs[i])
                out_id[i] = w
                out_len[i] = len(pay) if w else 0
                if w and self.cached + len(pay) <= self.CACHE_BYTES:
                    self.cache[pairs[i]] = (w, pay)
                    self.cached += len(pay)
            return 0
        except BaseException as e:  # noqa: BLE001 -- must not unwind through C
            self.error = e
            return 1

    def _emit(self, _user, pos, size, mid, dst, length):
        try:
            got = self.cache.get((int(pos), int(size)))
            if got is None:
                got = self.best(int(pos), int(size))
            w, pay = got
            if w != mid or pay is None or len(pay) != length:
                raise RuntimeError(f"host codec re-encode differs at {pos}+{size}: id {w} vs {mid}")
            C.memmove(dst, pay, length)
            return 0
        except BaseException as e:  # noqa: BLE001
            self.error = e
            return 1
