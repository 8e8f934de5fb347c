"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

numpy restatement of the "ambc-mixed v1" synthetic mixed-entropy generator
(SURVEY.md §8(d)).  The product ships the same generator in C
(``ambc_synth_fill`` in ``adaptive-compression_amd/csrc/ambc_host.cpp``);
``tests/test_synth.py`` checks the two byte-for-byte.

Spec (all arithmetic mod 2**64):
    GAMMA = 0x9E3779B97F4A7C15
    mix(z)  = splitmix64 finaliser
    seg RNG : s = seed; next() { s += GAMMA; return mix(s) }
    segments: idx = 0, pos = 0; while pos < n:
                  L = min(1024 + next() % 130049, n - pos)     # U[1024, 131072]
                  type = idx % 3  (0 zero-run, 1 uniform random, 2 ASCII words)
                  base = mix(seed ^ (idx * 0xD1B54A32D192ED03))
    zero    : L zero bytes
    random  : little-endian bytes of mix(base + (j+1)*GAMMA), j = 0,1,..; cut to L
    ASCII   : word_j = VOCAB[mix(base + (j+1)*GAMMA) >> 60] + b' '; concat; cut to L
"""
import numpy as np

GAMMA = 0x9E3779B97F4A7C15
SEG_MUL = 0xD1B54A32D192ED03
M64 = (1 << 64) - 1
VOCAB = [b"alpha", b"beta", b"gamma", b"delta", b"the", b"quick", b"brown", b"fox",
         b"jumps", b"over", b"lazy", b"dog", b"data", b"chunk", b"marker", b"stream"]
SEG_MIN, SEG_SPAN = 1024, 130049


def mix_int(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _mix_np(z):
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _stream(base, count):
    j = np.arange(1, count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _mix_np(np.uint64(base) + j * np.uint64(GAMMA))


def segments(n, seed):
    """Yield (pos, length, type, base) for the stream of n bytes."""
    s = seed & M64
    pos = idx = 0
    while pos < n:
        s = (s + GAMMA) & M64
        L = min(SEG_MIN + mix_int(s) % SEG_SPAN, n - pos)
        base = mix_int(seed ^ ((idx * SEG_MUL) & M64))
        yield pos, L, idx % 3, base
        pos += L
        idx += 1


_WORDS = [w + b" " for w in VOCAB]
_WLEN = np.array([len(w) for w in _WORDS], dtype=np.int64)
_WBUF = np.frombuffer(b"".join(_WORDS), dtype=np.uint8)
_WOFF = np.concatenate([[0], np.cumsum(_WLEN)[:-1]]).astype(np.int64)


def generate(n, seed=20250418):
    out = np.zeros(n, dtype=np.uint8)
    for pos, L, typ, base in segments(n, seed):
        if typ == 1:
            words = _stream(base, (L + 7) // 8)
            out[pos:pos + L] = words.view(np.uint8)[:L]
        elif typ == 2:
            cnt = L // 3 + 2          # every word is >= 4 bytes incl. the space
            wid = (_stream(base, cnt) >> np.uint64(60)).astype(np.int64)
            lens = _WLEN[wid]
            ends = np.cumsum(lens)
            k = int(np.searchsorted(ends, L)) + 1   # words needed to reach L
            wid, lens = wid[:k], lens[:k]
            starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
            idx = np.repeat(_WOFF[wid] - starts, lens) + np.arange(int(lens.sum()))
            out[pos:pos + L] = _WBUF[idx[:L]]
    return out.tobytes()


def random_bytes(n, seed):
    """Uniform random bytes (config C1) from the same splitmix64 stream."""
    return _stream(mix_int(seed), (n + 7) // 8).view(np.uint8)[:n].tobytes()
