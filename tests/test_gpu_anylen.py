"""The single-call plugins past one 64 KiB chunk (ambc_encode_any /
ambc_analyze_any, ambc_anylen.hip) against the oracle: RLE
(compression_methods.py:78-113), Huffman (:358-405), Delta (:586-607), LZ4
(advanced_compression.py:266-281: one frame of independent 64 KiB blocks), and
should_use of RLE / Huffman / Delta / Dictionary (:154-180, 540-574, 640-667,
315-343) at any length.

Covers: runs longer than 255 and across the 4 KiB blocks' edges, runs of 255 /
256 / 510 bytes, the Huffman table in first-occurrence order and codes longer
than 32 bits (Fibonacci counts), the reference's errors (one or 256 distinct
bytes), the any-length kernels agreeing with the single-chunk ones up to 64 KiB,
and round trips through the GPU decoders."""
import random

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(hip_lib):
    from ambc import _lib
    return _lib.default_context()


def _runs(n, seed):
    """runs of every length around the 255 split and the 4 KiB block edges"""
    rnd = random.Random(seed)
    out = bytearray()
    lens = [1, 2, 254, 255, 256, 509, 510, 511, 4095, 4096, 4097, 9000, 70000]
    while len(out) < n:
        out += bytes([rnd.randrange(4)]) * rnd.choice(lens + [rnd.randrange(1, 600)])
    return bytes(out[:n])


def _mixed(n, seed):
    rnd = random.Random(seed)
    words = [b"plugin ", b"length ", b"any ", b"chunk ", b"the ", b"\n"]
    out = bytearray()
    while len(out) < n:
        r = rnd.random()
        if r < 0.4:
            out += b"".join(rnd.choice(words) for _ in range(rnd.randrange(5, 60)))
        elif r < 0.7:
            out += bytes([rnd.randrange(256)]) * rnd.randrange(3, 900)
        else:
            out += rnd.randbytes(rnd.randrange(10, 500))
    return bytes(out[:n])


def _fib_data(nsym, seed):
    f = [1, 1]
    while len(f) < nsym:
        f.append(f[-1] + f[-2])
    d = np.concatenate([np.full(c, 40 + i, dtype=np.uint8) for i, c in enumerate(f)])
    return bytes(np.random.default_rng(seed).permutation(d))


def _plugins():
    from ambc.methods import DeltaCompression, HuffmanCompression, LZ4Compression, RLECompression
    return {1: RLECompression(), 3: HuffmanCompression(), 4: DeltaCompression(), 9: LZ4Compression()}


def _oracle(mid, d):
    if mid == 1:
        return orc.rle_encode(d)
    if mid == 3:
        return orc.huff_encode(d)
    if mid == 4:
        a = np.frombuffer(d, np.uint8)
        return bytes(np.concatenate([a[:1], (a[1:] - a[:-1]).astype(np.uint8)]))
    return orc.lz4_frame_encode(d)


def test_encoders_past_one_chunk(ctx):
    pl = _plugins()
    datas = [_runs(65537, 1), _runs(300000, 2), _mixed(65537 + 4096 * 3 + 5, 3), _mixed(1 << 20, 4),
             random.Random(5).randbytes(200000), bytes(140000) + b"\x01", _fib_data(27, 6)]
    for d in datas:
        for mid, m in pl.items():
            want = _oracle(mid, d)
            if want is None:                                  # Huffman on 256 distinct bytes raises
                with pytest.raises(ValueError):
                    m.compress(d)
                continue
            got = m.compress(d)
            assert got == want, (mid, len(d))
            if mid != 4 or len(d) <= (1 << 20):
                assert m.decompress(got, len(d)) == d, (mid, len(d))


def test_huffman_long_codes_and_errors(ctx):
    from ambc.methods import HuffmanCompression
    m = HuffmanCompression()
    d = _fib_data(35, 7)          # 24 M bytes: codes of 33 and 34 bits
    assert len(d) > (1 << 24)
    assert m.compress(d) == orc.huff_encode(d)
    with pytest.raises(ValueError):
        m.compress(bytes(100000))                           # one distinct byte
    with pytest.raises(ValueError):
        m.compress(bytes(range(256)) * 400)                 # 256 distinct bytes


def test_any_length_kernels_agree_within_one_chunk(ctx):
    from ambc.methods import _gpu_encode, _gpu_encode_any
    for n, seed in ((1, 1), (2, 2), (13, 3), (1000, 4), (4096, 5), (65535, 6), (65536, 7)):
        for d in (_mixed(n, seed), _runs(n, seed)):
            for mid in (1, 3, 4, 9):
                if mid == 3 and not 2 <= len(set(d)) <= 255:
                    continue
                assert _gpu_encode_any(mid, d) == _gpu_encode(mid, d) == _oracle(mid, d), (mid, n)


def test_should_use_past_one_chunk(ctx):
    pl = _plugins()
    from ambc.methods import DictionaryCompression
    dm = DictionaryCompression()
    rng = np.random.default_rng(8)
    datas = [_runs(70000, 9), _mixed(300000, 10), random.Random(11).randbytes(100000),
             bytes(rng.integers(0, 128, 128 * 1024, dtype=np.uint8)),        # entropy near 7.0
             bytes(np.repeat(np.arange(128, dtype=np.uint8), 1024)),          # exactly 7.0: not < 7.0
             bytes(rng.integers(0, 40, 99999, dtype=np.uint8)),
             bytes((np.arange(200000) // 3 % 7 * 9).astype(np.uint8))]
    for d in datas:
        for mid in (1, 3, 4):
            tab = orc.entropy_table(len(d)) if mid == 3 else None
            assert pl[mid].should_use(d) == orc.should_use(mid, d, tab), (mid, len(d))
        assert dm.should_use(d) == orc.should_use(2, d), len(d)
