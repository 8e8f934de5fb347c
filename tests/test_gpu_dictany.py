"""DictionaryCompression(window_size, lookahead_size) for any window, lookahead
and length on the GPU (k_da_*, ambc_dictany.hip, through ambc_dict_encode)
against the oracle's orc_dict_encode_wl (itself checked against a restatement
of compression_methods.py:195-233,279-313 in test_dict_window_oracle.py and
against the golden-pinned orc_dict_encode at the defaults).

Covers: the reference's defaults past k_dict's 8 KiB (block and group
boundaries of the path composition: 8192-position blocks, 64-block groups),
every window / lookahead rule (window <= 0, window past the start, Python's
slice for negative lookaheads, lookahead 0-2), jumps of 255 across block
boundaries, the ValueError of a >255-byte match on the path and none for one
off the path, round trips through the GPU decoder, should_use on large inputs,
and the two kernels agreeing where both apply."""
import random

import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(hip_lib):
    from ambc import _lib
    return _lib.default_context()


def _mixed(n, seed):
    """runs, words and random bytes"""
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


def _periodic(n, period, seed):
    rnd = random.Random(seed)
    unit = rnd.randbytes(period)
    return (unit * (n // period + 1))[:n]


def _enc(d, window, look):
    from ambc.methods import DictionaryCompression
    return DictionaryCompression(window_size=window, lookahead_size=look).compress(d)


def _check(d, window, look, roundtrip=False):
    try:
        want = orc.dict_encode_wl(d, window, look)
    except ValueError:
        with pytest.raises(ValueError):
            _enc(d, window, look)
        return
    got = _enc(d, window, look)
    assert got == want, (len(d), window, look)
    if roundtrip and 0 < look <= 255 and 0 < window <= 65535:
        from ambc.methods import DictionaryCompression
        assert DictionaryCompression().decompress(got, len(d)) == d


def test_defaults_past_the_batched_domain(ctx):
    for n, seed in ((8193, 1), (8192 * 3 - 1, 2), (8192 * 3 + 7, 3), (100003, 4), (262144, 5)):
        d = _mixed(n, seed)
        _check(d, 4096, 32, roundtrip=True)


def test_windows_and_lookaheads(ctx):
    rng = random.Random(21)
    datas = [_mixed(20000, 6), _periodic(12000, 7, 7), bytes(9000), rng.randbytes(10000),
             bytes(rng.choice(b"ab") for _ in range(9000))]
    grid = [(4096, 32), (16, 32), (1, 4), (3, 3), (0, 32), (-5, 32), (100, 0), (100, 2), (100, 255),
            (100, 256), (700, 1000), (1000, 300), (64, -1), (64, -400), (64, -50000), (1 << 40, 40),
            (70000, 16), (65536, 64), (65537, 8)]
    for d in datas:
        for w, lk in grid:
            _check(d, w, lk, roundtrip=True)


def test_jumps_across_block_and_group_boundaries(ctx):
    """lookahead 255 on long runs: 255-byte jumps enter blocks at offsets up to
    254; more than 64 blocks: two group tables"""
    n = 64 * 8192 + 8192 * 3 + 123
    d = bytearray(_mixed(n, 8))
    for b in range(1, n // 8192):
        off = b * 8192 - 200
        d[off:off + 400] = bytes([b & 0xFF]) * 400
    d = bytes(d)
    _check(d, 300, 255, roundtrip=True)
    _check(d[:8192 * 2 + 1], 300, 255)
    _check(bytes(8192 * 5 + 3), 300, 255, roundtrip=True)     # all zeros: literal, then 255-byte matches


def test_off_path_long_match_does_not_raise(ctx):
    from test_dict_window_oracle import off_path_long_match
    d = off_path_long_match(random.Random(9))
    assert _enc(d, 4096, 300) == orc.dict_encode_wl(d, 4096, 300)
    with pytest.raises(ValueError):
        _enc(d[:300] + d[300:330] + d[:300], 4096, 300)
    with pytest.raises(ValueError):
        _enc(bytes(10000), 4096, 256)


def test_both_kernels_agree_at_the_defaults(ctx):
    from ambc.methods import _gpu_dict_any, _gpu_encode
    for n, seed in ((1, 1), (3, 2), (100, 3), (4096, 4), (5000, 5), (8192, 6)):
        d = _mixed(n, seed)
        assert _gpu_dict_any(d, 4096, 32) == _gpu_encode(2, d) == orc.dict_encode(d), n


def test_should_use_any_length(ctx):
    from ambc.methods import DictionaryCompression
    m = DictionaryCompression()
    for n, seed in ((99, 1), (100, 2), (1002, 3), (1003, 4), (70000, 5), (300000, 6)):
        for d in (_mixed(n, seed), random.Random(seed).randbytes(n)):
            assert m.should_use(d) == orc.should_use(2, d), n
