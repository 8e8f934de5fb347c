"""The oracle's Dictionary encoder for any window / lookahead / length
(orc_dict_encode_wl, the checker of the GPU's k_da_* path) against a literal
pure-Python restatement of DictionaryCompression.compress
(compression_methods.py:195-233) and _find_longest_match (:279-313), on small
inputs; and against orc_dict_encode (pinned by the reference's golden vectors,
test_oracle.py) at the reference's defaults."""
import random

import pytest

from oracle import oracle as orc


def _py_dict(data, window, look):
    """the reference's loop, restated: greedy, earliest of the longest match in
    [max(0, pos - window), pos), lookahead = data[pos:pos + look] (Python slice)"""
    out = bytearray()
    pos = 0
    n = len(data)
    while pos < n:
        ahead = data[pos:pos + look]
        best_i, best_l = 0, 0
        for i in range(max(0, pos - window), pos):
            ln = 0
            while ln < len(ahead) and pos + ln < n and data[i + ln] == data[pos + ln]:
                ln += 1
            if ln > best_l:
                best_i, best_l = i, ln
        if best_l > 2:
            d = pos - best_i
            out += bytes((1, d & 0xFF, (d >> 8) & 0xFF))
            out.append(best_l)          # raises ValueError above 255, as the reference does
            pos += best_l
        else:
            out += bytes((0, data[pos]))
            pos += 1
    return bytes(out)


def _inputs(rng):
    yield b""
    yield b"a"
    yield b"ab" * 3
    yield bytes(300)
    yield bytes(rng.randrange(256) for _ in range(500))
    yield bytes(rng.choice(b"ab") for _ in range(700))
    yield (b"the quick brown fox jumps over the lazy dog. " * 30)[:1200]
    yield bytes(rng.choice(b"abc ") for _ in range(900)) + bytes(400)
    yield off_path_long_match(rng)


def off_path_long_match(rng):
    """a 260-byte repeat (longer than a token can say) whose start the greedy
    path jumps over: the reference does not raise (lookahead >= 260)"""
    rb = lambda k: bytes(rng.randrange(256) for _ in range(k))
    g, h = rb(260), rb(30)
    return g + rb(40) + h + g[:10] + rb(40) + h + g


@pytest.mark.parametrize("window,look", [(4096, 32), (16, 32), (1, 4), (3, 3), (0, 32), (-5, 32),
                                         (100, 0), (100, 2), (100, 255), (100, 256), (700, 1000), (1000, 300),
                                         (64, -1), (64, -400), (64, -5000), (1 << 40, 40)])
def test_dict_encode_wl_matches_restatement(window, look):
    rng = random.Random(window * 31 + look)
    for d in _inputs(rng):
        try:
            want = _py_dict(d, window, look)
        except ValueError:
            with pytest.raises(ValueError):
                orc.dict_encode_wl(d, window, look)
            continue
        assert orc.dict_encode_wl(d, window, look) == want, (len(d), window, look)


def test_dict_encode_wl_defaults_equal_the_pinned_encoder():
    rng = random.Random(5)
    for n in (1, 3, 100, 4095, 4096, 4097, 9000, 20000):
        d = bytes(rng.choice(b"abcdefgh  \n") for _ in range(n))
        assert orc.dict_encode_wl(d, 4096, 32) == orc.dict_encode(d)


def test_off_path_long_match_does_not_raise():
    rng = random.Random(9)
    d = off_path_long_match(rng)
    assert orc.dict_encode_wl(d, 4096, 300) == _py_dict(d, 4096, 300)
    with pytest.raises(ValueError):          # the same repeat on the path raises
        orc.dict_encode_wl(d[:300] + d[300:330] + d[:300], 4096, 300)
