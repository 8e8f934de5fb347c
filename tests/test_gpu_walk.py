"""The device header walk of the decode pipeline (ambc_walk.hip) against the
oracle's walk (oracle.decompress_body, adaptive_compressor.py:399-445), byte
for byte.  AMBC_DEVWALK_MIN=0 sends every body through the device walk and
AMBC_WALK_PIECE cuts it into small pieces, so that chains cross piece
boundaries at every kind of position; AMBC_DECODE_STRICT makes a fallback to
the host walk an error wherever the body needs none."""
import bz2
import lzma
import os
import struct
import zlib

import numpy as np
import pytest

from oracle import oracle as orc
from oracle import synth

pytestmark = pytest.mark.gpu

PIECES = (64, 1000, 4096, 1 << 16)


@pytest.fixture(scope="module")
def ctx(hip_lib):
    from ambc import _lib
    return _lib.default_context()


def _comp(**kw):
    from ambc import AdaptiveCompressor
    return AdaptiveCompressor(**kw)


def _pkg(t, orig, payload, clen=None):
    clen = len(payload) if clen is None else clen
    return b"\xff\xff\x00\x00" + bytes((t, 0)) + struct.pack("<III", orig, orig, clen) + payload


END = _pkg(0, 0, b"")[:16]


class _Env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _check(comp, body, osz, strict=True):
    """decode through the device walk; equal to the oracle (or both raise)"""
    try:
        want = orc.decompress_body(body, osz)
    except ValueError:
        with pytest.raises(ValueError, match="Marker mismatch"):
            comp._adaptive_decompress(body, osz)
        return
    env = {"AMBC_DECODE_STRICT": 1} if strict else {}
    with _Env(**env):
        got = comp._adaptive_decompress(body, osz)
    assert (got == want) is True, (len(body), osz)


def _crafted(rng):
    """packages of every kind the walk routes, fake headers inside payloads"""
    parts, orig = [], 0
    fake_chain = _pkg(255, 40, b"\x00" * 22)       # a valid-looking chain inside a payload
    for k in range(60):
        kind = k % 10
        raw = bytearray(rng.integers(0, 256, int(rng.integers(1, 9000)), dtype=np.uint8).tobytes())
        if kind == 0:
            for q in range(0, max(1, len(raw) - 40), 517):
                raw[q:q + 40] = fake_chain[:40]
            parts.append(_pkg(255, len(raw), bytes(raw)))
            orig += len(raw)
        elif kind == 1:
            parts.append(_pkg(77, 5, bytes(raw[:300])))          # unregistered: copied verbatim
            orig += 300
        elif kind == 2:
            d = bytes(raw[:2000]) * 2
            parts.append(_pkg(6, len(d), bz2.compress(d)))         # host codec (bz2)
            orig += len(d)
        elif kind == 3:
            d = bytes(raw[:1500]) * 3
            parts.append(_pkg(7, len(d), lzma.compress(d)))        # host codec (lzma)
            orig += len(d)
        elif kind == 4:
            d = bytes(raw[:100]) * 900                             # 90000 > 64 KiB: host zlib
            parts.append(_pkg(5, len(d), zlib.compress(d, 6)))
            orig += len(d)
        elif kind == 5:
            d = bytes(raw[:700]) * 5
            parts.append(_pkg(5, len(d), zlib.compress(d, 9)))     # GPU inflate
            orig += len(d)
        elif kind == 6:
            parts.append(_pkg(5, 100, b""))                        # empty zlib payload: nothing
        elif kind == 7:
            parts.append(_pkg(255, 64, b"\xff\xff\x00\x00" * 16))  # the densest candidates
            orig += 64
        elif kind == 8:
            d = bytes(raw[:3000])
            parts.append(_pkg(4, len(d), d))                       # Delta: min(clen, orig)
            orig += len(d)
        else:
            parts.append(_pkg(255, 9000, bytes(raw[:50])))         # raw short payload: zero padded
            orig += 9000
    return parts, orig


@pytest.mark.parametrize("piece", PIECES)
def test_device_walk_crafted_bodies(ctx, piece):
    rng = np.random.default_rng(piece)
    parts, orig = _crafted(rng)
    body = b"".join(parts) + END
    comp = _comp()
    with _Env(AMBC_DEVWALK_MIN=0, AMBC_WALK_PIECE=piece):
        for osz in (orig, orig - 1, orig // 2, orig + 777, 1, 0):
            _check(comp, body, osz)
        # stops: a type-0 header mid-body, a payload past the end, trailing bytes
        mid = len(b"".join(parts[:23]))
        _check(comp, body[:mid] + END + body[mid:], orig)
        _check(comp, body[:mid] + _pkg(255, 10, b"", clen=1 << 30) + body[mid:], orig)
        _check(comp, body[:-16] + b"\x01" * 17, orig)
        _check(comp, body[:-16] + b"\xff\xff\x00\x00" + b"\x01" * 13, orig)
        # marker mismatches: at each of a few packages (reached, or after the stop)
        starts = np.cumsum([0] + [len(p_) for p_ in parts])
        produced = [orc.decompress_body(p_ + END, 0, return_produced=True)[1] for p_ in parts]
        for k in (0, 1, 17, 40, 59):
            bad = bytearray(body)
            bad[int(starts[k]) + 2] ^= 0x40
            _check(comp, bytes(bad), orig)                     # reached: raises
            _check(comp, bytes(bad), sum(produced[:k]))        # the output is complete before it


@pytest.mark.parametrize("piece", (64, 4096))
def test_device_walk_tiny_bodies(ctx, piece):
    comp = _comp()
    with _Env(AMBC_DEVWALK_MIN=0, AMBC_WALK_PIECE=piece):
        for body in (b"", b"\x01", b"\xff\xff\x00\x00" + b"\x00" * 13, END, _pkg(255, 3, b"abc"),
                     _pkg(255, 3, b"abc") + END, b"\x00" * 18, _pkg(255, 3, b"abc")[:-1],
                     _pkg(1, 64, orc.rle_encode(b"\x07" * 64)) + END):
            for osz in (0, 3, 64, 100):
                _check(comp, body, osz)


@pytest.mark.parametrize("piece", PIECES)
def test_device_walk_real_bodies(ctx, piece):
    """bodies of the compressor (every GPU codec) and the reference's golden files"""
    from conftest import GOLDEN, load_golden
    with _Env(AMBC_DEVWALK_MIN=0, AMBC_WALK_PIECE=piece):
        for methods, chunk, mode in (((1, 2, 3, 4, 9), 4096, "native"), ((1, 3, 4, 5), 8192, "native"),
                                     ((1, 3, 4), 4096, "reference"), ((1, 2, 3, 4, 5, 9), 65536, "native")):
            d = synth.generate(600_000, 11)
            comp = _comp(chunk_size=chunk, mode=mode, methods=methods)
            body = comp._adaptive_compress(d)
            for osz in (len(d), len(d) - 4095, len(d) + 5):
                _check(comp, body, osz)
        n = 0
        for rec in load_golden("files.json"):
            with open(os.path.join(GOLDEN, rec["file"]), "rb") as f:
                blob = f.read()
            if blob[:4] != b"AMBC":
                continue
            data = synth.generate(rec["size"], rec["seed"])
            with _Env(AMBC_DECODE_STRICT=1):
                assert _comp().decompress_bytes(blob) == data, rec["name"]
            n += 1
        assert n >= 20


def test_device_walk_large_body_pieces(ctx):
    """a 96 MiB body of 4 KiB packages over the default 64 MiB pieces (the
    production configuration): the chain crosses a piece boundary inside a
    payload; stats report the device walk"""
    rng = np.random.default_rng(3)
    blk = rng.integers(0, 256, 4096, dtype=np.uint8).tobytes()
    one = _pkg(255, 4096, blk)
    npk = (96 << 20) // len(one)
    body = one * npk + END
    comp = _comp()
    orig = npk * 4096
    with _Env(AMBC_DECODE_STRICT=1):
        out = comp._adaptive_decompress(body, orig)
    assert len(out) == orig and out[:4096] == blk and out[-4096:] == blk
    assert out == blk * npk
    st = comp._last_device_stats
    assert st.total_chunks == npk and st.payload_bytes == orig
