"""id 8 (ZStandard, advanced_compression.py:219-261) through the GPU decode path:
bodies mixing GPU-decoded packages (RLE, Huffman, LZ4, DEFLATE, raw) with
libzstd-written level-19 frames -- valid, without a content size, damaged,
truncated, with trailing bytes -- decoded by ambc_decompress_ex (host walk and
device walk) with the id-8 packages handed back to ZstdCompression, equal to the
oracle's _adaptive_decompress with its restatement of python-zstandard's
decompress.  Unregistered, id 8 is copied verbatim like any unknown id
(adaptive_compressor.py:432-435).  And the host-scored walk with id 8 among the
reference's codecs against the oracle's reference loop.  Parity unpinned: the
reference holds no zstd fixture (python-zstandard absent)."""
import os
import struct
import zlib

import numpy as np
import pytest

from oracle import oracle as orc
from oracle import synth

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(orc.zstd_lib() is None, reason="libzstd.so.1 not loadable")]

REG8 = (1, 2, 3, 4, 5, 6, 7, 8, 9, 255)


@pytest.fixture(scope="module")
def ctx(hip_lib):
    from ambc import _lib
    return _lib.default_context()


def _pkg(t, orig, payload):
    return b"\xff\xff\x00\x00" + bytes((t, 0)) + struct.pack("<III", orig, orig, len(payload)) + payload


END = _pkg(0, 0, b"")[:16]


def _body(seed, n_pkgs=48):
    """(body, orig_size): every package kind, a third of them zstd in all its forms"""
    from test_library_plugins import zstd_cases
    rng = np.random.default_rng(seed)
    zc = zstd_cases()
    parts, orig = [], 0
    for k in range(n_pkgs):
        d = synth.generate(int(rng.integers(200, 6000)), seed * 100 + k)
        kind = k % 6
        if kind in (0, 3):
            payload, o = zc[int(rng.integers(0, len(zc)))]
            parts.append(_pkg(8, o, payload))
            orig += o
        elif kind == 1:
            parts.append(_pkg(1, len(d), orc.rle_encode(d)))
            orig += len(d)
        elif kind == 2:
            h = orc.huff_encode(d)
            parts.append(_pkg(3, len(d), h) if h is not None else _pkg(255, len(d), d))
            orig += len(d)
        elif kind == 4:
            parts.append(_pkg(9, len(d), orc.lz4_frame_encode(d)) if len(d) >= 1024 else
                         _pkg(5, len(d), zlib.compress(d, 9)))
            orig += len(d)
        else:
            parts.append(_pkg(255, len(d), d))
            orig += len(d)
    return b"".join(parts) + END, orig


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


def _comp(**kw):
    from ambc import AdaptiveCompressor
    return AdaptiveCompressor(**kw)


@pytest.mark.parametrize("walk", ["host", "device"])
def test_zstd_packages_decode_like_oracle(ctx, walk):
    comp = _comp()
    assert 8 in comp.method_lookup
    env = {"AMBC_DEVWALK_MIN": 0, "AMBC_WALK_PIECE": 4096} if walk == "device" else {}
    for seed in (1, 2, 3):
        body, orig = _body(seed)
        for osz in (orig, orig - 3000, orig + 500):
            want = orc.decompress_body(body, osz, registered=REG8)
            with _Env(**env):
                got = comp._adaptive_decompress(body, osz)
            assert got == want, (seed, osz)


def test_zstd_unregistered_is_verbatim(ctx):
    from ambc.methods import DECODE_METHODS
    comp = _comp()
    comp.method_lookup = {i: DECODE_METHODS[i]() for i in (1, 2, 3, 4, 5, 6, 7, 9, 255)}
    body, orig = _body(4)
    want = orc.decompress_body(body, orig, registered=(1, 2, 3, 4, 5, 6, 7, 9, 255))
    assert comp._adaptive_decompress(body, orig) == want


def test_zstd_host_scored_walk_matches_oracle(ctx):
    """the reference's default set with zstandard installed {1..8}: id 8 scored on
    host threads beside the device's encoders; bodies / stats equal the oracle's
    reference loop with the same library calls, and zstd wins somewhere."""
    ids = (1, 2, 3, 4, 5, 6, 7, 8)
    cands = [131072, 65536, 32768, 16384, 8192, 4096, 2048, 1024]
    used = 0
    for data in (synth.generate(150000, 61), synth.random_bytes(30000, 62) * 3 + bytes(5000)):
        for cs in (cands, [8192]):
            comp = _comp(methods=ids, mode="reference", deflate="zlib9")
            comp.CHUNK_SIZE_CANDIDATES = list(cs)
            body = comp._adaptive_compress(data)
            ref, st = orc.compress_body_multisize(data, cs, ids + (255,), deflate="zlib", reference_set=True)
            assert body == ref, (len(data), cs)
            for k in ("total_chunks", "compressed_chunks", "raw_chunks", "bytes_saved",
                      "compressed_size_without_overhead", "overhead_bytes"):
                assert comp.chunk_stats[k] == st[k], k
            used += comp.chunk_stats["method_usage"][8]
            assert comp._adaptive_decompress(body, len(data)) == data
    assert used > 0
