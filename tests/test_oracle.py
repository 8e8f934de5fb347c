"""Pin the CPU oracle against the reference's own outputs (tests/golden/).

Every vector here was produced by importing the reference
(tests/golden/make_golden.py); the oracle must reproduce each one exactly.
"""
import ctypes as C
import hashlib
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle import oracle as orc
from oracle import synth

REF_REGISTERED = (1, 2, 3, 4, 5, 6, 7, 255)   # methods registered in the reference here


@pytest.fixture(scope="module")
def codecs():
    return load_golden("codecs.json")


def test_rle_vectors(codecs):
    for rec in codecs:
        d = bytes.fromhex(rec["data"])
        assert orc.rle_encode(d).hex() == rec["rle"]["out"], rec["name"]


def test_huffman_vectors(codecs):
    for rec in codecs:
        d = bytes.fromhex(rec["data"])
        got = orc.huff_encode(d)
        if rec["huffman"]["ok"]:
            assert got is not None and got.hex() == rec["huffman"]["out"], rec["name"]
        else:
            assert got is None, rec["name"]


def test_dictionary_vectors(codecs):
    n = 0
    for rec in codecs:
        if "dictionary" in rec:
            d = bytes.fromhex(rec["data"])
            assert orc.dict_encode(d).hex() == rec["dictionary"]["out"], rec["name"]
            n += 1
    assert n > 20


def test_should_use_vectors(codecs):
    for rec in codecs:
        d = bytes.fromhex(rec["data"])
        for mid in (1, 2, 3, 4):
            assert orc.should_use(mid, d) == rec["should_use"][str(mid)], (rec["name"], mid)


def test_entropy_table_matches_scalar_numpy():
    # the vectorised table must equal the reference's scalar p*np.log2(p) terms
    for n in (100, 1024, 4096):
        t = orc.entropy_table(n)
        for c in (1, 2, 3, 7, 31, 32, 100, n // 3, n - 1, n):
            p = c / n
            assert t[c] == p * np.log2(p)


def test_huffman_code_tables():
    for rec in load_golden("huffman_codes.json"):
        hist = [tuple(x) for x in rec["hist"]]
        got = orc.huff_code_table(hist)
        assert {str(k): v for k, v in got.items()} == rec["codes"], hist[:4]


def test_decode_kats():
    for rec in load_golden("decode_kat.json"):
        body = bytes.fromhex(rec["body"])
        if rec["ok"]:
            out = orc.decompress_body(body, rec["orig_size"], REF_REGISTERED)
            assert out.hex() == rec["out"], rec["name"]
        else:
            with pytest.raises(ValueError, match="Marker mismatch"):
                orc.decompress_body(body, rec["orig_size"], REF_REGISTERED)


def _input_for(rec):
    data = synth.generate(rec["size"], rec["seed"])
    assert hashlib.sha256(data).hexdigest() == rec["input_sha256"]
    return data


def test_whole_files_native_and_reference():
    checked = 0
    for rec in load_golden("files.json"):
        if rec["mode"] not in ("native", "reference"):
            continue
        if set(rec["methods"]) - {1, 2, 3, 4, 5, 9, 255}:
            continue        # ids 6/7 (bz2/lzma) are host-library codecs the oracle does not restate
        data = _input_for(rec)
        blob, stats = orc.compress_file_bytes(data, rec["chunk"], rec["mode"], rec["methods"])
        with open(os.path.join(GOLDEN, rec["file"]), "rb") as f:
            ref = f.read()
        assert hashlib.sha256(blob).hexdigest() == rec["output_sha256"], rec["name"]
        assert blob == ref
        assert stats == rec["stats"], rec["name"]
        checked += 1
    assert checked >= 28  # every native/reference record, incl. the {1,3,5,255} file


def test_whole_files_decode():
    for rec in load_golden("files.json"):
        data = _input_for(rec)
        with open(os.path.join(GOLDEN, rec["file"]), "rb") as f:
            blob = f.read()
        if blob[:4] != b"AMBC":
            assert blob == data       # stored raw (adaptive_compressor.py:241-247)
            with pytest.raises(ValueError, match="Magic mismatch"):
                orc.decompress_file_bytes(blob)
            continue
        assert orc.decompress_file_bytes(blob, REF_REGISTERED) == data, rec["name"]


def test_config1_behaviour():
    rec = load_golden("config1.json")
    data = synth.random_bytes(rec["size"], rec["seed"])
    assert hashlib.sha256(data).hexdigest() == rec["input_sha256"]
    blob, stats = orc.compress_file_bytes(data, rec["chunk"], "reference", REF_REGISTERED)
    assert rec["output_equals_input"] and blob == data
    assert stats == rec["stats"]
    with pytest.raises(ValueError, match=rec["decompress_exception"]["msg"]):
        orc.decompress_file_bytes(blob)


def test_synth_c_matches_numpy():
    for n, seed in ((1, 1), (1000, 2), (300000, 20250418), (1 << 20, 7)):
        assert orc.synth(n, seed) == synth.generate(n, seed)
    assert orc.random_bytes(12345, 9) == synth.random_bytes(12345, 9)


def test_synth_pinned_sha():
    # pins the "ambc-mixed v1" stream definition
    d = synth.generate(1 << 20, 20250418)
    assert hashlib.sha256(d).hexdigest() == \
        "925fb804a49288d2eacf9f5036f89fbc31fa0b35e91e834e5b3d0479ea8969fd"


def _liblz4():
    try:
        return C.CDLL("liblz4.so.1")
    except OSError:
        pytest.skip("system liblz4 not present")


def test_lz4_frames_decode_with_system_liblz4():
    lz = _liblz4()
    lz.LZ4_decompress_safe.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int]
    lz.LZ4_decompress_safe.restype = C.c_int
    mixed = synth.generate(1 << 20, 3)
    cases = [bytes(4096), b"a" * 13, b"abcdefghijkl" * 300, os.urandom(4096)]
    cases += [mixed[o:o + n] for o, n in ((0, 4096), (70000, 4096), (140000, 8192),
                                           (400000, 65536), (5, 1024), (9, 17))]
    for d in cases:
        fr = orc.lz4_frame_encode(d)
        assert fr[:6] == b"\x04\x22\x4d\x18\x68\x40"
        assert fr[14] == (orc.xxh32(fr[4:14]) >> 8) & 0xFF
        bs = int.from_bytes(fr[15:19], "little")
        if bs & 0x80000000:
            assert fr[19:19 + (bs & 0x7FFFFFFF)] == d
            continue
        out = C.create_string_buffer(len(d) + 16)
        r = lz.LZ4_decompress_safe(fr[19:19 + bs], out, bs, len(d) + 16)
        assert r == len(d) and out.raw[:r] == d
        assert orc.decode_chunk(9, fr, len(d)) == d


def test_multi_block_lz4_frames_decode_with_system_liblz4():
    """past 64 KiB (the single-call plugin at any length): one frame of
    independent 64 KiB blocks, every block decoded alone by the system liblz4"""
    lz = _liblz4()
    lz.LZ4_decompress_safe.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int]
    lz.LZ4_decompress_safe.restype = C.c_int
    mixed = synth.generate(1 << 20, 4)
    for d in (mixed[:65537], mixed[1000:1000 + 300000], bytes(200000), os.urandom(140000), mixed):
        fr = orc.lz4_frame_encode(d)
        assert fr[:6] == b"\x04\x22\x4d\x18\x68\x40"
        assert int.from_bytes(fr[6:14], "little") == len(d)
        assert fr[14] == (orc.xxh32(fr[4:14]) >> 8) & 0xFF
        pos, got = 15, bytearray()
        while True:
            bs = int.from_bytes(fr[pos:pos + 4], "little")
            pos += 4
            if bs == 0:
                break
            if bs & 0x80000000:
                got += fr[pos:pos + (bs & 0x7FFFFFFF)]
                pos += bs & 0x7FFFFFFF
                continue
            out = C.create_string_buffer(65536 + 16)
            r = lz.LZ4_decompress_safe(fr[pos:pos + bs], out, bs, 65536 + 16)
            assert 0 < r <= 65536
            got += out.raw[:r]
            pos += bs
        assert pos == len(fr) and bytes(got) == d
        assert orc.decode_chunk(9, fr, len(d)) == d


def test_gdeflate_streams_are_valid_zlib():
    """"ambc-deflate v1" (the GPU's id-5 definition): every stream inflates with
    the same zlib the reference's DeflateCompression.decompress uses, for edge
    sizes, zero runs, random, periodic and mixed inputs; the parse covers the
    input exactly with legal DEFLATE matches."""
    import random
    import zlib
    mixed = synth.generate(1 << 22, 7)
    rng = random.Random(1)
    cases = [b"", b"a", b"ab" * 3, bytes(4096), b"x" * 70000, synth.random_bytes(4096, 5),
             synth.random_bytes(100000, 6), bytes(range(256)) * 16, b"abcab" * 900]
    for _ in range(150):
        o = rng.randrange(len(mixed) - 70000)
        n = rng.choice([64, 100, 1000, 1024, 4096, 8192, 16384, 65536, rng.randrange(1, 70000)])
        cases.append(mixed[o:o + n])
    tot = ztot = 0
    for d in cases:
        z = orc.gdeflate_encode(d)
        assert z[:2] == b"\x78\xda"
        assert zlib.decompress(z) == d, len(d)
        p = 0
        for pos, L, D in orc.gd_parse(d):
            assert pos >= p and 4 <= L <= 258 and 1 <= D <= min(pos, 32768)
            assert d[pos:pos + L] == bytes(d[pos - D + (i % D)] for i in range(L)) or \
                d[pos:pos + L] == (d[pos - D:pos] * (L // D + 1))[:L]
            p = pos + L
        tot += len(z)
        ztot += len(zlib.compress(d, 9))
    assert tot < 1.15 * ztot      # within 15 % of zlib level 9 on these inputs


def test_multisize_walk_matches_reference_golden():
    """The oracle's multi-size walk (adaptive_compressor.py:363-394,537-590, the
    reference's default eight CHUNK_SIZE_CANDIDATES, its stdlib method set
    {1..7}) reproduces the reference-generated default-candidates container."""
    from conftest import GOLDEN, load_golden
    rec = [r for r in load_golden("files.json") if r["name"] == "default_s3_n12288"][0]
    data = synth.generate(rec["size"], rec["seed"])
    with open(os.path.join(GOLDEN, rec["file"]), "rb") as f:
        blob = f.read()
    body, st = orc.compress_body_multisize(
        data, [131072, 65536, 32768, 16384, 8192, 4096, 2048, 1024], (1, 2, 3, 4, 5, 6, 7, 255),
        reference_set=True)
    assert body == blob[47:]
    cs = rec["stats"]["chunk_stats"]
    for k in ("total_chunks", "compressed_chunks", "raw_chunks", "bytes_saved",
              "compressed_size_without_overhead", "overhead_bytes"):
        assert st[k] == cs[k], k
    assert {str(k): v for k, v in st["method_usage"].items()} == cs["method_usage"]


def test_multisize_walk_remainder_raw():
    """No size beats raw at a position: the whole remainder becomes one raw
    package (adaptive_compressor.py:586-588), after the compressible head."""
    rnd = random.Random(4242)
    data = bytes(20000) + bytes(rnd.randrange(256) for _ in range(30000))
    body, st = orc.compress_body_multisize(data, [16384, 8192, 4096, 2048, 1024], (1, 3, 4, 255))
    assert st["raw_chunks"] == 1 and st["compressed_chunks"] >= 5
    assert orc.decompress_body(body, len(data)) == data
