"""integration/ambc_binding.py -- the reference-side binding INTEGRATION.md quotes --
applied to a stand-in class that carries the reference's attribute names and
method list shape (adaptive_compressor.py:49-178: ``compression_methods`` in the
reference's order with compression_fix.py's duplicates, ``method_lookup``,
``method_chunk_prefs``, ``CHUNK_SIZE_CANDIDATES``, ``marker_bytes_aligned``,
``_init_stats`` / ``chunk_stats``).  The stand-in is this repository's own code;
its method objects are ambc's plugins (the reference's wrappers for ids 5-8).

* the reference's own default container (tests/golden default_s3_n12288) is
  reproduced bit for bit through the binding and decodes;
* the golden reference-loop containers (one candidate) too;
* bodies and stats equal the oracle's reference loop on larger inputs, with ids
  6 / 7 scored on the host through the instance's own objects (never dropped);
* id 9 routed to the host through an LZ4 object gives the same body as the
  device's LZ4 (gpu_lz4=True);
* configurations the library cannot follow run the stand-in's own loop
  (BindingFallback), and host-decoded ids (6 / 7 / 8) decode through the
  instance's objects."""
import os
import sys
import warnings

import pytest

from conftest import GOLDEN, REPO, load_golden
from oracle import oracle as orc
from oracle import synth

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(REPO, "integration"))

REF_CANDS = [131072, 65536, 32768, 16384, 8192, 4096, 2048, 1024]


def _standin_class():
    from ambc import methods as M
    from ambc.registry import METHOD_CHUNK_PREFS

    class RefShaped:
        """the reference's AdaptiveCompressor surface the two loops read"""
        CHUNK_SIZE_CANDIDATES = list(REF_CANDS)

        def __init__(self, ids=(1, 2, 3, 4, 5, 6, 7), extra=()):
            basic = [M.RLECompression, M.DictionaryCompression, M.HuffmanCompression, M.DeltaCompression]
            lib = {5: M.DeflateCompression, 6: M.Bzip2Compression, 7: M.LZMACompression,
                   8: M.ZstdCompression}
            # adaptive_compressor.py:129-176: basic four, compression_fix's list
            # (basic four + raw + library codecs), the library codecs again, raw
            ms = [c() for i, c in zip((1, 2, 3, 4), basic) if i in ids]
            ms += [c() for i, c in zip((1, 2, 3, 4), basic) if i in ids] + [M.NoCompression()]
            ms += [lib[i]() for i in sorted(lib) if i in ids]
            ms += list(extra)
            ms += [lib[i]() for i in sorted(lib) if i in ids] + [M.NoCompression()]
            self.compression_methods = ms
            self.method_lookup = {m.type_id: m for m in ms}
            self.method_chunk_prefs = dict(METHOD_CHUNK_PREFS)
            self.marker_bytes_aligned = b"\xff\xff\x00\x00"
            self.chunk_stats = None
            self.own_loop_calls = 0

        def _init_stats(self, file_data):
            self.chunk_stats = {"total_chunks": 0, "compressed_chunks": 0, "raw_chunks": 0,
                                "method_usage": {}, "bytes_saved": 0, "original_size": len(file_data),
                                "compressed_size_without_overhead": 0, "overhead_bytes": 0}
            for m in self.compression_methods:
                self.chunk_stats["method_usage"][m.type_id] = 0

        # the "reference's own loops" of the stand-in: the oracle's restatement
        def _adaptive_compress(self, file_data):
            self.own_loop_calls += 1
            ids = tuple(sorted({m.type_id for m in self.compression_methods}))
            body, st = orc.compress_body_multisize(file_data, self.CHUNK_SIZE_CANDIDATES, ids,
                                                   prefs=self.method_chunk_prefs, deflate="zlib",
                                                   reference_set=True)
            self._init_stats(file_data)
            return body

        def _adaptive_decompress(self, data, orig_size):
            self.own_loop_calls += 1
            return orc.decompress_body(data, orig_size, registered=tuple(self.method_lookup))

    return RefShaped


@pytest.fixture(scope="module")
def Bound(hip_lib):
    import ambc_binding
    cls = _standin_class()
    ambc_binding.bind(cls)
    yield cls
    ambc_binding.unbind(cls)


def _stats_equal(cs, st):
    for k in ("total_chunks", "compressed_chunks", "raw_chunks", "bytes_saved",
              "compressed_size_without_overhead", "overhead_bytes"):
        assert cs[k] == st[k], k
    for mid, v in cs["method_usage"].items():
        assert v == st["method_usage"].get(str(mid), st["method_usage"].get(mid, 0)), mid


def test_binding_reproduces_reference_default_golden(Bound):
    rec = [r for r in load_golden("files.json") if r["name"] == "default_s3_n12288"][0]
    data = synth.generate(rec["size"], rec["seed"])
    with open(os.path.join(GOLDEN, rec["file"]), "rb") as f:
        blob = f.read()
    comp = Bound()
    assert [m.type_id for m in comp.compression_methods] == [1, 2, 3, 4, 1, 2, 3, 4, 255, 5, 6, 7,
                                                             5, 6, 7, 255]
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        body = comp._adaptive_compress(data)
        assert body == blob[47:]
        assert comp._adaptive_decompress(body, len(data)) == data
    _stats_equal(comp.chunk_stats, rec["stats"]["chunk_stats"])
    assert comp.own_loop_calls == 0


def test_binding_reproduces_golden_reference_loops(Bound):
    n = 0
    for rec in load_golden("files.json"):
        if rec["mode"] != "reference":
            continue
        data = synth.generate(rec["size"], rec["seed"])
        with open(os.path.join(GOLDEN, rec["file"]), "rb") as f:
            blob = f.read()
        if blob[:4] != b"AMBC":
            continue
        comp = Bound(ids=tuple(i for i in rec["methods"] if i != 255))
        comp.CHUNK_SIZE_CANDIDATES = [rec["chunk"]]
        body = comp._adaptive_compress(data)
        assert body == blob[47:], rec["name"]
        assert comp._adaptive_decompress(body, len(data)) == data
        _stats_equal(comp.chunk_stats, rec["stats"]["chunk_stats"])
        n += 1
    assert n >= 5


def _word_text(n, seed):
    import random
    rnd = random.Random(seed)
    vocab = ["".join(chr(97 + rnd.randrange(26)) for _ in range(rnd.randrange(2, 11))) for _ in range(3000)]
    out, have = [], 0
    while have < n:
        w = vocab[min(int(rnd.paretovariate(1.1)) - 1, 2999)] + (". " if rnd.random() < 0.07 else " ")
        out.append(w)
        have += len(w)
    return "".join(out).encode()[:n]


@pytest.mark.parametrize("cands", [REF_CANDS, [16384], [4096]])
def test_binding_full_default_set_matches_oracle(Bound, cands):
    """ids 1..7: 1-5 on the device (5 as zlib-9), 6 / 7 through the instance's own
    bz2 / lzma objects on host threads; never dropped, and they win somewhere."""
    used = {6: 0, 7: 0}
    for data in (_word_text(120000, 91), synth.generate(90000, 92), synth.random_bytes(30000, 93) * 3):
        comp = Bound()
        comp.CHUNK_SIZE_CANDIDATES = list(cands)
        body = comp._adaptive_compress(data)
        ref, st = orc.compress_body_multisize(data, cands, (1, 2, 3, 4, 5, 6, 7, 255), deflate="zlib",
                                              reference_set=True)
        assert body == ref, (cands, len(data))
        _stats_equal(comp.chunk_stats, st)
        for k in used:
            used[k] += comp.chunk_stats["method_usage"][k]
        assert comp._adaptive_decompress(body, len(data)) == data
    assert comp.own_loop_calls == 0
    assert used[6] > 0 or cands == [4096]


def test_binding_host_lz4_equals_device_lz4(hip_lib):
    """id 9 (python-lz4 in the reference) is host-scored unless gpu_lz4=True: an LZ4
    object with the device's own frame bytes gives the same body either way."""
    import ambc_binding
    from ambc.methods import CompressionMethod

    class OracleLZ4(CompressionMethod):
        type_id = 9

        def compress(self, data):
            return orc.lz4_frame_encode(bytes(data))

        def decompress(self, data, original_length):
            return orc.decode_chunk(9, data, original_length)

        def should_use(self, data, threshold=0.9):
            return len(data) >= 1024

    data = synth.generate(200000, 94)
    bodies = []
    for gpu_lz4 in (False, True):
        cls = _standin_class()
        ambc_binding.bind(cls, gpu_lz4=gpu_lz4)
        comp = cls(ids=(1, 3, 4), extra=[OracleLZ4()])
        for cands in (REF_CANDS, [4096]):
            comp.CHUNK_SIZE_CANDIDATES = list(cands)
            body = comp._adaptive_compress(data)
            assert comp._adaptive_decompress(body, len(data)) == data
            assert comp.chunk_stats["method_usage"][9] > 0
            bodies.append(body)
        assert comp.own_loop_calls == 0
    assert bodies[0] == bodies[2] and bodies[1] == bodies[3]
    ref, _ = orc.compress_body_multisize(data, [4096], (1, 3, 4, 9, 255))
    assert bodies[1] == ref


def test_binding_falls_back_where_it_cannot_follow(Bound):
    from ambc import methods as M
    data = synth.generate(40000, 95)
    comp = Bound(ids=(1, 3))
    comp.compression_methods.insert(0, M.Bzip2Compression())     # id 6 before id 1: list-order ties
    comp.method_lookup[6] = comp.compression_methods[0]
    with pytest.warns(ambc_binding_warning()):
        body = comp._adaptive_compress(data)
    assert comp.own_loop_calls == 1
    comp2 = Bound(ids=(1, 3))
    comp2.CHUNK_SIZE_CANDIDATES = [262144, 4096]                  # above the walk's 131072
    with pytest.warns(ambc_binding_warning()):
        comp2._adaptive_compress(data)
    assert comp2.own_loop_calls == 1
    assert comp._adaptive_decompress(body, len(data)) == data


def ambc_binding_warning():
    import ambc_binding
    return ambc_binding.BindingFallback


def test_binding_decodes_host_ids_through_instance_objects(Bound):
    """packages of ids 6 / 7 / 8 (bz2 / lzma / zstd) are handed to the instance's
    method objects; unregistered ids are verbatim; damaged ones decode to zeros."""
    import bz2
    import lzma
    import struct

    def pkg(t, orig, payload):
        return b"\xff\xff\x00\x00" + bytes((t, 0)) + struct.pack("<III", orig, orig, len(payload)) + payload

    a, b, c = synth.generate(5000, 1), synth.generate(7000, 2), synth.generate(3000, 3)
    parts = [pkg(6, len(a), bz2.compress(a)), pkg(1, len(b), orc.rle_encode(b)),
             pkg(7, len(c), lzma.compress(c)), pkg(6, 900, b"BZh9 damaged"), pkg(77, 4, b"abcd")]
    ids = (1, 2, 3, 4, 5, 6, 7)
    if orc.zstd_lib() is not None:
        parts += [pkg(8, len(a), orc.zstd_compress(a)), pkg(8, 50, orc.zstd_compress(a)[:9])]
        ids += (8,)
    body = b"".join(parts) + pkg(0, 0, b"")[:16]
    comp = Bound(ids=ids)
    orig = sum(int.from_bytes(p[10:14], "little") for p in parts)
    for osz in (orig, orig - 10, orig + 10):
        want = orc.decompress_body(body, osz, registered=tuple(comp.method_lookup))
        assert comp._adaptive_decompress(body, osz) == want
    assert comp.own_loop_calls == 0
