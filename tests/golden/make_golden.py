#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Run ONLY in the build container (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports /root/reference (read-only) through the test-only ``bitarray``
stand-in in ``tests/golden/_standin`` and records, as data:

* codecs.json        per-codec ``compress`` outputs / exceptions and ``should_use``
                     decisions (RLE, Dictionary, Huffman, Delta;
                     compression_methods.py:78-343,354-667)
* huffman_codes.json Huffman code tables from ``_build_huffman_tree`` +
                     ``_generate_codes`` (compression_methods.py:472-549)
* files/*.ambc +     whole-file containers from ``AdaptiveCompressor.compress``
  files.json         (adaptive_compressor.py:221-255) in three selector setups:
                     reference loop with CHUNK_SIZE_CANDIDATES=[C] ("reference"
                     mode, remainder-raw quirk), a per-chunk harness
                     (``_pick_best_chunk_and_method(chunk,0)`` + ``_process_chunk``
                     per C-byte chunk = "native" mode) and the default
                     8-candidate loop; plus the reference's stats dicts
* decode_kat.json    ``_adaptive_decompress`` outputs on crafted bodies
                     (adaptive_compressor.py:396-454), incl. lenient paths
* config1.json       C1 behaviour: 1 MiB random -> stored raw, decompress raises

Inputs are regenerated from seeds with ``oracle/synth.py`` (their SHA-256 is
stored), so no reference source ever enters the repository.
"""
import contextlib
import hashlib
import io
import json
import os
import random
import struct
import sys
import tempfile
import zlib

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "_standin"))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

from oracle import synth  # noqa: E402

_sink = io.StringIO()


@contextlib.contextmanager
def quiet():
    with contextlib.redirect_stdout(_sink), contextlib.redirect_stderr(_sink):
        yield
    _sink.seek(0)
    _sink.truncate()


with quiet():
    import adaptive_compressor as ac  # noqa: E402
    import compression_methods as cm  # noqa: E402


class _NoBar:
    def __init__(self, *a, **k):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def update(self, n):
        pass


ac.tqdm = _NoBar
MARKER = b"\xff\xff\x00\x00"


def H(b):
    return b.hex()


def sha(b):
    return hashlib.sha256(b).hexdigest()


# --------------------------------------------------------------------------
# case inputs
# --------------------------------------------------------------------------
def case_inputs():
    rnd = random.Random(1234)
    cases = []

    def add(name, data):
        cases.append((name, bytes(data)))

    for n in (1, 2, 3, 4, 5, 31, 32, 99, 100, 101, 255, 256, 257, 1000, 1024, 4096):
        add(f"zeros_{n}", bytes(n))
    for n in (4, 100, 1024, 4096):
        add(f"const_41_{n}", b"A" * n)
    for n in (100, 1024, 4096):
        add(f"ramp_{n}", bytes(i % 256 for i in range(n)))
        add(f"ramp20_{n}", bytes((100 + i % 20) % 256 for i in range(n)))
    for n in (3, 50, 100, 1000, 1024, 4096):
        add(f"random_{n}", bytes(rnd.getrandbits(8) for _ in range(n)))
    add("two_sym_4096", bytes(rnd.choice((7, 200)) for _ in range(4096)))
    add("two_sym_skew_1024", bytes(200 if rnd.random() < 0.05 else 7 for _ in range(1024)))
    s255 = list(range(255)) * 4 + [rnd.randrange(255) for _ in range(3076)]
    rnd.shuffle(s255)
    add("sym255_4096", bytes(s255))
    s256 = list(range(256)) * 2 + [rnd.getrandbits(8) for _ in range(512)]
    rnd.shuffle(s256)
    add("sym256_1024", bytes(s256))
    add("runs_600A_300B", b"A" * 600 + b"B" * 300 + b"C" * 256 + b"D" * 255 + b"E" * 510)
    add("runs_mixed_4096", b"".join(bytes([rnd.randrange(4)]) * rnd.randrange(1, 400)
                                    for _ in range(60))[:4096])
    add("text_1650", b"This is a test text file with some repeating content. " * 30)
    add("text_sentences", b"".join(f"This is test sentence {i} with some repetition. ".encode()
                                   for i in range(50)))
    add("repeated_3000", b"A" * 1000 + b"B" * 1000 + b"C" * 1000)
    mixed = synth.generate(1 << 20, 20250418)
    for i, (off, n) in enumerate([(0, 4096), (5000, 4096), (70000, 4096), (140000, 4096),
                                  (200000, 1024), (300000, 8192), (400000, 4096),
                                  (517000, 4096), (600000, 3000), (700001, 4096),
                                  (800000, 16384), (131000, 4096)]):
        add(f"mixed_{i}_{off}_{n}", mixed[off:off + n])
    for n in (100, 1024, 4096, 8192):
        ascii_ = synth.generate(300000, 7)[140000:140000 + n]
        add(f"ascii_{n}", ascii_)
    # Near the Huffman entropy threshold (7.0): 128 symbols x 32 = exactly 7.0
    eq = list(range(128)) * 32
    rnd.shuffle(eq)
    add("entropy_exact7_4096", bytes(eq))
    near = list(range(129)) * 31 + list(range(97))
    rnd.shuffle(near)
    add("entropy_near7_4096", bytes(near[:4096]))
    return cases


def run_codec(method, data):
    with quiet():
        try:
            out = method.compress(data)
            return {"ok": True, "out": H(out)}
        except Exception as e:  # noqa: BLE001 -- record the exception type
            return {"ok": False, "exc": type(e).__name__}


def gen_codecs():
    rle, dic, huf, dlt = (cm.RLECompression(), cm.DictionaryCompression(),
                          cm.HuffmanCompression(), cm.DeltaCompression())
    out = []
    for name, data in case_inputs():
        rec = {"name": name, "data": H(data)}
        with quiet():
            rec["should_use"] = {"1": bool(rle.should_use(data)),
                                 "2": bool(dic.should_use(data)),
                                 "3": bool(huf.should_use(data)),
                                 "4": bool(dlt.should_use(data))}
        rec["rle"] = run_codec(rle, data)
        rec["huffman"] = run_codec(huf, data)
        rec["delta"] = run_codec(dlt, data)
        if len(data) <= 1024 or name.startswith("ascii_4096"):
            rec["dictionary"] = run_codec(dic, data)
        out.append(rec)
    return out


def gen_huffman_codes():
    rnd = random.Random(99)
    huf = cm.HuffmanCompression()
    hists = []
    hists.append([(65, 10), (66, 10)])
    hists.append([(s, 5) for s in range(16)])
    hists.append([(s, 1) for s in range(255)])
    hists.append([(200 - s, 7) for s in range(40)])
    fib = [1, 1]
    while len(fib) < 24:
        fib.append(fib[-1] + fib[-2])
    hists.append([(s, fib[s]) for s in range(24)])
    hists.append([(23 - s, fib[s]) for s in range(24)])
    for t in range(55):
        k = rnd.choice([2, 3, 5, 8, 17, 30, 64, 100, 200, 255])
        syms = rnd.sample(range(256), k)
        mode = t % 3
        if mode == 0:
            hist = [(s, rnd.randint(1, 4096)) for s in syms]
        elif mode == 1:
            hist = [(s, rnd.choice([1, 2, 3, 4])) for s in syms]
        else:
            hist = [(s, rnd.randint(1, 20) * 16) for s in syms]
        hists.append(hist)
    res = []
    for hist in hists:
        freq = dict(hist)
        with quiet():
            tree = huf._build_huffman_tree(freq)
            codes = {}
            huf._generate_codes(tree, "", codes)
        res.append({"hist": hist, "codes": {str(k): v for k, v in sorted(codes.items())}})
    return res


def per_chunk_harness(comp, C):
    """Native-mode semantics: each C-byte chunk decided independently."""
    def _adaptive_compress(file_data):
        comp._init_stats(file_data)
        output = bytearray()
        for k, pos in enumerate(range(0, len(file_data), C)):
            chunk = file_data[pos:pos + C]
            _, mid = comp._pick_best_chunk_and_method(chunk, 0)
            pkg, st = comp._process_chunk(chunk, mid, k)
            comp._update_stats(st)
            output.extend(pkg)
        end = comp._create_end_chunk()
        output.extend(end)
        comp.chunk_stats["overhead_bytes"] += len(end)
        return bytes(output)
    return _adaptive_compress


def restrict(comp, ids):
    keep = []
    for m in comp.compression_methods:
        if m.type_id in ids and m.type_id not in [x.type_id for x in keep]:
            keep.append(m)
    comp.compression_methods = keep


def clean_stats(st):
    st = json.loads(json.dumps(st))
    st.pop("elapsed_time", None)
    st.pop("throughput_mb_per_sec", None)
    return st


def gen_files(tmp):
    fdir = os.path.join(HERE, "files")
    os.makedirs(fdir, exist_ok=True)
    manifest = []

    def run(name, data, setup, mode, C, ids, seed, gen):
        src = os.path.join(tmp, name + ".bin")
        dst = os.path.join(fdir, name + ".ambc")
        with open(src, "wb") as f:
            f.write(data)
        with quiet():
            comp = ac.AdaptiveCompressor()
            if ids is not None:
                restrict(comp, ids)
            if C is not None:
                comp.CHUNK_SIZE_CANDIDATES = [C]
            if mode == "native":
                comp._adaptive_compress = per_chunk_harness(comp, C)
            st = comp.compress(src, dst)
            back = os.path.join(tmp, name + ".dec")
            try:
                comp2 = ac.AdaptiveCompressor()
                comp2.decompress(dst, back)
                with open(back, "rb") as f:
                    rt = f.read() == data
                dexc = None
            except Exception as e:  # noqa: BLE001
                rt, dexc = False, f"{type(e).__name__}: {e}"
        with open(dst, "rb") as f:
            blob = f.read()
        manifest.append({"name": name, "file": f"files/{name}.ambc", "setup": setup,
                         "mode": mode, "chunk": C, "methods": ids, "gen": gen, "seed": seed,
                         "size": len(data), "input_sha256": sha(data),
                         "output_sha256": sha(blob), "stats": clean_stats(st),
                         "ref_roundtrip": rt, "ref_decompress_exc": dexc})

    gpu_set = [1, 3, 4, 255]
    for seed, n in ((20250418, 65536), (11, 262144), (12, 100000)):
        data = synth.generate(n, seed)
        for C in (1024, 4096, 8192, 16384):
            run(f"ref_s{seed}_n{n}_c{C}", data, "reference-loop", "reference", C, gpu_set,
                seed, "mixed")
            run(f"nat_s{seed}_n{n}_c{C}", data, "per-chunk-harness", "native", C, gpu_set,
                seed, "mixed")
    data = synth.generate(1 << 20, 20250418)
    run("nat_s20250418_n1048576_c4096", data, "per-chunk-harness", "native", 4096, gpu_set,
        20250418, "mixed")
    run("nat_rle_only_s5_c4096", synth.generate(200000, 5), "per-chunk-harness", "native",
        4096, [1, 255], 5, "mixed")
    run("nat_huff_only_s6_c2048", synth.generate(200000, 6), "per-chunk-harness", "native",
        2048, [3, 255], 6, "mixed")
    # Full default method set {1..7,255}, default 8 candidates, small input.
    run("default_s3_n12288", synth.generate(12288, 3), "default-loop", "default", None,
        None, 3, "mixed")
    run("deflate_set_s4_c4096", synth.generate(65536, 4), "per-chunk-harness", "native",
        4096, [1, 3, 5, 255], 4, "mixed")
    return manifest


def body(*chunks):
    return b"".join(chunks)


def pkg(t, orig, payload, marker=MARKER, used=None):
    used = orig if used is None else used
    return marker + bytes([t, 0]) + struct.pack("<III", used, orig, len(payload)) + payload


END = MARKER + b"\x00\x00" + b"\x00\x00" + b"\x00" * 8


def gen_decode_kat():
    rle, huf = cm.RLECompression(), cm.HuffmanCompression()
    with quiet():
        rle_ab = rle.compress(b"A" * 300 + b"B" * 20)
        huf_txt = huf.compress(b"abracadabra" * 40)
    huf_len = len(b"abracadabra" * 40)
    ascii_ = synth.generate(200000, 7)[140000:140000 + 4096]
    with quiet():
        huf_ascii = huf.compress(ascii_)
    k = huf_txt[0]
    nb_pos = 1 + 5 * k
    short_bits = bytearray(huf_txt)
    short_bits[nb_pos:nb_pos + 4] = struct.pack("<I", 37)
    cases = {
        "raw_exact": (body(pkg(255, 5, b"hello"), END), 5),
        "raw_short_payload_pad": (body(pkg(255, 8, b"hey"), END), 8),
        "raw_long_payload_trunc": (body(pkg(255, 2, b"hello"), pkg(255, 3, b"xyz"), END), 5),
        "rle_basic": (body(pkg(1, 320, rle_ab), END), 320),
        "rle_odd_tail": (body(pkg(1, 10, b"A\x05B\x03C"), END), 10),
        "rle_over": (body(pkg(1, 4, b"A\x05B\x03"), pkg(255, 2, b"zz"), END), 6),
        "rle_empty_payload": (body(pkg(1, 10, b""), pkg(255, 3, b"abc"), END), 13),
        "huff_basic": (body(pkg(3, huf_len, huf_txt), END), huf_len),
        "huff_ascii": (body(pkg(3, 4096, huf_ascii), END), 4096),
        "huff_short_bits": (body(pkg(3, huf_len, bytes(short_bits)), pkg(255, 4, b"tail"), END),
                            huf_len + 4),
        "huff_one_symbol_table": (body(pkg(3, 7, b"\x01A\x07\x00\x00\x00\x07\x00\x00\x00\x00"),
                                       pkg(255, 2, b"ok"), END), 9),
        "huff_zero_table": (body(pkg(3, 6, b"\x00\x00\x00\x00\x00"), pkg(255, 2, b"ok"), END), 8),
        "huff_truncated_table": (body(pkg(3, 6, b"\x03A\x01\x00"), pkg(255, 2, b"ok"), END), 8),
        "huff_dup_symbols": (body(pkg(3, 8, b"\x03A\x03\x00\x00\x00B\x02\x00\x00\x00A\x05\x00\x00\x00"
                                          b"\x0c\x00\x00\x00\x5a\xc0"), pkg(255, 2, b"ok"), END), 10),
        "huff_partial_count": (body(pkg(3, 5, b"\x02A\x03\x00\x00\x00B\x02"), END), 5),
        "huff_empty_payload": (body(pkg(3, 9, b""), pkg(255, 2, b"ok"), END), 11),
        "delta_basic": (body(pkg(4, 6, b"\x05\x01\x01\x01\xff\x00"), END), 6),
        "delta_short": (body(pkg(4, 6, b"\x05\x01"), pkg(255, 3, b"end"), END), 9),
        "delta_long": (body(pkg(4, 2, b"\x05\x01\x01\x01"), pkg(255, 3, b"end"), END), 5),
        "dict_basic": (body(pkg(2, 9, b"\x00a\x00b\x01\x02\x00\x05\x00c"), END), 9),
        "dict_rle_like": (body(pkg(2, 12, b"\x00z\x01\x01\x00\x0b"), END), 12),
        "dict_truncated_match": (body(pkg(2, 6, b"\x00a\x00b\x01\x02"), pkg(255, 2, b"ok"), END), 8),
        "deflate_chunk": (body(pkg(5, 1000, zlib.compress(b"q" * 1000, 9)), END), 1000),
        "deflate_bad": (body(pkg(5, 16, b"not a zlib stream"), pkg(255, 2, b"ok"), END), 18),
        "unknown_type_verbatim": (body(pkg(200, 3, b"abcdef"), pkg(255, 2, b"ok"), END), 8),
        "lz4_type_without_lib": (body(pkg(9, 3, b"xyz"), END), 3),
        "end_chunk_early": (body(pkg(255, 3, b"abc"), END, pkg(255, 3, b"def")), 6),
        "type0_stop": (body(pkg(255, 2, b"ab"), pkg(0, 3, b"xyz"), pkg(255, 2, b"cd")), 4),
        "payload_overrun_stop": (body(pkg(255, 3, b"abc"), MARKER + b"\xff\x00" +
                                      struct.pack("<III", 9, 9, 100) + b"short"), 12),
        "header_cut_short": (body(pkg(255, 3, b"abc"), MARKER + b"\xff\x00\x01"), 3),
        "stop_at_orig_size": (body(pkg(255, 4, b"abcd"), b"\x00garbage-not-a-header-at-all"), 4),
        "orig_size_smaller": (body(pkg(255, 4, b"abcd"), pkg(255, 4, b"efgh"), END), 6),
        "marker_mismatch": (body(pkg(255, 3, b"abc"), b"\x12\x34\x56\x78" + b"\xff\x00" +
                                 struct.pack("<III", 1, 1, 1) + b"z", END), 4),
        "empty_body": (b"", 5),
    }
    res = []
    comp = None
    with quiet():
        comp = ac.AdaptiveCompressor()
        comp._init_marker(MARKER, 32)
    for name, (bd, orig) in cases.items():
        with quiet():
            try:
                out = comp._adaptive_decompress(bd, orig)
                rec = {"ok": True, "out": H(out)}
            except Exception as e:  # noqa: BLE001
                rec = {"ok": False, "exc": type(e).__name__, "msg": str(e)}
        rec.update({"name": name, "body": H(bd), "orig_size": orig})
        res.append(rec)
    return res


def gen_config1(tmp):
    data = synth.random_bytes(1 << 20, 20250418)
    src, dst, back = (os.path.join(tmp, x) for x in ("c1.bin", "c1.ambc", "c1.dec"))
    with open(src, "wb") as f:
        f.write(data)
    with quiet():
        comp = ac.AdaptiveCompressor()
        comp.CHUNK_SIZE_CANDIDATES = [4096]
        st = comp.compress(src, dst)
    with open(dst, "rb") as f:
        blob = f.read()
    try:
        with quiet():
            ac.AdaptiveCompressor().decompress(dst, back)
        exc = None
    except Exception as e:  # noqa: BLE001
        exc = {"type": type(e).__name__, "msg": str(e)}
    return {"seed": 20250418, "size": len(data), "chunk": 4096,
            "input_sha256": sha(data), "output_equals_input": blob == data,
            "stats": clean_stats(st), "decompress_exception": exc}


def main():
    with tempfile.TemporaryDirectory() as tmp:
        jobs = [("codecs.json", gen_codecs), ("huffman_codes.json", gen_huffman_codes),
                ("decode_kat.json", gen_decode_kat),
                ("config1.json", lambda: gen_config1(tmp)),
                ("files.json", lambda: gen_files(tmp))]
        only = set(sys.argv[1:])
        for fname, fn in jobs:
            if only and fname not in only:
                continue
            data = fn()
            with open(os.path.join(HERE, fname), "w") as f:
                json.dump(data, f, indent=1, sort_keys=True)
            print("wrote", fname, file=sys.stderr)
    # provenance of the reference tree the vectors came from
    prov = {"reference": REF, "python": sys.version.split()[0],
            "numpy": __import__("numpy").__version__, "zlib": zlib.ZLIB_VERSION,
            "note": "bitarray replaced by tests/golden/_standin/bitarray.py (test-only)"}
    with open(os.path.join(HERE, "PROVENANCE.json"), "w") as f:
        json.dump(prov, f, indent=1)


if __name__ == "__main__":
    main()
