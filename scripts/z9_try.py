import sys, zlib, time
sys.path[:0] = ["/root/repo", "/root/repo/adaptive-compression_amd"]
from oracle import oracle as orc, synth
from ambc import AdaptiveCompressor
for n, chunk, methods in [(1 << 20, 4096, (5,)), (1 << 20, 4096, (1, 3, 4, 5)), (300000, 1024, (1, 3, 5, 9)), (500000, 2048, (5, 9))]:
    data = synth.generate(n, 7)
    for mode in ("native", "reference"):
        comp = AdaptiveCompressor(chunk_size=chunk, mode=mode, methods=methods, deflate="zlib9")
        body = comp._adaptive_compress(data)
        ref, st = orc.compress_body(data, orc.make_params(chunk, mode, methods, n_total=n, deflate="zlib"), nthreads=0)
        print(n, chunk, methods, mode, "equal" if body == ref else "DIFF", len(body), len(ref), flush=True)
        if body != ref:
            # first differing package
            pos = 0
            while pos + 18 <= min(len(body), len(ref)):
                if body[pos:pos+18] != ref[pos:pos+18] or True:
                    cl = int.from_bytes(body[pos+14:pos+18], "little"); cr = int.from_bytes(ref[pos+14:pos+18], "little")
                    if body[pos:pos+18+cl] != ref[pos:pos+18+cr]:
                        print("  pkg at", pos, "types", body[pos+4], ref[pos+4], "clen", cl, cr); break
                    pos += 18 + cl
        assert comp._adaptive_decompress(body, n) == data
