"""Debug aid: compress an input with the GPU zlib-9 encoder and save the first
id-5 package that differs from zlib.compress(chunk, 9) (chunk + GPU payload)
under gpurun_out/ for offline analysis."""
import os
import sys
import zlib

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adaptive-compression_amd"))
from oracle import synth  # noqa: E402


def main():
    n, seed, chunk = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    methods = tuple(int(x) for x in sys.argv[4].split(","))
    from ambc import AdaptiveCompressor
    data = synth.generate(n, seed)
    comp = AdaptiveCompressor(chunk_size=chunk, mode="native", methods=methods, deflate="zlib9")
    body = comp._adaptive_compress(data)
    pos = off = k = 0
    bad = 0
    while pos + 18 <= len(body) and body[pos + 4] != 0:
        t = body[pos + 4]
        orig = int.from_bytes(body[pos + 10:pos + 14], "little")
        clen = int.from_bytes(body[pos + 14:pos + 18], "little")
        if t == 5:
            raw = data[off:off + orig]
            pay = body[pos + 18:pos + 18 + clen]
            z = zlib.compress(raw, 9)
            if pay != z:
                i = next((j for j in range(min(len(pay), len(z))) if pay[j] != z[j]), min(len(pay), len(z)))
                print(f"chunk {k} off {off} orig {orig}: gpu {len(pay)} zlib {len(z)} first diff {i}")
                if bad == 0:
                    os.makedirs("gpurun_out", exist_ok=True)
                    open(f"gpurun_out/z9dbg_chunk.bin", "wb").write(raw)
                    open(f"gpurun_out/z9dbg_gpu.bin", "wb").write(pay)
                bad += 1
        pos += 18 + clen
        off += orig
        k += 1
    print("packages", k, "bad id-5", bad)


if __name__ == "__main__":
    main()
