"""Method ids, names, chunk-size preferences and routing tables.

Mirrors the reference's tables (adaptive_compressor.py:97-127) and records
which ids the MI355X path encodes and decodes.
"""

# adaptive_compressor.py:97-110
METHOD_NAMES = {
    1: "RLE", 2: "Dictionary", 3: "Huffman", 4: "Delta", 5: "DEFLATE", 6: "BZIP2", 7: "LZMA",
    8: "ZStandard", 9: "LZ4", 10: "Brotli", 11: "LZHAM", 255: "No Compression",
}

# adaptive_compressor.py:114-127 (min, max) chunk size per method
METHOD_CHUNK_PREFS = {
    1: (32, 4096), 2: (128, 8192), 3: (32, 8192), 4: (32, 4096), 5: (64, 65536),
    6: (1024, 262144), 7: (8192, 524288), 8: (512, 262144), 9: (1024, 65536),
    10: (1024, 262144), 11: (1024, 262144), 255: (1, 999999999),
}

# the reference's default candidate list (adaptive_compressor.py:61-62)
REFERENCE_CHUNK_SIZE_CANDIDATES = [131072, 65536, 32768, 16384, 8192, 4096, 2048, 1024]

# selector candidates with a gfx950 encoder; id 5 is "ambc-deflate v1" (a valid
# zlib stream, not zlib level-9 bytes) or zlib-9's own bytes, chunk_size <= 65536; id 2 (the reference's
# own Dictionary bytes) takes chunks <= 8192, its preferred maximum
GPU_ENCODE_IDS = (1, 2, 3, 4, 5, 9)
DEVICE_DECODE_IDS = (1, 2, 3, 4, 9, 255)
# ids whose ENCODERS are host libraries in the reference (zlib / bz2 / lzma / zstd);
# on the decode side id 5 is inflated on the GPU (k_decode_inflate), ids 6 / 7 / 8
# by the reference's library wrappers on the host (id 8 through the system libzstd)
HOST_LIBRARY_IDS = (5, 6, 7, 8)
# ids the walk scores on the host (the reference's bz2 / lzma / zstd wrappers, no
# GPU encoder): AdaptiveCompressor(methods=(..., 6, 7, 8)) in reference mode or
# with several CHUNK_SIZE_CANDIDATES -- see hostcodecs.py
HOST_SCORED_IDS = (6, 7, 8)
DEFAULT_METHODS = (1, 3, 4, 9)         # + 255 always
DEFAULT_CHUNK_SIZE = 4096


def method_mask(ids):
    m = 0
    for i in ids:
        if i == 255:
            continue
        if i not in GPU_ENCODE_IDS:
            raise ValueError(f"method id {i} has no GPU encoder (GPU ids: {GPU_ENCODE_IDS})")
        m |= 1 << i
    return m
