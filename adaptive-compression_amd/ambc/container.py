"""The .ambc container header (adaptive_compressor.py:196-219,303-358).

Layout (little-endian): 'AMBC' | version u8 = 2 | header_size u32 | marker_len
u8 | marker bytes | checksum_type u8 (1 = MD5) | MD5[16] | original_size u64 |
compressed_size u64 (= body length incl. the 16-byte end chunk).
"""
import struct

MAGIC_NUMBER = b"AMBC"
FORMAT_VERSION = 2
# _find_marker (adaptive_compressor.py:303-310): constant bitarray('1'*16 + '0'*16)
MARKER_BYTES = b"\xff\xff\x00\x00"
MARKER_LENGTH = 32


def marker_bytes_aligned(marker_bytes, marker_length):
    """_init_marker (adaptive_compressor.py:196-219)."""
    bits = "".join(format(b, "08b") for b in marker_bytes)[:marker_length]
    if marker_length <= 8:
        return bytes([int(bits or "0", 2) << (8 - marker_length)])
    while len(bits) % 8:
        bits += "0"
    return bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))


def build_header(marker_bytes, marker_len, checksum, original_size):
    """_build_header (adaptive_compressor.py:312-325)."""
    hdr = bytearray()
    hdr += MAGIC_NUMBER
    hdr.append(FORMAT_VERSION)
    hdr += b"\x00\x00\x00\x00"
    hdr.append(marker_len)
    hdr += marker_bytes
    hdr.append(1)
    hdr += checksum
    hdr += struct.pack("<Q", original_size)
    hdr += b"\x00" * 8
    hdr[5:9] = struct.pack("<I", len(hdr))
    return bytes(hdr)


def update_compressed_size(hdr, csize):
    """_update_header_compressed_size (adaptive_compressor.py:327-330)."""
    hdr = bytearray(hdr)
    hdr[-8:] = struct.pack("<Q", csize)
    return bytes(hdr)


def parse_header(data):
    """_parse_header (adaptive_compressor.py:332-358), same exceptions."""
    if data[:4] != MAGIC_NUMBER:
        raise ValueError("Magic mismatch")
    version = data[4]
    if version > FORMAT_VERSION:
        raise ValueError(f"Unsupported version: {version}")
    hdr_size = struct.unpack("<I", data[5:9])[0]
    marker_len = data[9]
    msize = (marker_len + 7) // 8
    marker = data[10:10 + msize]
    ctype = data[10 + msize]
    csum_size = 16 if ctype == 1 else 0
    csum = data[11 + msize:11 + msize + csum_size]
    orig_pos = 11 + msize + csum_size
    orig_size = struct.unpack("<Q", data[orig_pos:orig_pos + 8])[0]
    comp_pos = orig_pos + 8
    comp_size = struct.unpack("<Q", data[comp_pos:comp_pos + 8])[0]
    return {"format_version": version, "header_size": hdr_size, "marker_length": marker_len,
            "marker_bytes": marker, "checksum_type": ctype, "checksum": csum,
            "original_size": orig_size, "compressed_size": comp_size}
