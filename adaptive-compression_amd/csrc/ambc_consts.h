// ambc_consts.h -- constants shared by the kernels and the host code (no HIP
// types: the CPU sanitizer harness, tests/native/, includes it too).
#pragma once
#include <stdint.h>

namespace ambc {

constexpr uint32_t HDR = 18;       // chunk header: marker4 type k used4 orig4 clen4
constexpr uint32_t END_CHUNK = 16; // _create_end_chunk (u16 used field)
constexpr uint32_t LZ4_HASH_BITS = 10;   // "ambc-lz4 greedy v2" hash width
constexpr uint32_t ENC_FORCE = 1;    // CompressionMethod.compress(chunk) semantics
constexpr uint32_t ENC_ANALYZE = 2;  // also evaluate every should_use
constexpr uint32_t ENC_EMIT_PENDING = 4;  // emit only the chunks the first pass deferred and id 5 did not take
constexpr uint32_t ENC_RAW_IN_PLACE = 8;  // raw (255) payloads are not copied to the slot: k_compact reads the input
constexpr uint32_t ENC_IN_ALIGNED = 16;   // every chunk starts 16-byte aligned in the input (k_encode may read it in place)
constexpr uint32_t ENC_EVAL = 32;         // decision only (multi-size walk): plen / ids, no payload written
constexpr uint32_t LZ4_SUB_MAX = 8;       // EncArgs::sub_c entries

}  // namespace ambc
