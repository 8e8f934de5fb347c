// Internal launch structures shared by ambc_kernels.hip and ambc_host.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ambc_consts.h"

namespace ambc {


// k_deflate's per-chunk device scratch: the parse's matches (2 cmax bytes), then
// for chunks above 16 KiB the match-start masks (cmax / 8 bytes)
constexpr uint64_t gd_seq_bytes(uint32_t cmax) { return 2ull * cmax + cmax / 8; }

// per-chunk encode: one 64-lane workgroup per chunk
struct EncArgs {
    const uint8_t* in;       // device input
    uint64_t n_total;        // bytes in this shard/job
    uint32_t chunk_size;
    uint32_t n_chunks;
    uint8_t* slots;          // n_chunks * slot_stride scratch payloads
    uint32_t slot_stride;
    uint32_t method_mask;
    uint32_t* plen;          // payload length per chunk
    uint8_t* ids;            // method id per chunk (255 raw)
    uint64_t* sizes;         // 18 + plen per chunk (scan input)
    const double* ent_full;  // optional exact entropy terms (device)
    const double* ent_tail;
    uint8_t* su;             // optional: per-chunk should_use bits (1<<1 RLE, 1<<2 Dictionary, 1<<3 Huffman, 1<<4 Delta)
    uint32_t flags;          // ENC_FORCE: encode with the single enabled method, no gates
    unsigned long long* stamps;  // diagnostic build (-DAMBC_STAMPS): per-phase cycle sums
    uint32_t* bestpre;       // optional: best (len + 18) before LZ4 (k_deflate's threshold)
    uint8_t* gdseq;          // k_deflate: n_chunks x chunk-size scratch for the parse's matches
    uint32_t* z9rec;         // k_z9_parse -> k_z9_code: per-chunk match starts + matches (ambc_zlib9.hip)
    uint8_t* z9scr;          // chunks > 8192: k_z9_parse_big's scratch, z9_scratch_bytes(cmax, n_chunks)
    uint8_t* pending;        // with k_dict / k_deflate: 1 = the RLE/Huffman payload was not emitted (id 2 / 5 may win)
    uint32_t pref_min[16];
    uint32_t pref_max[16];
    const uint64_t* coff;    // optional chunk table (multi-size walk): chunk k = in[coff[k], coff[k] + clen[k])
    const uint32_t* clen;    //   (else chunk k = in[k * chunk_size, ...) clamped to n_total)
    uint32_t clen_all;       //   coff without clen: every chunk is clen_all bytes (the walk's batches)
    // ENC_EVAL + lz4sub: the LZ4 block length of every prefix [0, b) of the chunk
    // for b in sub_c[] (ascending) with b < n and id 9's prefs, from the chunk's
    // own parse ("ambc-lz4 greedy v2" is prefix-consistent: the prefix's parse is
    // the chunk's up to the last match start b - 12, that match capped at b - 5);
    // lz4sub[k * LZ4_SUB_MAX + j] for sub_c[j], others left untouched
    uint32_t* lz4sub;
    uint32_t sub_c[LZ4_SUB_MAX];
    uint32_t n_subc;
    uint32_t kbase;          // index of chunk 0 of this launch within the call
};

// gather the packages into the body at their scanned offsets
struct CompactArgs {
    const uint8_t* slots;
    uint32_t slot_stride;
    const uint32_t* plen;
    const uint8_t* ids;
    const uint64_t* off;     // exclusive scan of sizes (n_chunks+1)
    const uint64_t* base;    // optional: body offset added to off[] (pipelined segments)
    uint32_t n_chunks;       // packages to write
    const uint32_t* clen;    // optional: original length of package k (else clen_all, or chunk_size clamped to n_total)
    uint32_t clen_all;       // nonzero without clen: every package's original length (a walk's final batch)
    uint32_t resident;       // > 0: a grid of this many workgroups striding over the packages
    uint64_t n_total;
    uint32_t chunk_size;
    uint8_t* out;
    const uint8_t* in;       // optional (ENC_RAW_IN_PLACE): raw packages read from in + k * chunk_size
};

// one decode job per chunk package (built by the host header walk)
struct DecJob {
    uint64_t body_off;  // payload offset in body
    uint64_t out_off;   // output offset
    uint64_t scratch_off;  // device scratch for outputs that overshoot orig (~0 = none)
    uint64_t scratch_cap;
    uint32_t clen;
    uint32_t orig;
    uint32_t type;      // method id, or 256 = copy verbatim, 257 = skip (host codec)
    uint32_t expect;    // bytes the host walk assumed this chunk produces
};

struct DecArgs {
    const uint8_t* body;
    uint8_t* out;
    uint64_t out_cap;       // bytes writable in out
    const DecJob* jobs;
    uint32_t n_jobs;
    uint8_t* scratch;
    uint32_t* produced;     // actual produced bytes per job
    unsigned long long* stamps;  // diagnostic build (-DAMBC_STAMPS): per-job phase cycles
    const uint32_t* list;   // job indices this launch decodes (nullptr = 0..n_jobs-1)
    uint32_t n_list;
    const uint16_t* inf_fixed;  // optional: the fixed-Huffman decode tables (launch_inflate_fixed_tables)
};

// decode kernels by LDS footprint (host routes each job to one of them)
enum : int { DEC_KIND_LIGHT = 0, DEC_KIND_LZ4_4K = 1, DEC_KIND_LZ4_8K = 2, DEC_KIND_LZ4_16K = 3,
             DEC_KIND_LZ4_G = 4, DEC_KIND_INFLATE_4K = 5, DEC_KIND_INFLATE_8K = 6,
             DEC_KIND_INFLATE_16K = 7, DEC_KIND_HEAVY = 8, DEC_KIND_DICT_4K = 9, DEC_KIND_DICT_8K = 10,
             DEC_KIND_DICT_16K = 11, DEC_KIND_INFLATE_32K = 12,
             DEC_KIND_INFLATE_G = 13, DEC_KIND_HUFF_4K = 14, DEC_KIND_HUFF_8K = 15, DEC_KINDS = 16 };
// Huffman packages for k_decode_huff<4096|8192> (ambc_huffdec.hip), else k_decode
__host__ __device__ constexpr int huff_kind(uint32_t orig, uint32_t clen) {
    return clen && orig <= 4096 && clen <= 4096 ? DEC_KIND_HUFF_4K
         : clen && orig <= 8192 && clen <= 8192 ? DEC_KIND_HUFF_8K : DEC_KIND_HEAVY;
}
constexpr uint32_t DEC_PRODUCED_HOST = 0xFFFFFFFEu;  // k_decode_inflate: output too large, inflate on host

constexpr uint32_t DEC_VERBATIM = 256;
constexpr uint32_t DEC_SKIP = 257;

// ids with a device decoder; any other REGISTERED id (bz2 6, lzma 7, zstd 8, ...)
// is listed for the caller's host codec (ambc_host_chunk), an unregistered one is
// copied verbatim (adaptive_compressor.py:432-435)
__host__ __device__ constexpr bool device_decodes(uint32_t t) {
    return t == 1 || t == 2 || t == 3 || t == 4 || t == 5 || t == 9 || t == 255;
}

// ---- the device header walk (ambc_walk.hip), one body piece at a time ----
constexpr uint64_t WALK_ENDED = ~0ull;   // WalkState::entry once the walk has stopped
constexpr uint32_t WALK_GRID = 128;      // workgroups of the grid-stride walk kernels (small: they
                                         // share the chip with the decode of the piece before)

// ambc_host_chunk's layout (a package left to a host codec)
struct HostChunk {
    uint64_t body_off, out_off;
    uint32_t clen, orig, type, reserved;
};

struct WalkState {
    uint64_t entry;     // the chain's next header position (WALK_ENDED: stopped)
    uint64_t out;       // output bytes of all jobs so far
    uint64_t scr;       // this piece's scratch bytes
    uint64_t bneed;     // body bytes this piece's jobs read
    uint64_t tot_o, tot_s;
    uint32_t err;       // 1: a header without the marker where the walk reads one
    uint32_t nc, nchain, nj, stop, root;
    uint32_t nhost;     // packages for host codecs so far (all pieces)
    uint32_t pad;
    uint32_t kcount[16], kfill[16];   // jobs per decode kernel (lists in kind order)
    // decode checks (all pieces): a package decoded to another length than its
    // header announced, a job failed, packages the GPU handed back to host zlib
    uint32_t mismatch, failed, nhinf;
};

struct WalkArgs {
    const uint8_t* body;
    uint64_t blen;
    uint64_t a, e;            // candidate header positions [a, e) (bytes up to e + 17 uploaded)
    uint64_t orig_size;
    uint64_t reg[4];          // registered ids
    uint32_t last;            // the body's last piece
    uint32_t ntiles;
    WalkState* st;
    uint32_t* tcnt;           // per 64 KiB tile: candidates -> offsets
    uint64_t* cand;           // candidate positions, ascending
    uint32_t* ja;             // links (successor candidate, or nc: none)
    uint32_t* jb;             // where the path from a node leaves its block
    uint8_t* flg;
    uint8_t* mark;
    uint32_t* bc;             // per block of candidates: entry node, chain nodes -> offsets
    uint32_t* chain;          // the chain's candidates, in order
    uint64_t* olen;           // per chain node: output / scratch bytes
    uint64_t* slen;
    uint64_t* bo;             // per 1024 chain nodes: sums -> offsets
    uint64_t* bs;
    uint8_t* kind;
    DecJob* jobs;             // this piece's jobs, lists (by kind) and produced[]
    uint32_t* list;
    const uint32_t* produced;
    HostChunk* host;          // packages for host codecs (ids 6/7, zlib outside the GPU's domain)
    uint32_t host_cap;
    HostChunk* hinf;          // id-5 packages the GPU inflate handed back
    uint32_t hinf_cap;
    uint32_t nj;              // k_walk_check: the piece's jobs
};
// the walk of one piece on stream s
hipError_t launch_walk_piece(WalkArgs a, hipStream_t s);
// after the piece's decode: produced[] against the jobs' expected lengths
hipError_t launch_walk_check(const WalkArgs& a, hipStream_t s);

// launchers (ambc_kernels.hip)
hipError_t launch_encode(const EncArgs& a, hipStream_t s);
hipError_t launch_deflate(const EncArgs& a, hipStream_t s);   // ambc_deflate.hip
hipError_t launch_dict(const EncArgs& a, uint32_t cmax, hipStream_t s);   // ambc_dict.hip
// DictionaryCompression(window, lookahead) for any window / lookahead / length
// (ambc_dictany.hip): device scratch sized by the dict_any_* helpers
struct DictAnyArgs {
    const uint8_t* in;     // n bytes + 64 zero bytes of padding
    uint32_t n;
    int64_t window, look;  // the plugin's window_size / lookahead_size (clamped to +-2^62)
    uint32_t* tok;         // n: every position's token
    uint64_t* tab;         // dict_any_table_bytes(n): per block and entry offset
    uint64_t* gtab;        // dict_any_gtable_bytes(n): per group and entry offset
    uint32_t* gent;        // groups: entry offset
    uint64_t* gbase;       // groups: output base
    uint32_t* bent;        // blocks: entry offset
    uint64_t* bbase;       // blocks: output base
    uint64_t* res;         // [0] = body bytes | 1 << 63 when a path token is longer than 255 bytes
    uint8_t* out;          // the body (emit)
};
uint32_t dict_any_blocks(uint64_t n);
uint32_t dict_any_groups(uint64_t n);
uint64_t dict_any_table_bytes(uint64_t n);
uint64_t dict_any_gtable_bytes(uint64_t n);
hipError_t launch_dict_any_parse(const DictAnyArgs& a, hipStream_t s);
hipError_t launch_dict_any_emit(const DictAnyArgs& a, hipStream_t s);
// single-call plugins at any length (ambc_anylen.hip): blocks of 4 KiB, n < 2^32
uint32_t any_blocks(uint64_t n);
hipError_t launch_delta_any(const uint8_t* d, uint64_t n, uint8_t* out, hipStream_t s);
hipError_t launch_rle_any_count(const uint8_t* d, uint64_t n, int64_t* carry, int64_t* cnt, hipStream_t s);
hipError_t launch_rle_any_emit(const uint8_t* d, uint64_t n, const int64_t* carry, int64_t* cnt, uint32_t* pos,
                               uint64_t np, uint8_t* out, hipStream_t s);
hipError_t launch_huff_any_hist(const uint8_t* d, uint64_t n, uint32_t* hist, uint32_t* first, hipStream_t s);
hipError_t launch_huff_any_tree(const uint32_t* hist, const uint32_t* first, uint64_t* codes, uint8_t* hdr, int32_t* info,
                                hipStream_t s);
hipError_t launch_huff_any_bits(const uint8_t* d, uint64_t n, const uint64_t* codes, int64_t* bb, uint32_t* be,
                                uint64_t nbytes, uint8_t* out, hipStream_t s);
hipError_t launch_su_samples(const uint8_t* d, uint64_t n, uint64_t step, uint32_t* out2, hipStream_t s);
hipError_t launch_lz4_assemble(const uint8_t* slots, uint64_t stride, const uint32_t* plen, const uint64_t* off,
                               uint32_t m, uint64_t n, uint8_t* out, hipStream_t s);
// id 5 as zlib.compress(data, 9) (ambc_zlib9.hip): chunk_size <= z9 limit; the
// record scratch is n_chunks x z9_rec_words(z9_cmax(chunk_size)) u32 words
uint32_t z9_cmax(uint32_t chunk);   // 0: no zlib-9 encoder for this chunk size
size_t z9_rec_words(uint32_t cmax);
// chunks above 8192 (ambc_zlib9_big.hip) also need EncArgs::z9scr
size_t z9_scratch_bytes(uint32_t cmax, uint32_t n_chunks);
size_t z9_rec_words_big(uint32_t cmax);
hipError_t launch_zlib9_big(const EncArgs& a, hipStream_t s);
hipError_t launch_zlib9(const EncArgs& a, hipStream_t s);
// the small-chunk zlib-9 path in two parts: the parse, then trees + emission (chunks <= 8 KiB)
hipError_t launch_zlib9_parse(const EncArgs& a, hipStream_t s);
hipError_t launch_zlib9_tail(const EncArgs& a, hipStream_t s);
hipError_t launch_compact(const CompactArgs& a, hipStream_t s);
hipError_t launch_end_chunk(uint8_t* dst, hipStream_t s);
// out == null: only *off into acc_slot[0]
hipError_t launch_end_chunk_at(uint8_t* out, const uint64_t* off, uint64_t* acc_slot, hipStream_t s);
// base[1] = base[0] + off_last[0] + size_last[0] (a pipelined segment's end offset)
hipError_t launch_seg_base(uint64_t* base, const uint64_t* off_last, const uint64_t* size_last, hipStream_t s);
hipError_t launch_stats(const uint8_t* ids, const uint32_t* plen, uint32_t n_chunks,
                        uint64_t n_total, uint32_t chunk_size, uint64_t* acc, hipStream_t s);
hipError_t scan_sizes(const uint64_t* sizes, uint64_t* off, uint32_t count, void* tmp,
                      size_t* tmp_bytes, hipStream_t s);
hipError_t launch_copy(uint8_t* dst, const uint8_t* src, uint64_t len, hipStream_t s);
hipError_t launch_results_to_host(const uint32_t* plen, const uint8_t* ids, const uint32_t* lz, uint32_t cnt, uint32_t nlz,
                                  uint32_t* hplen, uint8_t* hids, uint32_t* hlz, hipStream_t s);
hipError_t launch_decode(int kind, const DecArgs& a, hipStream_t s);
hipError_t launch_inflate(int kind, const DecArgs& a, hipStream_t s);   // ambc_inflate.hip
hipError_t launch_huff(int kind, const DecArgs& a, hipStream_t s);      // ambc_huffdec.hip
// the fixed-Huffman (btype 1) decode tables, built once per device into out
constexpr int INF_LUTB = 9;   // primary lookup bits of the inflate tables (longer codes: canonical search)
constexpr size_t INF_FIXED_U16 = 2 * (1 << INF_LUTB) + 2 * 288 + 3 * 2 * 16;
hipError_t launch_inflate_fixed_tables(uint16_t* out, hipStream_t s);
// bytes [lo, hi) of the synthetic stream (segment table seg) into out[0, hi - lo)
hipError_t launch_synth(uint8_t* out, uint64_t lo, uint64_t hi, const uint64_t* seg, uint32_t nseg,
                        uint64_t seed, hipStream_t s);
hipError_t launch_equal(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t* neq, hipStream_t s);

}  // namespace ambc
