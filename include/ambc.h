/*
 * ambc.h -- C-ABI of libambc_hip.so, the MI355X (gfx950) implementation of the
 * per-chunk method-selection + encode/decode loop of
 * KalharPandya/adaptive-compression's AdaptiveCompressor.
 *
 * The reference has no FFI of its own (it is pure Python).  These entry points
 * replace its two hot loops, exactly where SURVEY.md §8(b) places the boundary:
 *
 *   ambc_compress_batch    replaces AdaptiveCompressor._adaptive_compress
 *                          (adaptive_compressor.py:363-394) together with
 *                          _pick_best_chunk_and_method (:537-590),
 *                          _process_chunk (:631-700), _create_chunk (:609-621)
 *                          and _create_end_chunk (:595-607): input bytes in,
 *                          .ambc body (chunk packages + 16-B end chunk) out.
 *   ambc_decompress_batch  replaces AdaptiveCompressor._adaptive_decompress
 *   ambc_decompress_ex     (adaptive_compressor.py:396-454): body in, original
 *                          bytes out, with the reference's lenient rules.
 *   ambc_compress_bound    worst-case body size (n + 18*ceil(n/C) + 16).
 *
 * The 47-byte header, MD5 and the whole-file raw fallback
 * (adaptive_compressor.py:221-255,312-358) stay in the Python host layer
 * (adaptive-compression_amd/ambc/compressor.py); see INTEGRATION.md for the
 * ctypes binding a maintainer adds to the reference.
 *
 * Conventions: every buffer is caller-allocated; the library never keeps a
 * pointer after a call returns.  Calls block; ctypes releases the GIL around
 * them.  One ambc_ctx per host thread.  Return 0 on success, a negative
 * AMBC_E* code otherwise; ambc_last_error() gives a thread-local message.
 * There is no CPU fallback: without a usable gfx950 device ambc_init fails.
 */
#ifndef AMBC_H
#define AMBC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMBC_ABI_VERSION 3

#define AMBC_OK 0
#define AMBC_E_INVAL (-1)     /* bad argument */
#define AMBC_E_DEVICE (-2)    /* HIP runtime error / no gfx950 device */
#define AMBC_E_NOMEM (-3)     /* device or pinned allocation failed */
#define AMBC_E_RANGE (-4)     /* a u32 chunk field would overflow (reference: struct.error) */
#define AMBC_E_MARKER (-5)    /* "Marker mismatch in chunk header." (reference ValueError) */
#define AMBC_E_CAPACITY (-6)  /* output buffer too small */
#define AMBC_E_HOSTCODEC (-7) /* body holds packages for host codecs (ids 6/7/8): use ambc_decompress_ex */
#define AMBC_E_CODEC (-8)     /* the codec raises in the reference (e.g. Huffman on 1 or 256 symbols) */
#define AMBC_E_COMM (-9)      /* RCCL error, or another rank / shard of the call failed */

#define AMBC_MODE_NATIVE 0    /* every C-byte chunk decided independently */
#define AMBC_MODE_REFERENCE 1 /* CHUNK_SIZE_CANDIDATES=[C] loop incl. the remainder-raw rule */

#define AMBC_FLAG_NO_END_CHUNK 1u /* shard bodies for multi-GPU reassembly */
#define AMBC_FLAG_ZLIB9 2u        /* id 5 = zlib.compress(data, 9)'s own bytes (the reference's,
                                     advanced_compression.py:76-81; chunk_size <= 65536) instead
                                     of "ambc-deflate v1" */
#define AMBC_FLAG_INPUT_PADDED 4u /* device-resident calls: at least 64 readable bytes follow the
                                     input (chunks >= 4 KiB are then read in place instead of
                                     through an LDS copy; host-fed calls always qualify) */

/* GPU-routable method ids (bit i of method_mask = method id i) */
#define AMBC_M_RLE 1
#define AMBC_M_DICT 2  /* GPU encoder k_dict: the reference's bytes; batched chunks <= 8192 (any length: ambc_dict_encode) */
#define AMBC_M_HUFFMAN 3
#define AMBC_M_DELTA 4 /* never selected: payload length == n (compression_methods.py:598-608) */
#define AMBC_M_DEFLATE 5 /* GPU encoder "ambc-deflate v1" (chunk_size <= 65536) or zlib-9 (AMBC_FLAG_ZLIB9,
                           <= 65536); decode: GPU inflate (packages <= 65536) */
#define AMBC_M_LZ4 9
#define AMBC_M_RAW 255

#define AMBC_MAX_CHUNK 65536u

typedef struct ambc_ctx ambc_ctx;

typedef struct {
    uint32_t chunk_size;    /* C: 16 <= C <= 65536, multiple of 16 */
    uint32_t mode;          /* AMBC_MODE_* */
    uint32_t method_mask;   /* enabled method ids (bits 1..15) */
    uint32_t flags;         /* AMBC_FLAG_* */
    uint32_t pref_min[16];  /* method_chunk_prefs (adaptive_compressor.py:114-127) */
    uint32_t pref_max[16];
    /* Optional numpy-exact entropy terms p*np.log2(p) indexed by count
     * (HuffmanCompression.should_use, compression_methods.py:566-574): the
     * encoder sums them in place of a device log2 per symbol, and near the 7.0
     * threshold (within 1e-9) re-adds them in numpy's first-occurrence order.
     * NULL: the device log2 is used for both. */
    const double* ent_full; /* n == chunk_size, length chunk_size+1 */
    const double* ent_tail; /* n == total % chunk_size, length (total % chunk_size)+1 */
} ambc_params;

typedef struct {
    uint64_t method_usage[256]; /* compressed chunks per method id (stats dict) */
    uint64_t total_chunks, compressed_chunks, raw_chunks;
    uint64_t bytes_saved, payload_bytes, overhead_bytes;
    uint64_t kernel_ns;  /* device time of the kernels (hipEvents) */
    uint64_t h2d_ns, d2h_ns, walk_ns, total_ns;
    uint64_t host_codec_ns; /* decode: id-5 (zlib) chunks inflated on host threads */
} ambc_stats;

/* A chunk the library leaves to the caller: a registered id without a device
 * decoder (6 bz2, 7 lzma, 8 zstd, ...; id 5 zlib chunks the GPU cannot inflate
 * are inflated inside the library on host threads). */
typedef struct {
    uint64_t body_off; /* payload offset in the body */
    uint64_t out_off;  /* where its decoded bytes go in the output */
    uint32_t clen;     /* payload length */
    uint32_t orig;     /* original_length field */
    uint32_t type;
    uint32_t reserved;
} ambc_host_chunk;

int ambc_abi_version(void);
const char* ambc_last_error(void);

int ambc_device_count(int* count);
int ambc_init(const int* device_ids, int n_devices, ambc_ctx** out);
void ambc_destroy(ambc_ctx* ctx);

uint64_t ambc_compress_bound(uint64_t n, uint32_t chunk);

/* Host buffers in, host buffers out (H2D -> kernels -> D2H). */
int ambc_compress_batch(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p,
                        uint8_t* out, uint64_t out_cap, uint64_t* out_len, ambc_stats* st);

/* The reference's multi-size walk (several CHUNK_SIZE_CANDIDATES): replaces
 * _adaptive_compress (adaptive_compressor.py:363-394) with
 * _pick_best_chunk_and_method (:537-590) when CHUNK_SIZE_CANDIDATES holds more
 * than one size.  cands[0..n_cands) in the reference's list order (each in
 * [1, 131072]); p supplies method_mask and the prefs (chunk_size and mode are
 * ignored).  ent_sizes/ent_tabs: optional numpy-exact p*log2(p) tables for the
 * chunk sizes Huffman may take (see ambc_params.ent_full).  Writes the .ambc
 * body (packages + end chunk); AMBC_E_INVAL when a size the walk needs has an
 * eligible method the GPU encoders do not take at that size (Dictionary > 8192,
 * any > 65536), AMBC_E_RANGE for a raw remainder > 4 GiB.  out == NULL: the
 * body stays on the device, *out_len gives its size, and ambc_fetch_body copies
 * it out (a caller can then allocate exactly the body's size). */
int ambc_compress_multisize(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p,
                            const uint32_t* cands, uint32_t n_cands, const uint32_t* ent_sizes,
                            const double* const* ent_tabs, uint32_t n_ent, uint8_t* out,
                            uint64_t out_cap, uint64_t* out_len, ambc_stats* st);
/* Host-scored methods for the walk: the reference's library codecs without a GPU
 * encoder (bz2 / lzma, ids 6 / 7: advanced_compression.py:112-213), evaluated by
 * the caller.  eval: for the (position, size) pairs of one walk round, id[i] =
 * the host method that wins size[i] bytes at pos[i] among the host codecs (ids
 * ascending, strict "<" on len + 18, only below len + 18 < size; 0: none) and
 * len[i] its payload bytes.  emit: a host-won package's payload (len bytes) into
 * dst.  Both return 0, or nonzero to fail the call (AMBC_E_CODEC). */
typedef struct {
    int (*eval)(void* user, const uint64_t* pos, const uint32_t* size, uint32_t count, uint8_t* id,
                uint32_t* len);
    int (*emit)(void* user, uint64_t pos, uint32_t size, uint8_t id, uint8_t* dst, uint32_t len);
    void* user;
} ambc_host_codecs;

/* ambc_compress_multisize with host-scored methods beside the GPU's (hc may be
 * NULL): at every size the host winner joins the GPU's in id order (the smaller
 * len; a tie to the lower id).  CHUNK_SIZE_CANDIDATES = [C] is the reference
 * loop of reference mode. */
int ambc_compress_multisize_ex(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p,
                               const uint32_t* cands, uint32_t n_cands, const uint32_t* ent_sizes,
                               const double* const* ent_tabs, uint32_t n_ent, const ambc_host_codecs* hc,
                               uint8_t* out, uint64_t out_cap, uint64_t* out_len, ambc_stats* st);

/* the body the last ambc_compress_multisize(out = NULL) left on the device into
 * out (cap >= its size); AMBC_E_INVAL when there is none */
int ambc_fetch_body(ambc_ctx* ctx, uint8_t* out, uint64_t cap);
/* of the last ambc_compress_multisize: batched evaluation rounds, chunk encodes,
 * wall time of the walks and of the final encode + body assembly */
int ambc_last_multisize_info(ambc_ctx* ctx, uint32_t* steps, uint64_t* evaluated, uint64_t* walk_ns,
                             uint64_t* emit_ns);

int ambc_decompress_batch(ambc_ctx* ctx, const uint8_t* body, uint64_t body_len,
                          uint64_t orig_size, uint8_t* out, ambc_stats* st);

/* As ambc_decompress_batch; packages of registered ids without a device decoder
 * (6 bz2, 7 lzma, 8 zstd, ...) are not decoded but listed in host_chunks
 * (capacity host_cap, count in *n_host) for the caller to fill.
 * registered[id>>6] bit (id&63) marks ids with a registered method
 * (method_lookup); an unregistered id's payload is copied verbatim
 * (adaptive_compressor.py:432-435).  NULL registered = {1,2,3,4,5,6,7,9,255}. */
int ambc_decompress_ex(ambc_ctx* ctx, const uint8_t* body, uint64_t body_len, uint64_t orig_size,
                       const uint64_t registered[4], uint8_t* out, ambc_host_chunk* host_chunks,
                       uint32_t host_cap, uint32_t* n_host, ambc_stats* st);

/* Multi-GPU decode: cut the body at package boundaries into
 * nparts ranges of about orig_size / nparts decoded bytes (the reference's
 * header walk with each package's expected length, adaptive_compressor.py:
 * 396-454).  body_off / out_off hold nparts + 1 entries; part r is body bytes
 * [body_off[r], body_off[r+1]) decoding to output bytes [out_off[r],
 * out_off[r+1]); empty parts have equal offsets.  Host code only (no device). */
int ambc_split_body(const uint8_t* body, uint64_t body_len, uint64_t orig_size,
                    const uint64_t registered[4], uint32_t nparts, uint64_t* body_off,
                    uint64_t* out_off);

/* As ambc_decompress_ex, but the decoded bytes stay in device memory d_out
 * (orig_size bytes on device dev); AMBC_E_HOSTCODEC if any package needs a host
 * codec.  stats->payload_bytes = bytes the packages produced before the final
 * pad / truncate (equal to orig_size for a well-formed body). */
int ambc_decompress_device(ambc_ctx* ctx, int dev, const uint8_t* body, uint64_t body_len,
                           uint64_t orig_size, const uint64_t registered[4], void* d_out,
                           ambc_stats* st);

/* Device-resident variants (inputs already in HBM; used by bench.py and the
 * multi-GPU path).  dev = index into the ctx's device list; stream may be NULL. */
int ambc_compress_device(ambc_ctx* ctx, int dev, const void* d_in, uint64_t n,
                         const ambc_params* p, void* d_out, uint64_t out_cap, uint64_t* out_len,
                         ambc_stats* st, void* stream);

/* Single-chunk plugin calls (CompressionMethod API, compression_methods.py:7-67).
 * ambc_encode_method = method.compress(chunk) for id 1, 2, 3, 4 or 9 (n <= 65536; id 2: n <= 8192),
 * no gates; AMBC_E_CODEC where the reference raises.  ambc_analyze returns, per
 * C-byte chunk, the winning id, its payload length and the should_use bits
 * (1<<1 RLE, 1<<2 Dictionary, 1<<3 Huffman, 1<<4 Delta) the selector evaluated. */
int ambc_encode_method(ambc_ctx* ctx, int method_id, const uint8_t* in, uint32_t n, uint8_t* out,
                       uint32_t out_cap, uint32_t* out_len);
int ambc_analyze(ambc_ctx* ctx, const uint8_t* in, uint64_t n, const ambc_params* p, uint8_t* ids,
                 uint32_t* payload_len, uint8_t* should_use);
/* DictionaryCompression(window_size, lookahead_size).compress(data) for any
 * window, lookahead and length n < 2^32 - 2^24 (replaces compression_methods.py:
 * 187-233 with :279-313; the lookahead is Python's slice data[pos:pos+lookahead],
 * window <= 0 finds no match).  AMBC_E_CODEC where the reference raises (a
 * match longer than 255 bytes reaches bytearray.append), AMBC_E_CAPACITY with
 * *out_len = the body's size when out_cap is short. */
int ambc_dict_encode(ambc_ctx* ctx, const uint8_t* in, uint64_t n, int64_t window_size,
                     int64_t lookahead_size, uint8_t* out, uint64_t out_cap, uint64_t* out_len);
/* method.compress(data) for RLE (1), Huffman (3), Delta (4) and LZ4 (9) at any
 * length n < 2^32 - 2^24, where ambc_encode_method takes one chunk of at most
 * 65536 bytes (replaces compression_methods.py:78-113, 358-405, 586-607 and
 * advanced_compression.py:266-281; LZ4: one frame of independent 64 KiB blocks,
 * the same bytes as ambc_encode_method up to 64 KiB).  AMBC_E_CODEC where the
 * reference raises (Huffman on 1 or 256 distinct bytes), AMBC_E_RANGE where its
 * 4-byte bit count overflows, AMBC_E_CAPACITY with *out_len = the size. */
int ambc_encode_any(ambc_ctx* ctx, int method_id, const uint8_t* in, uint64_t n, uint8_t* out,
                    uint64_t out_cap, uint64_t* out_len);
/* should_use statistics at any length (compression_methods.py:154-180, 540-574,
 * 640-667): stats[0] = pairs i = 0, step, 2 step, ... < n - 1 with
 * data[i] == data[i + 1], stats[1] = those with |data[i] - data[i + 1]| < 32,
 * stats[2 + b] = count of byte b, stats[258 + b] = its first position
 * (0xFFFFFFFF: absent). */
int ambc_analyze_any(ambc_ctx* ctx, const uint8_t* in, uint64_t n, uint64_t step, uint32_t* stats);

/* ---------------------------------------------------------------------------
 * Multi-GPU.  The reference is single-threaded
 * (adaptive_compressor.py:363-394); native-mode chunks are independent, so the
 * input shards into contiguous chunk ranges: rank r of W owns chunks
 * [M*r/W, M*(r+1)/W) of the M = ceil(n_total/C) chunks (ambc_shard_range).
 * Exchanges, all RCCL over xGMI: AllGather of the per-rank body sizes (file
 * offsets), AllReduce(SUM) of the statistics, reference mode's AllReduce(MIN) of
 * the first chunk with no winner (the remainder-raw rule is global,
 * adaptive_compressor.py:586-588), and optionally a grouped Send/Recv gather of
 * the bodies into file order on rank 0.
 *
 * Process per GPU: rank 0 calls ambc_comm_unique_id, the caller hands the 128
 * bytes to every rank (ambc.comm does it over TCP), each rank calls
 * ambc_comm_init_rank on a one-device ctx.  Without ambc_comm_init_rank a ctx
 * is one rank of one.  In one process, ambc_compress_batch /
 * ambc_decompress_multi on a ctx with several devices run one host thread per
 * device (ncclCommInitAll over distinct devices; a ctx listing a device twice
 * holds several shards on that GPU and exchanges through host memory).
 * ------------------------------------------------------------------------- */
#define AMBC_COMM_ID_BYTES 128
#define AMBC_OP_SUM 0
#define AMBC_OP_MIN 1
#define AMBC_OP_MAX 2

typedef struct {
    uint64_t local_len;   /* bytes this rank produced (its packages / decoded range) */
    uint64_t offset;      /* where they sit in the file-order body / output */
    uint64_t total;       /* bytes of the whole body (end chunk included) / output */
    uint64_t shard_begin; /* compress: input bytes [begin, end) of this rank */
    uint64_t shard_end;   /* decompress: body bytes [begin, end) it decoded */
} ambc_shard_info;

int ambc_comm_unique_id(uint8_t* id);  /* AMBC_COMM_ID_BYTES bytes; host only */
int ambc_comm_init_rank(ambc_ctx* ctx, int nranks, int rank, const uint8_t* id);
int ambc_comm_size(ambc_ctx* ctx, int* nranks, int* rank);
int ambc_comm_barrier(ambc_ctx* ctx);  /* AllReduce of one word + device synchronize */
int ambc_comm_allreduce_u64(ambc_ctx* ctx, uint64_t* v, uint32_t k, int op);
int ambc_comm_allgather_u64(ambc_ctx* ctx, const uint64_t* mine, uint32_t k, uint64_t* all);
/* every rank's d_src (len bytes) into file order in rank 0's d_dst (grouped
 * ncclSend/ncclRecv); *offset = this rank's offset, *total = all bytes */
int ambc_comm_gather(ambc_ctx* ctx, const void* d_src, uint64_t len, void* d_dst, uint64_t dst_cap,
                     uint64_t* offset, uint64_t* total);

/* [*begin, *end) = input bytes of rank `rank` (host only) */
int ambc_shard_range(uint64_t n_total, uint32_t chunk, int nranks, int rank, uint64_t* begin, uint64_t* end);

/* This rank's shard (d_shard = input bytes [begin, end) of ambc_shard_range on
 * the device) of an n_total-byte input.  root 0: rank 0's d_out receives the
 * whole body in file order (its own packages first; out_cap >= the body);
 * root -1: every rank keeps its packages, info->offset places them.  The last
 * rank's packages end with the 16-B end chunk (unless AMBC_FLAG_NO_END_CHUNK).
 * st = statistics of the whole body (AllReduce SUM).  The result equals
 * ambc_compress_batch of the whole input on one GPU, byte for byte, in both modes. */
int ambc_compress_shard(ambc_ctx* ctx, const void* d_shard, uint64_t n_total, const ambc_params* p, void* d_out,
                        uint64_t out_cap, int root, ambc_shard_info* info, ambc_stats* st);

/* Decode across the ranks; every rank passes the whole host body.  root 0:
 * rank 0's d_out (out_cap >= orig_size) receives the whole output; root -1:
 * every rank keeps its decoded range (info->offset / local_len).  A body whose
 * packages decode to other lengths than their headers announce is decoded by
 * rank 0 alone (root 0; root -1 fails with AMBC_E_INVAL). */
int ambc_decompress_shard(ambc_ctx* ctx, const uint8_t* body, uint64_t body_len, uint64_t orig_size,
                          const uint64_t registered[4], void* d_out, uint64_t out_cap, int root,
                          ambc_shard_info* info, ambc_stats* st);

/* In-process decode over all devices of the ctx into the host buffer out
 * (each device decodes a range and copies it back at its offset). */
int ambc_decompress_multi(ambc_ctx* ctx, const uint8_t* body, uint64_t body_len, uint64_t orig_size,
                          const uint64_t registered[4], uint8_t* out, ambc_stats* st);

/* memory / device helpers (so the Python layer needs no PyTorch) */
void* ambc_host_alloc(uint64_t bytes);        /* pinned */
void ambc_host_free(void* p);
void* ambc_device_alloc(ambc_ctx* ctx, int dev, uint64_t bytes);
void ambc_device_free(ambc_ctx* ctx, int dev, void* p);
int ambc_memcpy_h2d(ambc_ctx* ctx, int dev, void* d_dst, const void* h_src, uint64_t bytes);
int ambc_memcpy_d2h(ambc_ctx* ctx, int dev, void* h_dst, const void* d_src, uint64_t bytes);
int ambc_memcpy_d2d(ambc_ctx* ctx, int dev, void* d_dst, const void* d_src, uint64_t bytes);
int ambc_memset_device(ambc_ctx* ctx, int dev, void* d_dst, int value, uint64_t bytes);
int ambc_synchronize(ambc_ctx* ctx, int dev);

/* "ambc-mixed v1" synthetic input: host fill and device fill */
void ambc_synth_fill(uint8_t* out, uint64_t n, uint64_t seed);
int ambc_synth_device(ambc_ctx* ctx, int dev, void* d_out, uint64_t n, uint64_t seed);
/* bytes [begin, end) of the n_total-byte stream into d_out[0, end - begin) (a rank's shard) */
int ambc_synth_device_range(ambc_ctx* ctx, int dev, void* d_out, uint64_t n_total, uint64_t begin,
                            uint64_t end, uint64_t seed);
/* *equal = (the n bytes at a and b on device dev are identical) */
int ambc_device_equal(ambc_ctx* ctx, int dev, const void* a, const void* b, uint64_t n, int* equal);

/* bench instrumentation: device time (ns) of the last compress call's encode
 * launches (k_encode and, when enabled, k_dict / k_deflate), measured with HIP
 * events on the stream they were launched on, and of the scan / compaction the
 * encode did not hide.  A native-mode call over >= 16384 chunks runs as
 * n_launch pipelined segments (segment i+1 encodes while segment i is
 * compacted on a second stream): encode_ns spans all of them. */
int ambc_last_kernel_times(ambc_ctx* ctx, int dev, uint64_t* encode_ns, uint64_t* scan_ns,
                           uint64_t* compact_ns);
int ambc_last_encode_launches(ambc_ctx* ctx, int dev, uint32_t* n_launch);

/* diagnostics, host code only: the threaded host header walk of the decode path
 * (used for bodies below the device walk's size and for the lenient re-walk) over
 * a host body -> packages, output bytes, wall ns (threads 0 = default);
 * AMBC_E_MARKER where _adaptive_decompress would raise */
int ambc_debug_walk(const uint8_t* body, uint64_t body_len, uint64_t orig_size, uint32_t threads,
                    uint64_t* n_pkgs, uint64_t* total, uint64_t* ns);

/* test hook, never set by the library itself: the sharded compress of rank
 * `rank` fails right after its pre-flight (-1, the default: no injection) --
 * tests/test_gpu_distributed.py drives the failure paths with it.  Process-wide;
 * returns the previous value. */
int ambc_test_inject_failure(int rank);

#ifdef __cplusplus
}
#endif
#endif
