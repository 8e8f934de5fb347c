// ambc_decode.hip -- per-package decoders for gfx950.
//
// The host walks the 18-byte chunk headers (adaptive_compressor.py:399-445)
// and hands one DecJob per package to k_decode: one 64-lane workgroup per
// package, each decoding straight to the package's byte offset in the output.
// Semantics follow the reference codecs including their lenient paths:
//   255 raw      pad / truncate to orig            (compression_methods.py:691-713)
//   1   RLE      pairs, odd tail ignored, pad/trunc (:116-152); empty -> b''
//   2   Dict     flag/literal/match stream, Python negative indexing (:236-281)
//   3   Huffman  table -> tree (:472-532), bit walk, may stop short (:407-470)
//   4   Delta    byte prefix sum mod 256, truncate (:610-638)
//   9   LZ4      frame (advanced_compression.py:283-296), pad/trunc
//   verbatim     unregistered id: payload copied as is (adaptive_compressor.py:432-435)
// A codec exception becomes orig zero bytes (:440-442).  produced[] reports
// what each job actually wrote so the host can re-walk when a Huffman or
// Dictionary chunk comes out short.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {

constexpr uint32_t STAGE = 8192;   // LDS output staging per package
constexpr uint32_t PIN = 8192;     // LDS copy of the compressed payload
constexpr uint32_t LUT_BITS = 10;

#ifdef AMBC_STAMPS
// diagnostic build only: per-job phase cycles in A.stamps[job*8 + phase]
#define DSTAMP(ph)                                              \
    do {                                                        \
        __builtin_amdgcn_s_waitcnt(0xC07F);                     \
        const uint64_t _t = __builtin_amdgcn_s_memtime();       \
        if (lane == 0 && _stp) _stp[ph] = _t - _st_t;           \
        _st_t = _t;                                             \
    } while (0)
#define DSTAMP_DECL                                             \
    uint64_t _st_t = __builtin_amdgcn_s_memtime();              \
    unsigned long long* _stp = A.stamps ? A.stamps + (uint64_t)blockIdx.x * 8 : nullptr;
#define DSTAMP_PARAMS , unsigned long long* _stp, uint64_t& _st_t
#define DSTAMP_ARGS , _stp, _st_t
// accumulate into register sums (inside loops), flushed with DACC_FLUSH
#define DACC(ph)                                                \
    do {                                                        \
        __builtin_amdgcn_s_waitcnt(0xC07F);                     \
        const uint64_t _t = __builtin_amdgcn_s_memtime();       \
        _acc[ph] += _t - _st_t;                                 \
        _st_t = _t;                                             \
    } while (0)
#define DACC_PARAMS , uint64_t* _acc, uint64_t& _st_t
#define DACC_ARGS , _acc, _st_t
#else
#define DSTAMP(ph) do {} while (0)
#define DSTAMP_DECL
#define DSTAMP_PARAMS
#define DSTAMP_ARGS
#define DACC(ph) do {} while (0)
#define DACC_PARAMS
#define DACC_ARGS
#endif

// LZ4 source map entry flag: payload byte (else an earlier output byte)
template <typename T> struct SrcLit;
template <> struct SrcLit<uint16_t> { static constexpr uint32_t v = 0x8000u; };      // LDS maps
template <> struct SrcLit<uint32_t> { static constexpr uint32_t v = 0x80000000u; };  // global maps

struct DecSmem {
    alignas(16) uint8_t pin[PIN + 64];
    union {
        uint16_t src[STAGE];  // LZ4 block decode: source of every output byte
        struct {
            alignas(16) uint8_t stage[STAGE + 64];
            uint32_t lut[1u << LUT_BITS];  // Huffman: leaf (sym | len<<8 | 1<<31) or node | 10<<16
            uint16_t child[512][2];
            unsigned long long w[256];
            uint8_t syms[256];
            int16_t idx[256];
        };
    };
    uint32_t misc[8];
};

// ---- wave-wide byte movers (dst may be unaligned) ----
__device__ void wave_copy(uint8_t* dst, const uint8_t* src, uint64_t len, uint32_t lane) {
    if (len == 0) return;
    const uint64_t head = min((uint64_t)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3), len);
    if (lane < head) dst[lane] = src[lane];
    const uint64_t nw = (len - head) >> 2;
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + head);
    const uint8_t* s = src + head;
    const uintptr_t sa = reinterpret_cast<uintptr_t>(s);
    const uint32_t sh = (uint32_t)(sa & 3);
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(sa & ~(uintptr_t)3);
    for (uint64_t w = lane; w < nw; w += 64) {
        if (sh == 0) d32[w] = s32[w];
        else d32[w] = __builtin_amdgcn_alignbyte(s32[w + 1], s32[w], sh);
    }
    for (uint64_t i = head + (nw << 2) + lane; i < len; i += 64) dst[i] = src[i];
}

__device__ void wave_zero(uint8_t* dst, uint64_t len, uint32_t lane) {
    if (len == 0) return;
    const uint64_t head = min((uint64_t)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3), len);
    if (lane < head) dst[lane] = 0;
    const uint64_t nw = (len - head) >> 2;
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + head);
    for (uint64_t w = lane; w < nw; w += 64) d32[w] = 0;
    for (uint64_t i = head + (nw << 2) + lane; i < len; i += 64) dst[i] = 0;
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// serial XXH32 (lane-local), for LZ4 frame checksums
__device__ uint32_t xxh32(const uint8_t* p, uint64_t len, uint32_t seed) {
    const uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U,
                   P5 = 374761393U;
    const uint8_t* e = p + len;
    uint32_t h;
    auto rd = [](const uint8_t* q) {
        return (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
    };
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const uint8_t* lim = e - 16;
        do {
            v1 = rotl(v1 + rd(p) * P2, 13) * P1; p += 4;
            v2 = rotl(v2 + rd(p) * P2, 13) * P1; p += 4;
            v3 = rotl(v3 + rd(p) * P2, 13) * P1; p += 4;
            v4 = rotl(v4 + rd(p) * P2, 13) * P1; p += 4;
        } while (p <= lim);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    while (p + 4 <= e) { h = rotl(h + rd(p) * P3, 17) * P4; p += 4; }
    while (p < e) { h = rotl(h + (*p) * P5, 11) * P1; p++; }
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

__device__ __forceinline__ uint64_t le_partial(const uint8_t* p, uint64_t pos, uint64_t plen, int nb) {
    uint64_t v = 0;
    for (int b = 0; b < nb; b++)
        if (pos + b < plen) v |= (uint64_t)p[pos + b] << (8 * b);
    return v;
}

// ---------------------------------------------------------------------------
// RLE: 64 pairs per step, inclusive scan of counts, cooperative fill
// ---------------------------------------------------------------------------
__device__ void dec_rle(const uint8_t* p, uint32_t plen, uint32_t orig, uint8_t* dst, uint32_t lane,
                        uint32_t* scan_lds) {
    const uint32_t np = plen / 2;
    uint32_t o = 0;
    for (uint32_t g = 0; g < np && o < orig; g += 64) {
        const uint32_t j = g + lane;
        const uint32_t c = j < np ? p[2 * j + 1] : 0;
        const uint32_t incl = wave_incl_sum(c);
        scan_lds[lane] = incl;
        const uint32_t tot = __shfl(incl, 63);
        wave_sync();
        const uint32_t lim = min(tot, orig - o);
        for (uint32_t q = lane; q < lim; q += 64) {
            uint32_t lo = 0, hi = 63;  // first lane with incl > q
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (scan_lds[mid] > q) hi = mid; else lo = mid + 1;
            }
            dst[o + q] = p[2 * (g + lo)];
        }
        o += lim;
        wave_sync();
    }
    if (o < orig) wave_zero(dst + o, orig - o, lane);
}

// Delta: prefix sum mod 256 over min(plen, orig) bytes
__device__ void dec_delta(const uint8_t* p, uint32_t m, uint8_t* dst, uint32_t lane) {
    uint32_t carry = 0;
    for (uint32_t g = 0; g < m; g += 64 * 16) {
        const uint32_t b0 = g + lane * 16;
        uint32_t loc[16];
        uint32_t s = 0;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const uint32_t v = b0 + t < m ? p[b0 + t] : 0;
            s += v;
            loc[t] = s;
        }
        const uint32_t incl = wave_incl_sum(s);
        const uint32_t ex = carry + incl - s;
#pragma unroll
        for (int t = 0; t < 16; t++)
            if (b0 + t < m) dst[b0 + t] = (uint8_t)(ex + loc[t]);
        carry += __shfl(incl, 63);
    }
}

// ---------------------------------------------------------------------------
// Huffman (id 3)
// returns produced bytes, or -1 for a Python exception
// ---------------------------------------------------------------------------
__device__ int64_t dec_huffman(const uint8_t* p, uint32_t plen, uint32_t orig, uint8_t* dst,
                               DecSmem& S, uint32_t lane) {
    // table parse (lane 0)
    if (lane == 0) {
        for (int s = 0; s < 256; s++) S.idx[s] = -1;
        const uint32_t k = p[0];
        uint64_t pos = 1;
        int nf = 0, err = 0;
        for (uint32_t e = 0; e < k; e++) {
            if (pos >= plen) { err = 1; break; }
            const uint32_t b = p[pos++];
            const uint64_t c = le_partial(p, pos, plen, 4);
            pos += 4;
            if (S.idx[b] < 0) { S.idx[b] = (int16_t)nf; S.syms[nf] = (uint8_t)b; nf++; }
            S.w[S.idx[b]] = c;
        }
        S.misc[0] = err;
        S.misc[1] = (uint32_t)nf;
        S.misc[2] = (uint32_t)min(pos, (uint64_t)0xFFFFFFFFu);
    }
    wave_sync();
    if (S.misc[0] || S.misc[1] < 2) return -1;   // IndexError paths
    const uint32_t nf = S.misc[1];
    uint64_t pos = S.misc[2];
    // tree by repeated wave-min merges of (weight, first symbol) keys
    unsigned long long key[4];
    uint32_t nid[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t s = lane + 64 * j;
        const int ix = S.idx[s];
        key[j] = ix >= 0 ? ((S.w[ix] << 8) | s) : ~0ull;
        nid[j] = s;
    }
    for (uint32_t m = 0; m + 1 < nf; m++) {
        unsigned long long lm = key[0];
#pragma unroll
        for (int j = 1; j < 4; j++) lm = key[j] < lm ? key[j] : lm;
        const unsigned long long k1 = wave_min_u64(lm);
        unsigned long long lm2 = ~0ull;
#pragma unroll
        for (int j = 0; j < 4; j++) if (key[j] != k1 && key[j] < lm2) lm2 = key[j];
        const unsigned long long k2 = wave_min_u64(lm2);
        const uint32_t s1 = (uint32_t)(k1 & 255), s2 = (uint32_t)(k2 & 255);
        const unsigned long long merged = (((k1 >> 8) + (k2 >> 8)) << 8) | s1;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (lane + 64 * j == s1) {
                S.child[256 + m][0] = (uint16_t)nid[j];
                key[j] = merged; nid[j] = 256 + m;
            } else if (lane + 64 * j == s2) {
                S.child[256 + m][1] = (uint16_t)nid[j];
                key[j] = ~0ull;
            }
        }
    }
    wave_sync();
    const uint32_t root = 256 + nf - 2;
    // LUT over LUT_BITS-bit prefixes
    for (uint32_t v = lane; v < (1u << LUT_BITS); v += 64) {
        uint32_t nd = root, d = 0;
        while (d < LUT_BITS && nd >= 256) {
            nd = S.child[nd][(v >> (LUT_BITS - 1 - d)) & 1];
            d++;
        }
        S.lut[v] = nd < 256 ? (0x80000000u | d << 8 | nd) : (LUT_BITS << 16 | nd);
    }
    wave_sync();
    int64_t produced = 0;
    if (lane == 0) {
        uint64_t nbits = le_partial(p, pos, plen, 4);
        pos += 4;
        const uint64_t avail = pos < plen ? (uint64_t)(plen - pos) * 8 : 0;
        if (nbits > avail) nbits = avail;
        const uint8_t* bitsrc = p + pos;
        uint64_t bp = 0, o = 0;
        uint64_t buf = 0;
        int have = 0;
        uint64_t nextbyte = 0;
        const uint64_t nbytes = (nbits + 7) / 8;
        const uint64_t lim = orig ? orig : 1;   // (the reference tests len(out) >= orig after appending)
        while (bp < nbits && o < lim) {
            while (have <= 56) {
                const uint64_t b = nextbyte < nbytes ? bitsrc[nextbyte] : 0;
                nextbyte++;
                buf |= b << (56 - have);
                have += 8;
            }
            const uint32_t e = S.lut[buf >> (64 - LUT_BITS)];
            uint32_t nd;
            uint32_t used;
            if (e & 0x80000000u) { used = (e >> 8) & 0xFF; nd = e & 0xFF; }
            else { used = LUT_BITS; nd = e & 0xFFFF; }
            if (bp + used > nbits) {
                // not enough bits for the LUT step: walk the remaining bits one by one
                uint32_t cur = root;
                bool leaf = false;
                uint64_t q = bp;
                uint64_t bb = buf;
                while (q < nbits) {
                    cur = S.child[cur][(bb >> 63) & 1];
                    bb <<= 1; q++;
                    if (cur < 256) { leaf = true; break; }
                }
                if (!leaf) break;
                dst[o++] = (uint8_t)cur;
                const uint32_t u = (uint32_t)(q - bp);
                buf <<= u; have -= u; bp = q;
                continue;
            }
            buf <<= used; have -= used; bp += used;
            if (nd >= 256) {
                bool leaf = false;
                while (bp < nbits) {
                    if (have <= 0) {
                        const uint64_t b = nextbyte < nbytes ? bitsrc[nextbyte] : 0;
                        nextbyte++;
                        buf |= b << 56;
                        have += 8;
                    }
                    nd = S.child[nd][(buf >> 63) & 1];
                    buf <<= 1; have--; bp++;
                    if (nd < 256) { leaf = true; break; }
                }
                if (!leaf) break;
            }
            dst[o++] = (uint8_t)nd;
        }
        produced = (int64_t)o;
    }
    return __shfl(produced, 0);
}

// ---------------------------------------------------------------------------
// LZ4 frame (id 9); lane 0 parses, the wave copies.  Output goes to `dst`
// (LDS stage when the content fits, else global memory written by lane 0
// only so that its own back-references stay coherent).
// returns content bytes, or -1 on a frame error
// ---------------------------------------------------------------------------
__device__ int64_t dec_lz4(const uint8_t* p, uint32_t plen, uint8_t* dst, uint64_t cap, bool wave_ok,
                           DecSmem& S, uint32_t lane) {
    // header (every lane reads the same bytes)
    auto rd32 = [&](uint64_t q) {
        return (uint32_t)p[q] | (uint32_t)p[q + 1] << 8 | (uint32_t)p[q + 2] << 16 | (uint32_t)p[q + 3] << 24;
    };
    if (plen < 7 || rd32(0) != 0x184D2204u) return -1;
    const uint32_t flg = p[4], bd = p[5];
    if ((flg >> 6) != 1 || (flg & 0x02) || (bd & 0x8F)) return -1;
    const uint32_t bsid = (bd >> 4) & 7;
    if (bsid < 4) return -1;
    const uint64_t bmax = 1ull << (8 + 2 * bsid);
    uint64_t hp = 6, csize = 0;
    const bool has_cs = (flg >> 3) & 1, has_bck = (flg >> 4) & 1, has_cck = (flg >> 2) & 1,
               has_dict = flg & 1;
    if (has_cs) { if (hp + 8 > plen) return -1; csize = le_partial(p, hp, plen, 8); hp += 8; }
    if (has_dict) { if (hp + 4 > plen) return -1; hp += 4; }
    if (hp >= plen) return -1;
    if (((xxh32(p + 4, hp - 4, 0) >> 8) & 0xFF) != p[hp]) return -1;
    hp++;
    if (has_cs && csize > cap) return -1;  // caller sized cap from the content size when present
    uint64_t op = 0;
    for (;;) {
        if (hp + 4 > plen) return -1;
        const uint32_t bs = rd32(hp);
        hp += 4;
        if (bs == 0) break;
        const uint32_t sz = bs & 0x7FFFFFFFu;
        if (sz > bmax || hp + sz > plen) return -1;
        if (bs & 0x80000000u) {
            if (op + sz > cap) return -1;
            if (wave_ok) { for (uint32_t t = lane; t < sz; t += 64) dst[op + t] = p[hp + t]; }
            else if (lane == 0) { for (uint32_t t = 0; t < sz; t++) dst[op + t] = p[hp + t]; }
            op += sz;
        } else {
            const uint8_t* s = p + hp;
            const uint64_t lim = min(op + bmax, cap);
            uint64_t ip = 0;
            for (;;) {
                if (ip >= sz) return -1;
                const uint32_t tok = s[ip++];
                uint64_t lit = tok >> 4;
                if (lit == 15) {
                    uint32_t b;
                    do { if (ip >= sz) return -1; b = s[ip++]; lit += b; } while (b == 255);
                }
                if (ip + lit > sz || op + lit > lim) return -1;
                if (wave_ok) { for (uint64_t t = lane; t < lit; t += 64) dst[op + t] = s[ip + t]; }
                else if (lane == 0) { for (uint64_t t = 0; t < lit; t++) dst[op + t] = s[ip + t]; }
                ip += lit; op += lit;
                if (ip == sz) break;
                if (ip + 2 > sz) return -1;
                const uint64_t off = s[ip] | (uint64_t)s[ip + 1] << 8;
                ip += 2;
                if (off == 0 || off > op) return -1;
                uint64_t ml = tok & 15;
                if (ml == 15) {
                    uint32_t b;
                    do { if (ip >= sz) return -1; b = s[ip++]; ml += b; } while (b == 255);
                }
                ml += 4;
                if (op + ml > lim) return -1;
                if (wave_ok) {
                    wave_sync();
                    if (off >= ml) {
                        for (uint32_t t = lane; t < (uint32_t)ml; t += 64) dst[op + t] = dst[op - off + t];
                    } else {
                        for (uint32_t t = lane; t < (uint32_t)ml; t += 64)
                            dst[op + t] = dst[op - off + (t % (uint32_t)off)];
                    }
                    wave_sync();
                } else if (lane == 0) {
                    for (uint64_t t = 0; t < ml; t++) dst[op + t] = dst[op - off + t];
                }
                op += ml;
            }
        }
        hp += sz;
        if (has_bck) {
            if (hp + 4 > plen) return -1;
            if (xxh32(p + hp - sz, sz, 0) != rd32(hp)) return -1;
            hp += 4;
        }
        wave_sync();
    }
    if (has_cck) {
        if (hp + 4 > plen) return -1;
        wave_sync();
        uint32_t hsh = 0;
        if (lane == 0) hsh = xxh32(dst, op, 0);
        hsh = __shfl(hsh, 0);
        if (hsh != rd32(hp)) return -1;
    }
    if (has_cs && op != csize) return -1;
    return (int64_t)op;
}

// ---------------------------------------------------------------------------
// LZ4 frame, parallel form (output <= STAGE, payload < 32 KiB, no content
// checksum).  Three phases instead of a byte-serial copy loop:
//   1. the token stream is parsed by the whole wave in lock step from a
//      256-byte register window (4 bytes per lane, bytes fetched with
//      v_readlane, so the parse runs on the scalar unit); each sequence only
//      records, per output byte, where the byte comes from: SRC_LIT|payload
//      index for literals and stored blocks, the earlier output index for
//      match bytes;
//   2. pointer jumping over the source map until every entry names a payload
//      byte (log2 of the longest match chain passes, usually 1-2);
//   3. gather: out[q] = payload[src[q]], dword stores.
// Validity checks are exactly dec_lz4's, in the same order.
// Returns decoded length, -1 for an invalid frame, -2 for "use dec_lz4".
// ---------------------------------------------------------------------------
struct ByteWin {
    uint32_t v;   // 4 payload bytes per lane
    int32_t lo;   // payload index of lane 0's first byte (wave-uniform)
};

// g must point into device global memory with >= 3 readable bytes past g+plen
// (the body buffer has 64 bytes of slack); the window is dword aligned.
__device__ __forceinline__ void win_load(ByteWin& W, const uint8_t* g, uint32_t i, uint32_t plen,
                                         uint32_t lane) {
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(g + i) & 3);
    W.lo = (int32_t)__builtin_amdgcn_readfirstlane(i - mis);
    const uint32_t* a = reinterpret_cast<const uint32_t*>(g + i - mis);
    W.v = (W.lo + 4 * (int32_t)lane < (int32_t)plen) ? a[lane] : 0u;
}

__device__ __forceinline__ uint32_t win_byte(ByteWin& W, const uint8_t* g, uint32_t i, uint32_t plen,
                                             uint32_t lane) {
    uint32_t r = __builtin_amdgcn_readfirstlane((uint32_t)((int32_t)i - W.lo));
    if (r >= 256) {  // uniform branch
        win_load(W, g, i, plen, lane);
        r = __builtin_amdgcn_readfirstlane((uint32_t)((int32_t)i - W.lo));
    }
    return __builtin_amdgcn_readfirstlane((readlane(W.v, r >> 2) >> ((r & 3) * 8)) & 0xFF);
}

// One sequence of an LZ4 block parsed from payload index x (token byte tok),
// with dec_lz4's bounds checks: literal start y, literal length L, offset
// position z, match length ml.  Returns the next token's index, TOK_END (the
// literals reach the block end: last sequence) or TOK_ERR.
constexpr uint32_t TOK_END = 0xFFFFFFFFu, TOK_ERR = 0xFFFFFFFEu, TOK_SLOW = 0xFFFFFFFDu;

__device__ __forceinline__ uint32_t seq_parse(const uint8_t* g, uint32_t x, uint32_t tok, uint32_t end,
                                              uint32_t& y, uint32_t& L, uint32_t& z, uint32_t& ml) {
    y = x + 1;
    L = tok >> 4;
    if (L == 15) {
        uint32_t b;
        do { if (y >= end) return TOK_ERR; b = g[y++]; L += b; } while (b == 255);
    }
    if (y + L > end) return TOK_ERR;
    z = y + L;
    if (z == end) return TOK_END;
    if (z + 2 > end) return TOK_ERR;
    uint32_t w = z + 2;
    ml = tok & 15;
    if (ml == 15) {
        uint32_t b;
        do { if (w >= end) return TOK_ERR; b = g[w++]; ml += b; } while (b == 255);
    }
    ml += 4;
    return w;
}

// the same without length-extension bytes (TOK_SLOW when the token has any)
__device__ __forceinline__ uint32_t seq_next_fast(uint32_t x, uint32_t tok, uint32_t end) {
    const uint32_t L = tok >> 4;
    if (L == 15) return TOK_SLOW;
    const uint32_t z = x + 1 + L;
    if (z > end) return TOK_ERR;
    if (z == end) return TOK_END;
    if (z + 2 > end) return TOK_ERR;
    if ((tok & 15) == 15) return TOK_SLOW;
    return z + 2;
}

// source-map entries of one sequence (o = output index of its first literal).
// Overlapping matches (off < ml) point into the period before the match, so no
// entry's source chain grows with the match length.
template <typename T>
__device__ __forceinline__ void seq_write_lane(T* src, uint32_t o, uint32_t y, uint32_t L,
                                               uint32_t off, uint32_t ml) {
    for (uint32_t t = 0; t < L; t++) src[o + t] = (T)(SrcLit<T>::v | (y + t));
    const uint32_t m0 = o + L - off;
    uint32_t c = 0;
    for (uint32_t t = 0; t < ml; t++) {
        src[o + L + t] = (T)(m0 + c);
        if (++c == off) c = 0;
    }
}

template <typename T>
__device__ __forceinline__ void seq_write_wave(T* src, uint32_t o, uint32_t y, uint32_t L,
                                               uint32_t off, uint32_t ml, uint32_t lane) {
    for (uint32_t b = 0; b < L; b += 64)
        if (b + lane < L) src[o + b + lane] = (T)(SrcLit<T>::v | (y + b + lane));
    if (ml == 0) return;
    const uint32_t m0 = o + L - off;
    if (off >= ml) {  // no overlap: a plain copy
        for (uint32_t b = 0; b < ml; b += 64)
            if (b + lane < ml) src[o + L + b + lane] = (T)(m0 + b + lane);
        return;
    }
    const uint32_t lmod = lane % off;   // (b + lane) % off = (b % off + lane % off) mod off
    uint32_t bmod = 0;
    for (uint32_t b = 0; b < ml; b += 64) {
        uint32_t c = bmod + lmod;
        if (c >= off) c -= off;
        if (b + lane < ml) src[o + L + b + lane] = (T)(m0 + c);
        bmod = (bmod + 64) % off;
    }
}

// One compressed block [hp, end) of a frame, 256 payload positions at a time
// (lane l holds positions wlo + l + 64q, q = 0..3):
//   1. every lane takes each of its positions as a possible token and computes
//      where the next token would start (no extension bytes; TOK_SLOW if any);
//   2. the scalar unit follows the real token chain through the window, one
//      v_readlane per sequence, marking chain positions in four 64-bit masks;
//   3. the marked sequences are decoded in parallel, laid out by wave prefix
//      sums of their output lengths (in position order), validated, and their
//      source-map entries written (long ones by the whole wave).
// Returns the output index after the block or -1.
constexpr uint32_t SEQ_LONG = 32;

template <typename T>
__device__ __forceinline__ int64_t lz4_block_par(const uint8_t* g, uint32_t hp, uint32_t end, uint32_t op,
                                                 uint32_t lim, uint32_t plen, T* src,
                                                 uint32_t lane DACC_PARAMS) {
    uint32_t x0 = hp;
    for (;;) {
        if (x0 >= end) return -1;  // a token must start inside the block
        const uint32_t wlo = x0;
        uint32_t tb[4], nx[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t pos = wlo + lane + 64 * q;
            tb[q] = pos < plen ? g[pos] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t pos = wlo + lane + 64 * q;
            nx[q] = pos < end ? seq_next_fast(pos, tb[q], end) : TOK_ERR;
        }
        DACC(0);
        // the token chain through this window (scalar): the inner loop is one
        // v_readlane and a compare per sequence; tokens with extension bytes,
        // the last sequence and errors leave it (all codes are >= end)
        uint64_t mk[4] = {0, 0, 0, 0};
        uint32_t s = x0, st = 0;  // st: 0 walking, 1 last sequence, 2 invalid
#pragma unroll
        for (int q = 0; q < 4; q++) {
            while (st == 0) {
                const uint32_t lim_r = 64u * (q + 1);
                if (s - wlo >= lim_r) break;  // on to the next 64 positions
                uint64_t m = 0;
                uint32_t cur = s, t;
                const uint32_t climit = min(end, wlo + lim_r);  // codes are all >= end
                do {  // single-exit loop: keeps the scalar code branch-light
                    const uint32_t r = cur - wlo;
                    m |= 1ull << (r & 63);
                    t = readlane(nx[q], r & 63);
                    s = cur;
                    cur = t;
                } while (t < climit);
                mk[q] |= m;
                if (t < end) { s = t; break; }
                if (t == TOK_SLOW) {
                    uint32_t y, L, z, ml;
                    t = __builtin_amdgcn_readfirstlane(
                        seq_parse(g, s, readlane(tb[q], (s - wlo) & 63), end, y, L, z, ml));
                    if (t < end) { s = t; continue; }
                }
                st = t == TOK_END ? 1 : 2;  // TOK_ERR, or a block ending right after a match
                break;
            }
        }
        if (st == 2) return -1;
        DACC(1);
        // the marked sequences, in position order (q major, lane minor)
        uint32_t ky[4], kL[4], koff[4], kml[4], ko[4];
        bool lng = false, bad = false;
        uint32_t base = op;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            ky[q] = kL[q] = koff[q] = kml[q] = 0;
            uint32_t tot = 0;
            if ((mk[q] >> lane) & 1) {
                const uint32_t pos = wlo + lane + 64 * q;
                uint32_t y, L, z, ml = 0;
                const uint32_t nt = seq_parse(g, pos, tb[q], end, y, L, z, ml);
                ky[q] = y;
                kL[q] = L;
                if (nt != TOK_END) { koff[q] = (uint32_t)g[z] | (uint32_t)g[z + 1] << 8; kml[q] = ml; }
                tot = L + kml[q];
                lng |= L > SEQ_LONG || kml[q] > SEQ_LONG;
            }
            const uint32_t incl = wave_incl_sum(tot);
            ko[q] = base + incl - tot;
            base += readlane(incl, 63);
            if ((mk[q] >> lane) & 1) {
                const uint32_t o = ko[q] + kL[q];
                if (o > lim) bad = true;
                if (kml[q] && (koff[q] == 0 || koff[q] > o || o + kml[q] > lim)) bad = true;
            }
        }
        if (__any(bad)) return -1;
        DACC(2);
        if (!lng) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                if ((mk[q] >> lane) & 1) seq_write_lane(src, ko[q], ky[q], kL[q], koff[q], kml[q]);
        }
        // lanes holding a long sequence: written by the whole wave, one lane at a time
        uint64_t lm = __ballot(lng);
        while (lm) {
            const uint32_t l = (uint32_t)__builtin_ctzll(lm);
            lm &= lm - 1;
#pragma unroll
            for (int q = 0; q < 4; q++)
                if ((mk[q] >> l) & 1)
                    seq_write_wave(src, readlane(ko[q], l), readlane(ky[q], l), readlane(kL[q], l),
                                   readlane(koff[q], l), readlane(kml[q], l), lane);
        }
        DACC(3);
        op = base;
        if (st == 1) return (int64_t)op;
        x0 = s;
    }
}

template <typename T>
__device__ __forceinline__ int64_t dec_lz4_par(const uint8_t* p, uint32_t plen, T* src, uint32_t cap,
                               uint32_t lane DSTAMP_PARAMS) {
    constexpr uint32_t SRC_LIT = SrcLit<T>::v;
    if (plen >= SRC_LIT || cap > SRC_LIT || plen < 7) return -2;
#ifdef AMBC_STAMPS
    uint64_t _acc[4] = {0, 0, 0, 0};
#endif
    ByteWin W;
    win_load(W, p, 0, plen, lane);
    auto B = [&](uint32_t i) { return win_byte(W, p, i, plen, lane); };
    auto rd32 = [&](uint32_t q) { return B(q) | B(q + 1) << 8 | B(q + 2) << 16 | B(q + 3) << 24; };
    if (rd32(0) != 0x184D2204u) return -1;
    const uint32_t flg = B(4), bd = B(5);
    if ((flg >> 6) != 1 || (flg & 0x02) || (bd & 0x8F)) return -1;
    const uint32_t bsid = (bd >> 4) & 7;
    if (bsid < 4) return -1;
    if ((flg >> 2) & 1) return -2;  // content checksum: the byte-serial decoder hashes its output
    const uint64_t bmax = 1ull << (8 + 2 * bsid);
    uint32_t hp = 6;
    uint64_t csize = 0;
    const bool has_cs = (flg >> 3) & 1, has_bck = (flg >> 4) & 1, has_dict = flg & 1;
    if (has_cs) {
        if (hp + 8 > plen) return -1;
        for (int b = 0; b < 8; b++) csize |= (uint64_t)B(hp + b) << (8 * b);
        hp += 8;
    }
    if (has_dict) { if (hp + 4 > plen) return -1; hp += 4; }
    if (hp >= plen) return -1;
    if (((xxh32(p + 4, hp - 4, 0) >> 8) & 0xFF) != B(hp)) return -1;
    hp++;
    if (has_cs && csize > cap) return -1;
    uint32_t op = 0;
    for (;;) {
        if (hp + 4 > plen) return -1;
        const uint32_t bs = rd32(hp);
        hp += 4;
        if (bs == 0) break;
        const uint32_t sz = bs & 0x7FFFFFFFu;
        if (sz > bmax || (uint64_t)hp + sz > plen) return -1;
        if (bs & 0x80000000u) {
            if ((uint64_t)op + sz > cap) return -1;
            for (uint32_t t = lane; t < sz; t += 64) src[op + t] = (T)(SRC_LIT | (hp + t));
            op += sz;
        } else {
            const uint64_t lim = min((uint64_t)op + bmax, (uint64_t)cap);
            const int64_t r = lz4_block_par(p, hp, hp + sz, op, (uint32_t)lim, plen, src, lane DACC_ARGS);
            if (r < 0) return -1;
            op = (uint32_t)r;
        }
        hp += sz;
        if (has_bck) {
            if (hp + 4 > plen) return -1;
            if (xxh32(p + hp - sz, sz, 0) != rd32(hp)) return -1;
            hp += 4;
        }
    }
    if (has_cs && op != csize) return -1;
    wave_sync();
    DSTAMP(1);
#ifdef AMBC_STAMPS
    if (lane == 0 && _stp) { _stp[1] = _acc[0]; _stp[2] = _acc[1]; _stp[3] = _acc[2]; _stp[4] = _acc[3]; }
#endif
    uint32_t passes = 0;
    (void)passes;
    // pointer jumping: every pass at least doubles the distance each entry skips
    for (;;) {
        bool more = false;
        for (uint32_t q0 = lane * 4; q0 < op; q0 += 256) {
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = q0 + k < op ? src[q0 + k] : SRC_LIT;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (!(v[k] & SRC_LIT)) {
                    v[k] = src[v[k]];
                    src[q0 + k] = (T)v[k];
                    more |= !(v[k] & SRC_LIT);
                }
        }
        wave_sync();
        passes++;
        if (!__any(more)) break;
    }
    DSTAMP(5);
    return (int64_t)op;
}

// out[0, m) = payload bytes named by the resolved source map
template <typename T>
__device__ void lz4_gather(uint8_t* out, const uint8_t* p, const T* src, uint32_t m, uint32_t lane) {
    constexpr uint32_t MSK = SrcLit<T>::v - 1;
    const uint32_t head = min((uint32_t)((4 - (reinterpret_cast<uintptr_t>(out) & 3)) & 3), m);
    if (lane < head) out[lane] = p[src[lane] & MSK];
    const uint32_t nw = (m - head) >> 2;
    uint32_t* o32 = reinterpret_cast<uint32_t*>(out + head);
    for (uint32_t w = lane; w < nw; w += 64) {
        const uint32_t q = head + 4 * w;
        o32[w] = (uint32_t)p[src[q] & MSK] | (uint32_t)p[src[q + 1] & MSK] << 8 |
                 (uint32_t)p[src[q + 2] & MSK] << 16 | (uint32_t)p[src[q + 3] & MSK] << 24;
    }
    for (uint32_t i = head + (nw << 2) + lane; i < m; i += 64) out[i] = p[src[i] & MSK];
}

// Dictionary (id 2): serial by lane 0 (back-references into its own output)
__device__ int64_t dec_dict(const uint8_t* p, uint32_t plen, uint32_t orig, uint8_t* dst,
                            uint64_t cap, uint32_t lane) {
    int64_t ret = 0;
    if (lane == 0) {
        uint64_t L = 0, pos = 0;
        while (pos < plen && L < orig) {
            const uint32_t flag = p[pos++];
            if (flag == 0) {
                if (pos < plen) dst[L++] = p[pos++];
            } else if (pos + 2 < plen) {
                const uint32_t dist = p[pos] | (uint32_t)p[pos + 1] << 8;
                const uint32_t length = p[pos + 2];
                pos += 3;
                const int64_t start = (int64_t)L - (int64_t)dist;
                for (uint32_t i = 0; i < length; i++) {
                    int64_t ix = start + i;
                    if (L >= cap) { ret = -1; break; }   // host sized cap = orig + 255
                    if (ix < (int64_t)L) {
                        if (ix < 0) ix += (int64_t)L;
                        if (ix < 0) { ret = -1; break; }
                        dst[L] = dst[ix];
                    } else {
                        if (L == 0) { ret = -1; break; }
                        dst[L] = dst[L - 1];
                    }
                    L++;
                }
                if (ret < 0) break;
            }
        }
        if (ret == 0) ret = (int64_t)(L < orig ? L : orig);
    }
    return __shfl(ret, 0);
}

// ---------------------------------------------------------------------------
// Dictionary (id 2), parallel form: the token stream is self-delimiting
// (flag 0: [0, b], else [1, dist_lo, dist_hi, len]; a token cut by the payload
// end is one byte), so the decode runs like lz4_block_par: 256 payload
// positions per step, every lane computes where the token at each of its
// positions would end, the scalar unit follows the real chain (one v_readlane
// per token), the marked tokens are laid out by wave prefix sums of their
// output lengths and write source-map entries, and pointer jumping resolves
// the map.  Semantics of DictionaryCompression.decompress
// (compression_methods.py:236-281): tokens run while the output is shorter
// than orig; a match copies output[len - dist + i] with Python indexing
// (negative indices count from the current end; dist == 0 repeats the last
// byte); an index error is the codec exception (orig zero bytes).
// Returns min(output, orig), -1 for an index error.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t dict_next(uint32_t pos, uint32_t flag, uint32_t plen) {
    return flag == 0 ? (pos + 1 < plen ? pos + 2 : pos + 1) : (pos + 3 < plen ? pos + 4 : pos + 1);
}

// source of output byte O + i of a match (O: output length before it); false: index error
__device__ __forceinline__ bool dict_src(uint32_t O, uint32_t dist, uint32_t i, uint32_t& s) {
    if (dist == 0) { s = O - 1; return O > 0; }              // decompressed[-1]
    if (O >= dist) { s = O - dist + i % dist; return true; }  // the period before the match
    const int32_t ix = (int32_t)O - (int32_t)dist + (int32_t)i;
    if (ix >= 0) { s = (uint32_t)ix; return true; }
    const int32_t py = (int32_t)(O + i) + ix;               // Python negative index
    s = (uint32_t)py;
    return py >= 0;
}

template <typename T>
__device__ int64_t dec_dict_par(const uint8_t* g, uint32_t plen, uint32_t orig, T* src, uint32_t cap,
                                uint32_t lane) {
    constexpr uint32_t SRC_LIT = SrcLit<T>::v;
    uint32_t op = 0, x0 = 0;
    bool bad = false;
    while (x0 < plen && op < orig) {
        const uint32_t wlo = x0;
        uint32_t fb[4], nx[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t pos = wlo + lane + 64 * q;
            fb[q] = pos < plen ? g[pos] : 0u;
            nx[q] = pos < plen ? dict_next(pos, fb[q], plen) : TOK_END;
        }
        // the token chain through this window (scalar)
        uint64_t mk[4] = {0, 0, 0, 0};
        uint32_t s = x0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t hi = wlo + 64u * (q + 1);
            uint64_t m = 0;
            while (s < hi && s < plen) {
                const uint32_t r = s - wlo - 64u * q;
                m |= 1ull << r;
                s = readlane(nx[q], r);
            }
            mk[q] = m;
        }
        // output length of every marked token, laid out in position order; a
        // token starting at or after orig is not run (the loop test), nor any after it
        uint32_t kO[4], kol[4], kd[4], ky[4];
        uint32_t base = op;
        bool lng = false;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t pos = wlo + lane + 64 * q;
            kol[q] = kd[q] = 0;
            ky[q] = pos + 1;
            if ((mk[q] >> lane) & 1) {
                if (fb[q] == 0) {
                    kol[q] = pos + 1 < plen ? 1u : 0u;
                } else if (pos + 3 < plen) {
                    kd[q] = (uint32_t)g[pos + 1] | (uint32_t)g[pos + 2] << 8;
                    kol[q] = g[pos + 3];
                }
            }
            const uint32_t incl = wave_incl_sum(kol[q]);
            kO[q] = base + incl - kol[q];
            base += readlane(incl, 63);
        }
        uint32_t run_end = base;            // output length after the last token run
        bool stop = false;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bool run = ((mk[q] >> lane) & 1) && kO[q] < orig;
            const uint64_t cut = __ballot(((mk[q] >> lane) & 1) && kO[q] >= orig);
            if (cut && !stop) {             // the first token not run: its start ends the output
                run_end = readlane(kO[q], (uint32_t)__builtin_ctzll(cut));
                stop = true;
            }
            if (!run) kol[q] = 0;
            else lng |= kol[q] > 32;
        }
        if (run_end > cap) return -1;       // (cap >= orig + 255 by the host: never)
        // source-map entries: literals and short matches per lane, long matches by the wave
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (kol[q] == 0 || kol[q] > 32) continue;
            if (fb[q] == 0) {
                src[kO[q]] = (T)(SRC_LIT | ky[q]);
            } else if (kd[q] && kO[q] >= kd[q]) {   // the common case: the period before the match
                const uint32_t m0 = kO[q] - kd[q];
                uint32_t c = 0;
                for (uint32_t i = 0; i < kol[q]; i++) {
                    src[kO[q] + i] = (T)(m0 + c);
                    if (++c == kd[q]) c = 0;
                }
            } else {
                for (uint32_t i = 0; i < kol[q]; i++) {
                    uint32_t sidx;
                    bad |= !dict_src(kO[q], kd[q], i, sidx);
                    src[kO[q] + i] = (T)sidx;
                }
            }
        }
        uint64_t lm = __ballot(lng);
        while (lm) {
            const uint32_t l = (uint32_t)__builtin_ctzll(lm);
            lm &= lm - 1;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t ol = readlane(kol[q], l);
                if (ol <= 32) continue;
                const uint32_t O = readlane(kO[q], l), dd = readlane(kd[q], l);
                if (dd && O >= dd) {
                    const uint32_t lmod = lane % dd;
                    uint32_t bmod = 0;
                    for (uint32_t b = 0; b < ol; b += 64) {
                        uint32_t c = bmod + lmod;
                        if (c >= dd) c -= dd;
                        if (b + lane < ol) src[O + b + lane] = (T)(O - dd + c);
                        bmod = (bmod + 64) % dd;
                    }
                } else {
                    for (uint32_t b = 0; b < ol; b += 64)
                        if (b + lane < ol) {
                            uint32_t sidx;
                            bad |= !dict_src(O, dd, b + lane, sidx);
                            src[O + b + lane] = (T)sidx;
                        }
                }
            }
        }
        op = run_end;
        if (stop) break;
        x0 = s;
    }
    if (__any(bad)) return -1;
    wave_sync();
    // pointer jumping: every entry names an earlier output byte or a payload byte
    for (;;) {
        bool more = false;
        for (uint32_t q0 = lane * 4; q0 < op; q0 += 256) {
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = q0 + k < op ? src[q0 + k] : SRC_LIT;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (!(v[k] & SRC_LIT)) {
                    v[k] = src[v[k]];
                    src[q0 + k] = (T)v[k];
                    more |= !(v[k] & SRC_LIT);
                }
        }
        wave_sync();
        if (!__any(more)) break;
    }
    return (int64_t)min(op, orig);
}

// raw / verbatim / skip / RLE / Delta: no LDS beyond a 64-entry scan
__device__ __forceinline__ bool decode_light(const DecJob& J, const uint8_t* p, uint8_t* out,
                                             uint32_t lane, uint32_t* scan, int64_t& produced) {
    const uint32_t orig = J.orig, clen = J.clen;
    switch (J.type) {
    case DEC_SKIP:
        produced = J.expect;
        return true;
    case DEC_VERBATIM:
        wave_copy(out, p, clen, lane);
        produced = clen;
        return true;
    case 255: {
        const uint32_t m = min(clen, orig);
        wave_copy(out, p, m, lane);
        wave_zero(out + m, orig - m, lane);
        produced = orig;
        return true;
    }
    case 1:
        if (clen) { dec_rle(p, clen, orig, out, lane, scan); produced = orig; }
        return true;
    case 4:
        if (clen) { produced = min(clen, orig); dec_delta(p, (uint32_t)produced, out, lane); }
        return true;
    default:
        return false;
    }
}

__device__ __forceinline__ uint32_t job_index(const DecArgs& A) {
    return uniform_u32(A.list ? A.list[blockIdx.x] : blockIdx.x);
}

__device__ __forceinline__ void put_produced(const DecArgs& A, uint32_t j, int64_t produced,
                                             uint32_t lane) {
    if (lane == 0) A.produced[j] = (uint32_t)(produced < 0 ? 0xFFFFFFFFu : (uint32_t)produced);
}

__global__ __launch_bounds__(64) void k_decode_light(DecArgs A) {
    __shared__ uint32_t scan[64];
    const uint32_t lane = threadIdx.x;
    const uint32_t j = job_index(A);
    const DecJob J = A.jobs[j];
    int64_t produced = 0;
    if (!decode_light(J, A.body + J.body_off, A.out + J.out_off, lane, scan, produced)) produced = -1;
    put_produced(A, j, produced, lane);
}

// LZ4 frames the host routed here: no content checksum, content bound <=
// OUTMAX and payload < 32 KiB (LDS source map of u16), or any size with the
// map in the job's device scratch window (u32 entries, k_decode_lz4_g) -- so
// dec_lz4_par never asks for the serial decoder
template <typename T>
__device__ __forceinline__ void lz4_job(const DecArgs& A, uint32_t j, const DecJob& J, T* src, uint32_t cap,
                                        uint32_t lane) {
    DSTAMP_DECL
    const uint8_t* g = uniform_ptr(A.body + J.body_off);
    uint8_t* out = uniform_ptr(A.out + J.out_off);
    const uint32_t orig = uniform_u32(J.orig);
    DSTAMP(0);
    const int64_t r = dec_lz4_par(g, uniform_u32(J.clen), src, uniform_u32(cap), lane DSTAMP_ARGS);
    wave_sync();
    if (r < 0) {
        wave_zero(out, orig, lane);
    } else {
        const uint32_t m = min((uint32_t)r, orig);
        lz4_gather(out, g, src, m, lane);
        wave_zero(out + m, orig - m, lane);
    }
    DSTAMP(6);
#ifdef AMBC_STAMPS
    if (lane == 0 && _stp) _stp[7] = 9;
#endif
    put_produced(A, j, r == -2 ? -1 : (int64_t)orig, lane);
}

template <uint32_t OUTMAX>
__global__ __launch_bounds__(64) void k_decode_lz4(DecArgs A) {
    __shared__ uint16_t src[OUTMAX];
    const uint32_t j = job_index(A);
    const DecJob J = A.jobs[j];
    lz4_job(A, j, J, src, OUTMAX, threadIdx.x);
}

__global__ __launch_bounds__(64) void k_decode_lz4_g(DecArgs A) {
    const uint32_t j = job_index(A);
    const DecJob J = A.jobs[j];
    lz4_job(A, j, J, reinterpret_cast<uint32_t*>(A.scratch + J.scratch_off), (uint32_t)J.scratch_cap,
            threadIdx.x);
}

// Dictionary packages whose output (+ one match of overshoot) fits the LDS map
template <uint32_t OUTMAX>
__global__ __launch_bounds__(64) void k_decode_dict(DecArgs A) {
    __shared__ uint16_t src[OUTMAX];
    const uint32_t lane = threadIdx.x;
    const uint32_t j = job_index(A);
    const DecJob J = A.jobs[j];
    const uint8_t* g = uniform_ptr(A.body + J.body_off);
    uint8_t* out = uniform_ptr(A.out + J.out_off);
    const uint32_t orig = uniform_u32(J.orig);
    const int64_t r = dec_dict_par(g, uniform_u32(J.clen), orig, src, OUTMAX, lane);
    wave_sync();
    int64_t produced;
    if (r < 0) {
        wave_zero(out, orig, lane);
        produced = orig;
    } else {
        lz4_gather(out, g, src, (uint32_t)r, lane);
        produced = r;
    }
    put_produced(A, j, produced, lane);
}

// everything else: Huffman, Dictionary, LZ4 frames that need the serial decoder
__global__ __launch_bounds__(64) void k_decode(DecArgs A) {
    __shared__ DecSmem S;
    const uint32_t lane = threadIdx.x;
    const uint32_t j = job_index(A);
    const DecJob J = A.jobs[j];
    const uint8_t* p = A.body + J.body_off;
    const uint8_t* g = p;  // the payload in global memory
    uint8_t* out = A.out + J.out_off;
    const uint32_t orig = J.orig, clen = J.clen;
    int64_t produced = 0;
    if (decode_light(J, p, out, lane, reinterpret_cast<uint32_t*>(S.stage), produced)) {
        put_produced(A, j, produced, lane);
        return;
    }
    if ((J.type == 2 || J.type == 3 || J.type == 9) && clen && clen <= PIN) {
        // serial parsers read the payload byte by byte: keep it in LDS
        wave_copy(S.pin, p, clen, lane);
        if (lane < 8) S.pin[clen + lane] = 0;
        wave_sync();
        p = S.pin;
    }
    switch (J.type) {
    case 3: {
        if (clen == 0) break;
        const bool staged = orig <= STAGE;
        int64_t r = dec_huffman(p, clen, orig, staged ? S.stage : out, S, lane);
        wave_sync();
        if (r < 0) { wave_zero(out, orig, lane); produced = orig; }
        else {
            if (staged) wave_copy(out, S.stage, (uint64_t)r, lane);
            produced = r;
        }
        break;
    }
    case 9: {
        if (clen == 0) break;
        // decoded content may exceed orig (then truncated): LDS when it fits, else
        // the job's device scratch window sized by the host walk
        const bool staged = J.scratch_off == ~0ull;
        uint8_t* dst = staged ? S.stage : A.scratch + J.scratch_off;
        (void)g;
        const int64_t r = dec_lz4(p, clen, dst, staged ? STAGE : J.scratch_cap, staged, S, lane);
        wave_sync();
        if (r < 0) { wave_zero(out, orig, lane); }
        else {
            const uint64_t m = min((uint64_t)r, (uint64_t)orig);
            if (staged) wave_copy(out, dst, m, lane);
            else if (lane == 0) for (uint64_t i = 0; i < m; i++) out[i] = dst[i];  // lane 0 wrote it
            wave_zero(out + m, orig - m, lane);
        }
        produced = orig;
        break;
    }
    case 2: {
        if (clen == 0) break;
        const bool staged = J.scratch_off == ~0ull;
        uint8_t* dst = staged ? S.stage : A.scratch + J.scratch_off;
        const int64_t r = dec_dict(p, clen, orig, dst, staged ? STAGE : J.scratch_cap, lane);
        wave_sync();
        if (r < 0) { wave_zero(out, orig, lane); produced = orig; }
        else {
            if (staged) wave_copy(out, dst, (uint64_t)r, lane);
            else if (lane == 0) for (int64_t i = 0; i < r; i++) out[i] = dst[i];
            produced = r;
        }
        break;
    }
    default:  // registered id with no device codec (should have been DEC_SKIP)
        produced = -1;
        break;
    }
    put_produced(A, j, produced, lane);
}

hipError_t launch_decode(int kind, const DecArgs& a, hipStream_t s) {
    if (a.n_list == 0) return hipSuccess;
    switch (kind) {
    case DEC_KIND_LIGHT: hipLaunchKernelGGL(k_decode_light, dim3(a.n_list), dim3(64), 0, s, a); break;
    case DEC_KIND_LZ4_4K: hipLaunchKernelGGL(k_decode_lz4<4096>, dim3(a.n_list), dim3(64), 0, s, a); break;
    case DEC_KIND_LZ4_8K: hipLaunchKernelGGL(k_decode_lz4<8192>, dim3(a.n_list), dim3(64), 0, s, a); break;
    case DEC_KIND_LZ4_16K: hipLaunchKernelGGL(k_decode_lz4<16384>, dim3(a.n_list), dim3(64), 0, s, a); break;
    case DEC_KIND_LZ4_G: hipLaunchKernelGGL(k_decode_lz4_g, dim3(a.n_list), dim3(64), 0, s, a); break;
    case DEC_KIND_DICT_4K: hipLaunchKernelGGL(k_decode_dict<4352>, dim3(a.n_list), dim3(64), 0, s, a); break;
    case DEC_KIND_DICT_8K: hipLaunchKernelGGL(k_decode_dict<8448>, dim3(a.n_list), dim3(64), 0, s, a); break;
    case DEC_KIND_DICT_16K: hipLaunchKernelGGL(k_decode_dict<16640>, dim3(a.n_list), dim3(64), 0, s, a); break;
    case DEC_KIND_INFLATE_4K:
    case DEC_KIND_INFLATE_8K:
    case DEC_KIND_INFLATE_16K:
    case DEC_KIND_INFLATE_32K:
    case DEC_KIND_INFLATE_G: return launch_inflate(kind, a, s);
    case DEC_KIND_HUFF_4K:
    case DEC_KIND_HUFF_8K: return launch_huff(kind, a, s);
    default: hipLaunchKernelGGL(k_decode, dim3(a.n_list), dim3(64), 0, s, a); break;
    }
    return hipGetLastError();
}

}  // namespace ambc
