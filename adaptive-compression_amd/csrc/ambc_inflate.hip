// ambc_inflate.hip -- zlib inflate (id 5 payloads) on gfx950, one wavefront per
// package.  Semantics are DeflateCompression.decompress's
// (advanced_compression.py:83-96): zlib.decompress(payload) with the default
// window, i.e. zlib's inflate() checks -- header (CM 8, window <= 32 KiB, FCHECK,
// no preset dictionary), block types, code-length sets (over-subscribed or
// incomplete sets are errors except a single 1-bit literal/distance code),
// "invalid bit length repeat", missing end-of-block code, invalid codes,
// distances too far back, an unfinished stream and the Adler-32 check -- then
// pad / truncate to orig; any error decodes the package to orig zero bytes.
// Bytes after the stream's end are ignored.
//
// Layout: the payload is read through a 256-byte register window (4 bytes per
// lane, fetched with v_readlane) into a 64-bit bit buffer on the scalar unit;
// Huffman codes resolve through 10-bit LDS lookup tables (longer codes by the
// canonical first-code search).  Output bytes are produced as a source map in
// LDS (u16 per byte: 0x8000 | value for a literal, else the earlier output
// index it copies), match copies written by the whole wave; pointer jumping
// resolves the map, which then yields the Adler-32 and the output.  Output
// larger than the map (OUTMAX) is handed back to the host zlib path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {
namespace {

#ifdef AMBC_STAMPS
#define ISTAMP(ph)                                              \
    do {                                                        \
        __builtin_amdgcn_s_waitcnt(0xC07F);                     \
        const uint64_t _t = __builtin_amdgcn_s_memtime();       \
        _acc[ph] += _t - _st_t;                                 \
        _st_t = _t;                                             \
    } while (0)
#else
#define ISTAMP(ph) do {} while (0)
#endif

constexpr uint32_t IN_LIT = 0x8000u;
constexpr int LUTB = INF_LUTB;       // primary lookup bits (9: 2 KB of tables, 13 workgroups/CU at 4 KiB)
// lookup entries: symbol << 5 | length << 1 | 1; 0 = no code, 2 = a code
// longer than LUTB bits (canonical search)
constexpr uint16_t LUT_BAD = 0;
constexpr uint16_t LUT_LONG = 2;

__constant__ uint8_t c_clord2[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// packages above 32 KiB (OUTMAX 65536): the map lives in the job's device
// scratch window with u32 entries (bit 31 = literal), its capacity the job's orig
template <uint32_t OUTMAX> using inf_map_t = typename std::conditional<(OUTMAX > 32768), uint32_t, uint16_t>::type;
template <uint32_t OUTMAX> constexpr uint32_t inf_lit = OUTMAX > 32768 ? 0x80000000u : IN_LIT;

template <uint32_t OUTMAX>
struct InfSmem {
    static constexpr bool G = OUTMAX > 32768;
    inf_map_t<OUTMAX> srcl[G ? 1 : OUTMAX];   // output source map (LDS)
    inf_map_t<OUTMAX>* srcg;                  // G: the map in device scratch
    uint32_t capg;                            // G: its entries
    __device__ __forceinline__ inf_map_t<OUTMAX>* src() {
        if constexpr (G) return srcg; else return srcl;
    }
    __device__ __forceinline__ uint32_t cap() const {
        if constexpr (G) return capg; else return OUTMAX;
    }
    uint16_t lut[2][1 << LUTB];       // [0] literal/length (or code lengths), [1] distance
    uint16_t sorted[2][288];          // symbols in canonical (length, symbol) order
    uint16_t first[2][16], cnt[2][16], offs[2][16];
    uint8_t lens[320];                // code lengths of the current dynamic block
};

// payload byte stream through a 256-byte register window
struct InBits {
    const uint8_t* g;
    uint32_t plen;
    uint32_t win;      // 4 payload bytes per lane
    uint32_t wlo;      // payload index of the window's first byte (multiple of 4 from g)
    uint64_t buf;      // bit buffer (LSB = next bit)
    uint32_t cnt;      // bits in buf
    uint32_t pos;      // next payload byte to load into buf
    uint32_t lane;
};

// 4 payload bytes per lane starting at the 4-aligned index wlo; zeros past plen
__device__ __noinline__ uint32_t in_load(const uint8_t* g, uint32_t plen, uint32_t wlo, uint32_t lane) {
    const uint32_t q = wlo + 4 * lane;
    uint32_t x = 0;
    if (q + 4 <= plen) {
        x = (uint32_t)g[q] | (uint32_t)g[q + 1] << 8 | (uint32_t)g[q + 2] << 16 | (uint32_t)g[q + 3] << 24;
    } else {
#pragma unroll
        for (int b = 0; b < 4; b++)
            if (q + b < plen) x |= (uint32_t)g[q + b] << (8 * b);
    }
    return x;
}

__device__ __forceinline__ void in_window(InBits& I, uint32_t at) {
    I.wlo = __builtin_amdgcn_readfirstlane(at & ~3u);
    I.win = in_load(I.g, I.plen, I.wlo, I.lane);
}

// 4 payload bytes from the window (little-endian; zeros past the payload)
__device__ __forceinline__ uint32_t in_word(InBits& I, uint32_t at) {
    uint32_t r = __builtin_amdgcn_readfirstlane(at - I.wlo);
    if (r > 248) {  // uniform: keep lane (r >> 2) + 1 inside the window
        in_window(I, at);
        r = __builtin_amdgcn_readfirstlane(at - I.wlo);
    }
    const uint32_t lo = readlane(I.win, r >> 2), hi = readlane(I.win, (r >> 2) + 1);
    return __builtin_amdgcn_readfirstlane(__builtin_amdgcn_alignbyte(hi, lo, r & 3));
}

// top the bit buffer up with the next (at most 4) payload bytes when it holds
// 32 bits or fewer; the caller checks I.cnt against what it consumes
__device__ __forceinline__ void in_fill(InBits& I) {
    if (I.cnt > 32 || I.pos >= I.plen) return;
    const uint32_t avail = min(4u, I.plen - I.pos);
    I.buf |= (uint64_t)in_word(I, I.pos) << I.cnt;
    I.cnt += 8 * avail;
    I.pos += avail;
}

// take n bits (n <= 32); false when the payload is exhausted
__device__ __forceinline__ bool in_take(InBits& I, uint32_t n, uint32_t& v) {
    if (I.cnt < n) {
        in_fill(I);
        if (I.cnt < n) return false;
    }
    v = (uint32_t)(I.buf & ((n >= 32) ? 0xFFFFFFFFull : ((1ull << n) - 1)));
    I.buf >>= n;
    I.cnt -= n;
    return true;
}

// Build the decode tables of code lengths len[0..nsym) into table t.
// kind: 0 = code-length code (incomplete sets are errors), 1 = literal/length
// or distance (a single 1-bit code may be incomplete).  Returns false on an
// over-subscribed or invalid incomplete set (zlib inflate_table's -1).
template <int J, uint32_t OUTMAX>
__device__ bool inf_build(InfSmem<OUTMAX>& S, int t, const uint8_t* len, int nsym, int kind, uint32_t lane) {
    // J: symbol blocks of 64 (nsym <= 64 J)
    uint32_t l[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int s = lane + 64 * j;
        l[j] = s < nsym ? len[s] : 0u;
    }
    uint32_t count[16];
    uint32_t maxl = 0;
#pragma unroll
    for (int b = 1; b < 16; b++) {
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < J; j++) c += (uint32_t)__popcll(__ballot(l[j] == (uint32_t)b));
        count[b] = c;
        if (c) maxl = b;
    }
    if (maxl == 0) {  // no symbols: decoding any code is an error (zlib: valid table)
        for (uint32_t i = lane; i < (1u << LUTB); i += 64) S.lut[t][i] = LUT_BAD;
        if (lane < 16) { S.cnt[t][lane] = 0; S.first[t][lane] = 0; S.offs[t][lane] = 0; }
        wave_sync();
        return true;
    }
    int left = 1;
#pragma unroll
    for (int b = 1; b < 16; b++) {
        left <<= 1;
        left -= (int)count[b];
        if (left < 0) return false;  // over-subscribed
    }
    if (left > 0 && (kind == 0 || maxl != 1)) return false;  // incomplete
    // canonical codes; sorted order (length, symbol)
    uint32_t first = 0, prev = 0, off = 0;
    uint32_t code[J];
    uint32_t fL[LUTB + 1], oL[LUTB + 1], lim[LUTB + 1];   // per length <= LUTB (wave-uniform)
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (int b = 1; b < 16; b++) {
        first = (first + prev) << 1;
        if (b <= LUTB) {
            fL[b] = first;
            oL[b] = off;
            lim[b] = (first + count[b]) << (LUTB - b);
        }
        if (lane == (uint32_t)b) {
            S.first[t][b] = (uint16_t)first;
            S.cnt[t][b] = (uint16_t)count[b];
            S.offs[t][b] = (uint16_t)off;
        }
        uint32_t seen = 0;
#pragma unroll
        for (int j = 0; j < J; j++) {
            const uint64_t m = __ballot(l[j] == (uint32_t)b);
            if (l[j] == (uint32_t)b) {
                const uint32_t r = seen + (uint32_t)__popcll(m & lt);
                code[j] = first + r;
                S.sorted[t][off + r] = (uint16_t)(lane + 64 * j);
            }
            seen += (uint32_t)__popcll(m);
        }
        prev = count[b];
        off += count[b];
    }
    wave_sync();
    // lookup entries: entry x holds the code whose bits (read LSB first) prefix
    // x.  Left-justified, a canonical code's codes of length L fill the 10-bit
    // MSB-first range [fL[L] << (10 - L), lim[L]) and the ranges follow each
    // other by length: the first L with v < lim[L] is the code's length
    for (uint32_t x = lane; x < (1u << LUTB); x += 64) {
        const uint32_t v = __builtin_bitreverse32(x) >> (32 - LUTB);  // MSB-first LUTB-bit window
        uint32_t L = 0, f = 0, o = 0;
#pragma unroll
        for (int b = LUTB; b >= 1; b--) {
            const bool in = v < lim[b];
            L = in ? (uint32_t)b : L;
            f = in ? fL[b] : f;
            o = in ? oL[b] : o;
        }
        uint32_t e;
        if (L) e = (uint32_t)S.sorted[t][o + (v >> (LUTB - L)) - f] << 5 | L << 1 | 1;
        else e = maxl > (uint32_t)LUTB ? LUT_LONG : LUT_BAD;   // a longer code, or none (incomplete set)
        S.lut[t][x] = (uint16_t)e;
    }
    (void)code;
    wave_sync();
    return true;
}

// decode one symbol of table t; -1 = invalid / truncated
template <uint32_t OUTMAX>
__device__ __forceinline__ int inf_sym(InfSmem<OUTMAX>& S, int t, InBits& I) {
    if (I.cnt < 15) in_fill(I);
    // (LDS values are not known to be wave-uniform: readfirstlane keeps the
    // decode loop on the scalar unit)
    const uint32_t e = __builtin_amdgcn_readfirstlane(S.lut[t][I.buf & ((1u << LUTB) - 1)]);
    if (e & 1) {
        const uint32_t L = (e >> 1) & 15;
        if (L > I.cnt) return -1;
        I.buf >>= L;
        I.cnt -= L;
        return e >> 5;
    }
    if (e == LUT_BAD) return -1;
    // canonical search for a code of 11..15 bits
    uint32_t c = 0;
    for (uint32_t L = 1; L <= 15; L++) {
        if (L > I.cnt) return -1;
        c = c << 1 | (uint32_t)((I.buf >> (L - 1)) & 1);
        if (L <= (uint32_t)LUTB) continue;
        const uint32_t cnt = __builtin_amdgcn_readfirstlane(S.cnt[t][L]);
        const uint32_t f = __builtin_amdgcn_readfirstlane(S.first[t][L]);
        if (c - f < cnt && c >= f) {
            I.buf >>= L;
            I.cnt -= L;
            return (int)__builtin_amdgcn_readfirstlane(S.sorted[t][__builtin_amdgcn_readfirstlane(S.offs[t][L]) + (c - f)]);
        }
    }
    return -1;
}

// the fixed-Huffman block's tables (RFC 1951 3.2.6): literal/length 0..287,
// distance 0..29 (+30, 31: codes that decode as invalid)
template <uint32_t OUTMAX>
__device__ void fixed_tables_build(InfSmem<OUTMAX>& S, uint32_t lane) {
    for (uint32_t s = lane; s < 320; s += 64)
        S.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
    wave_sync();
    (void)inf_build<5>(S, 0, S.lens, 288, 1, lane);
    (void)inf_build<1>(S, 1, S.lens + 288, 32, 1, lane);
}

// table parts of InfSmem in the global layout of launch_inflate_fixed_tables:
// lut[2][1 << LUTB] | sorted[2][288] | first[2][16] | cnt[2][16] | offs[2][16]
template <uint32_t OUTMAX>
__device__ __forceinline__ uint16_t* fixed_part(InfSmem<OUTMAX>& S, uint32_t i) {
    if (i < (2u << LUTB)) return &S.lut[0][0] + i;
    i -= 2u << LUTB;
    if (i < 576) return &S.sorted[0][0] + i;
    i -= 576;
    if (i < 32) return &S.first[0][0] + i;
    i -= 32;
    if (i < 32) return &S.cnt[0][0] + i;
    return &S.offs[0][0] + (i - 32);
}

template <uint32_t OUTMAX>
__device__ __forceinline__ void fixed_tables_in(InfSmem<OUTMAX>& S, const uint16_t* fixed, uint32_t lane) {
    for (uint32_t i = lane; i < INF_FIXED_U16; i += 64) *fixed_part(S, i) = fixed[i];
    wave_sync();
}

__global__ __launch_bounds__(64) void k_inflate_fixed(uint16_t* out) {
    __shared__ InfSmem<64> S;
    fixed_tables_build(S, threadIdx.x);
    for (uint32_t i = threadIdx.x; i < INF_FIXED_U16; i += 64) out[i] = *fixed_part(S, i);
}

// reposition the reader at absolute payload bit `bit`
__device__ __forceinline__ void in_seek(InBits& I, uint32_t bit) {
    I.pos = bit >> 3;
    I.buf = 0;
    I.cnt = 0;
    in_window(I, I.pos & ~3u);
    uint32_t v;
    if (bit & 7) (void)in_take(I, bit & 7, v);
}

// one item (literal, length/distance pair or end of block) decoded serially
// through the reader: 1 = end of block, 0 = item done, -1 invalid, -2 too large
template <uint32_t OUTMAX>
__device__ int inf_item_serial(InfSmem<OUTMAX>& S, InBits& I, uint32_t& op, uint32_t lane) {
    const int sy = inf_sym(S, 0, I);
    if (sy < 0) return -1;
    if (sy < 256) {
        if (op >= S.cap()) return -2;
        if (lane == 0) S.src()[op] = (inf_map_t<OUTMAX>)(inf_lit<OUTMAX> | (uint32_t)sy);
        op++;
        return 0;
    }
    if (sy == 256) return 1;
    const uint32_t k = (uint32_t)sy - 257;
    if (k >= 29) return -1;  // 286, 287
    uint32_t L;
    if (k < 8) {
        L = 3 + k;
    } else if (k == 28) {
        L = 258;
    } else {
        const uint32_t eb = (k >> 2) - 1, base = ((4u | (k & 3)) << eb) + 3;
        uint32_t x;
        if (!in_take(I, eb, x)) return -1;
        L = base + x;
    }
    const int ds = inf_sym(S, 1, I);
    if (ds < 0 || ds >= 30) return -1;
    uint32_t D;
    if (ds < 4) {
        D = (uint32_t)ds + 1;
    } else {
        const uint32_t eb = ((uint32_t)ds >> 1) - 1, base = ((2u | ((uint32_t)ds & 1)) << eb) + 1;
        uint32_t x;
        if (!in_take(I, eb, x)) return -1;
        D = base + x;
    }
    if (D > op) return -1;  // invalid distance too far back
    if (op + L > S.cap()) return -2;
    // entries point into the period before the match (chains stay short)
    const uint32_t m0 = op - D;
    if (D >= L) {
        for (uint32_t b = 0; b < L; b += 64)
            if (b + lane < L) S.src()[op + b + lane] = (inf_map_t<OUTMAX>)(m0 + b + lane);
    } else {
        const uint32_t lmod = lane % D;
        uint32_t bmod = 0;
        for (uint32_t b = 0; b < L; b += 64) {
            uint32_t c = bmod + lmod;
            if (c >= D) c -= D;
            if (b + lane < L) S.src()[op + b + lane] = (inf_map_t<OUTMAX>)(m0 + c);
            bmod = (bmod + 64) % D;
        }
    }
    op += L;
    return 0;
}

#ifdef AMBC_STAMPS
#define ISTAMP_PARAMS , uint64_t* _acc, uint64_t& _st_t
#define ISTAMP_ARGS , _acc, _st_t
#else
#define ISTAMP_PARAMS
#define ISTAMP_ARGS
#endif

// ---- speculative parallel symbol decode of one Huffman-coded block ----
// Every lane decodes a whole item (literal, length + distance with their extra
// bits, or end of block) at each of 4 bit positions of a 256-bit window
// (lane l: window start + l + 64q) through the LDS tables; the scalar unit
// then follows the real item chain with one v_readlane per item; the chain's
// items are laid out by wave prefix sums of their output lengths, validated
// (distance too far back, map overflow) and their source-map entries written
// in parallel.  Codes longer than the table (canonical search) are decoded by
// inf_item_serial in order.  Same results as the serial loop: any error in a
// window is reported (an error and an overflow both end in orig zero bytes,
// the overflow through the host zlib path).
#ifndef INF_SHORT
#define INF_SHORT 32u   // matches up to this length: one lane each; longer: the whole wave
#endif
constexpr uint32_t IT_EOB = 0xFFFFFFF0u, IT_SLOW = 0xFFFFFFF1u, IT_ERR = 0xFFFFFFF2u;
enum : uint32_t { IK_LIT = 0, IK_MATCH = 1, IK_EOB = 2, IK_OTHER = 3 };

// the payload as dwords of the 4-aligned stream around it: 64 of them in a
// register (dword wbase + lane), the bits of any position fetched by ds_bpermute
struct SpecWin {
    const uint32_t* a0;   // payload start rounded down to 4 bytes
    uint32_t boff;        // bit offset of payload byte 0 in that stream
    uint32_t ndw;         // dwords that may be read (payload + the body's slack)
    uint32_t wbase;       // stream dword held by lane 0
    uint32_t v;
};

__device__ __forceinline__ void spec_win_at(SpecWin& W, uint32_t dw, uint32_t lane) {
    W.wbase = __builtin_amdgcn_readfirstlane(dw);
    W.v = W.wbase + lane < W.ndw ? W.a0[W.wbase + lane] : 0u;
}

template <uint32_t OUTMAX>
__device__ __forceinline__ uint32_t spec_item(const InfSmem<OUTMAX>& S, const SpecWin& W, uint32_t p,
                                              uint32_t nbits, uint32_t& kind, uint32_t& val,
                                              uint32_t& L, uint32_t& D) {
    // 64 payload bits from bit p (zero past the payload): three window dwords
    const uint32_t P = p + W.boff;
    const int di = (int)((P >> 5) - W.wbase) << 2;
    const uint32_t sh = P & 31;
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_ds_bpermute(di, (int)W.v);
    const uint32_t d1 = (uint32_t)__builtin_amdgcn_ds_bpermute(di + 4, (int)W.v);
    const uint32_t d2 = (uint32_t)__builtin_amdgcn_ds_bpermute(di + 8, (int)W.v);
    const uint64_t lo = (uint64_t)d0 | (uint64_t)d1 << 32;
    uint64_t b = sh ? (lo >> sh) | ((uint64_t)d2 << (64 - sh)) : lo;
    const uint32_t avail = nbits > p ? nbits - p : 0u;
    if (avail < 64) b &= (1ull << avail) - 1;
    // branch-free: both the literal and the length/distance reading are
    // computed for every lane (the distance table is read unconditionally)
    const uint32_t e = S.lut[0][b & ((1u << LUTB) - 1)];
    const uint32_t c1 = (e >> 1) & 15, sym = e >> 5;
    const bool lit = sym < 256, eob = sym == 256;
    const uint32_t k = min(sym - 257u, 28u);                  // (literals: clamped, unused)
    const uint32_t eb = (k < 8 || k == 28) ? 0u : (k >> 2) - 1;
    const uint32_t lbase = k < 8 ? 3 + k : k == 28 ? 258u : ((4u | (k & 3)) << eb) + 3;
    const uint32_t o2 = c1 + eb;
    const uint32_t e2 = S.lut[1][(b >> o2) & ((1u << LUTB) - 1)];
    const uint32_t c2 = (e2 >> 1) & 15, ds = min(e2 >> 5, 29u);
    const uint32_t deb = ds < 4 ? 0u : (ds >> 1) - 1;
    const uint32_t dbase = ds < 4 ? ds + 1 : ((2u | (ds & 1)) << deb) + 1;
    const bool match = !lit && !eob;
    const uint32_t need = match ? o2 + c2 + deb : c1;
    kind = lit ? IK_LIT : eob ? IK_EOB : IK_MATCH;
    val = sym;
    L = eob ? c1 : lbase + (uint32_t)((b >> c1) & ((1u << eb) - 1));
    D = dbase + (uint32_t)((b >> (o2 + c2)) & ((1u << deb) - 1));
    // a code beyond the tables goes to the serial decoder (which also sees any
    // error of that item); otherwise every zlib error of the item
    const bool slow = e == LUT_LONG || (match && (e & 1) && sym - 257u < 29u && e2 == LUT_LONG);
    const bool bad = !(e & 1) || (match && (sym - 257u >= 29u || !(e2 & 1) || (e2 >> 5) >= 30)) || need > avail;
    return slow ? IT_SLOW : bad ? IT_ERR : eob ? IT_EOB : p + need;
}

// symbols of one Huffman block from the reader's position to its end-of-block
// code; the reader is left after it.  0 done, -1 invalid, -2 too large.
template <uint32_t OUTMAX>
__device__ int inflate_block_par(InfSmem<OUTMAX>& S, InBits& I, const uint8_t* g, uint32_t plen,
                                 uint32_t& op, uint32_t lane ISTAMP_PARAMS) {
    const uint32_t nbits = plen * 8;
    uint32_t p0 = __builtin_amdgcn_readfirstlane(I.pos * 8 - I.cnt);
    SpecWin W;
    W.a0 = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(g) & ~(uintptr_t)3);
    W.boff = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 3) * 8;
    W.ndw = (W.boff / 8 + plen + 64) / 4;
    spec_win_at(W, (p0 + W.boff) >> 5, lane);
    for (;;) {
        const uint32_t w0 = p0;
        // positions w0 .. w0 + 255 read up to 64 bits each: stream dwords
        // (w0 + boff) / 32 .. + 10 must be in the register window
        if (((w0 + W.boff) >> 5) + 11 > W.wbase + 64) spec_win_at(W, (w0 + W.boff) >> 5, lane);
        uint32_t nx[4], kd[4], vl[4], ln[4], dd[4];
#pragma unroll
        for (int q = 0; q < 4; q++) nx[q] = spec_item(S, W, w0 + lane + 64 * q, nbits, kd[q], vl[q], ln[q], dd[q]);
        ISTAMP(4);
        // the item chain through this window (scalar): positions relative to
        // the current 64-position block, next positions >= 2^31 are stops
        // (items are shorter than 64 bits: a block's chain ends in the next)
        uint32_t nr[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            nr[q] = nx[q] >= IT_EOB ? 0x80000000u | (nx[q] - IT_EOB) : nx[q] - (w0 + 64u * q);
        uint64_t mk[4] = {0, 0, 0, 0};
        uint32_t r = 0, rp = 0, qs = 0, stop = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (r < 64) {
                uint64_t m = 0;
                do {
                    const uint32_t t = readlane(nr[q], r);
                    m |= 1ull << r;
                    rp = r;
                    r = t;
                } while (r < 64);
                mk[q] = m;
                if (r >= 0x80000000u) {
                    stop = IT_EOB + (r & 0x7FFFFFFFu);
                    qs = q;
                } else {
                    r -= 64;
                }
            }
        }
        // s: the stop item's position, else the first position past the window
        uint32_t s = stop ? w0 + 64u * qs + rp : w0 + 256u + r;
        if (stop == IT_SLOW) {   // (the serial decoder writes that item)
#pragma unroll
            for (int q = 0; q < 4; q++) mk[q] &= qs == (uint32_t)q ? ~(1ull << rp) : ~0ull;
        }
        ISTAMP(5);
        if (stop == IT_ERR) return -1;
        // the chain's items in bit order: output offsets, checks, entries
        uint32_t ko[4];
        uint32_t base = op;
        bool bad = false, big = false, lng = false;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bool me = (mk[q] >> lane) & 1;
            const uint32_t ol = me ? (kd[q] == IK_LIT ? 1u : kd[q] == IK_MATCH ? ln[q] : 0u) : 0u;
            const uint32_t incl = wave_incl_sum(ol);
            ko[q] = base + incl - ol;
            base += readlane(incl, 63);
            if (me && kd[q] == IK_MATCH) {
                bad |= dd[q] > ko[q];
                lng |= ln[q] > INF_SHORT;
            }
            if (me && ol) big |= ko[q] + ol > S.cap();
        }
        if (__any(bad)) return -1;
        if (__any(big)) return -2;
        ISTAMP(1);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (!((mk[q] >> lane) & 1)) continue;
            if (kd[q] == IK_LIT) {
                S.src()[ko[q]] = (inf_map_t<OUTMAX>)(inf_lit<OUTMAX> | vl[q]);
            } else if (kd[q] == IK_MATCH && ln[q] <= INF_SHORT) {
                const uint32_t m0 = ko[q] - dd[q];
                uint32_t c = 0;
                for (uint32_t t = 0; t < ln[q]; t++) {
                    S.src()[ko[q] + t] = (inf_map_t<OUTMAX>)(m0 + c);
                    if (++c == dd[q]) c = 0;
                }
            }
        }
        uint64_t lm = __ballot(lng);
        while (lm) {
            const uint32_t l = (uint32_t)__builtin_ctzll(lm);
            lm &= lm - 1;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (!((mk[q] >> l) & 1) || readlane(kd[q], l) != IK_MATCH) continue;
                const uint32_t Lm = readlane(ln[q], l);
                if (Lm <= INF_SHORT) continue;
                const uint32_t O = readlane(ko[q], l), Dm = readlane(dd[q], l), m0 = O - Dm;
                if (Dm >= Lm) {   // no overlap: the entries run along the source
                    for (uint32_t b = lane; b < Lm; b += 64) S.src()[O + b] = (inf_map_t<OUTMAX>)(m0 + b);
                } else {          // the period before the match: m0 + t mod D (rcp estimate, fixed up)
                    const float rd = __builtin_amdgcn_rcpf((float)Dm);
                    for (uint32_t b = lane; b < Lm; b += 64) {
                        int r = (int)b - (int)((float)b * rd) * (int)Dm;
                        r += r < 0 ? (int)Dm : 0;
                        r -= r >= (int)Dm ? (int)Dm : 0;
                        S.src()[O + b] = (inf_map_t<OUTMAX>)(m0 + (uint32_t)r);
                    }
                }
            }
        }
        op = base;
        ISTAMP(6);
        if (stop == IT_EOB) {                    // the block ends after the end-of-block code
            const uint32_t r = s - w0;
            uint32_t c1;
            switch (r >> 6) {   // (constant register indices)
            case 0: c1 = readlane(ln[0], r & 63); break;
            case 1: c1 = readlane(ln[1], r & 63); break;
            case 2: c1 = readlane(ln[2], r & 63); break;
            default: c1 = readlane(ln[3], r & 63); break;
            }
            in_seek(I, s + c1);
            return 0;
        }
        if (stop == IT_SLOW) {                   // a code beyond the table: the serial decoder
            in_seek(I, s);
            const int rc = inf_item_serial(S, I, op, lane);
            if (rc < 0) return rc;
            if (rc == 1) return 0;
            p0 = __builtin_amdgcn_readfirstlane(I.pos * 8 - I.cnt);
            continue;
        }
        p0 = s;
    }
}

// ---- the dynamic block header's code lengths (RFC 1951 3.2.7), decoded like
// the symbols: every lane decodes one code-length item (symbol 0..15, or 16 /
// 17 / 18 with their 2 / 3 / 7 extra bits) at each of 4 bit positions of a
// 256-bit window; the scalar unit follows the item chain (next position and
// count per item, stopping when nlen + ndist lengths are known); the chain's
// items are laid out by prefix sums of their counts, a 16 takes the value of
// the last earlier non-16 item (a max scan), and lengths land at [0, nlen)
// and [288, 288 + ndist) of lens[] (zeroed: 17 and 18 write nothing).
// Same errors as the serial loop: a 16 first, a count past the total, a code
// outside the table, a truncated payload.
template <uint32_t OUTMAX>
__device__ int inflate_lens_par(InfSmem<OUTMAX>& S, InBits& I, const uint8_t* g, uint32_t plen,
                                uint32_t nlen, uint32_t ndist, uint32_t lane) {
    const uint32_t nbits = plen * 8, tot = nlen + ndist;
    uint32_t p0 = __builtin_amdgcn_readfirstlane(I.pos * 8 - I.cnt);
    SpecWin W;
    W.a0 = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(g) & ~(uintptr_t)3);
    W.boff = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 3) * 8;
    W.ndw = (W.boff / 8 + plen + 64) / 4;
    spec_win_at(W, (p0 + W.boff) >> 5, lane);
    uint32_t have = 0, last = 0x100u;   // last: the latest length + 1 (0x100: none yet)
    for (;;) {
        const uint32_t w0 = p0;
        if (((w0 + W.boff) >> 5) + 11 > W.wbase + 64) spec_win_at(W, (w0 + W.boff) >> 5, lane);
        uint32_t nx[4], sy[4], ct[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t p = w0 + lane + 64 * q;
            const uint32_t P = p + W.boff;
            const int di = (int)((P >> 5) - W.wbase) << 2;
            const uint32_t sh = P & 31;
            const uint32_t d0 = (uint32_t)__builtin_amdgcn_ds_bpermute(di, (int)W.v);
            const uint32_t d1 = (uint32_t)__builtin_amdgcn_ds_bpermute(di + 4, (int)W.v);
            uint32_t b = sh ? (d0 >> sh) | (d1 << (32 - sh)) : d0;   // 32 bits from p
            const uint32_t avail = nbits > p ? nbits - p : 0u;
            if (avail < 32) b &= (1u << avail) - 1u;
            const uint32_t e = S.lut[0][b & ((1u << LUTB) - 1)];
            const uint32_t c = (e >> 1) & 15, y = e >> 5;
            const uint32_t eb = y == 16 ? 2u : y == 17 ? 3u : y == 18 ? 7u : 0u;
            const uint32_t x = (b >> c) & ((1u << eb) - 1u);
            sy[q] = y;
            ct[q] = y < 16 ? 1u : y == 18 ? 11u + x : 3u + x;
            nx[q] = (e & 1) && c + eb <= avail ? p + c + eb : IT_ERR;
        }
        // the chain through this window (scalar): stops at the total
        uint64_t mk[4] = {0, 0, 0, 0};
        uint32_t s = p0, h = have;
        bool err = false;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t hi = w0 + 64u * (q + 1);
            uint64_t m = 0;
            while (!err && h < tot && s < hi) {
                const uint32_t r = s - w0 - 64u * q;
                const uint32_t t = readlane(nx[q], r);
                const uint32_t k = readlane(ct[q], r);
                if (t == IT_ERR || h + k > tot) { err = true; break; }
                m |= 1ull << r;
                h += k;
                s = t;
            }
            mk[q] = m;
        }
        if (err) return -1;
        // offsets (prefix sums of counts in bit order) and 16's values (the
        // latest earlier non-16 item: a max scan of position | value + 1)
        uint32_t base = have, lastv = last;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bool me = (mk[q] >> lane) & 1u;
            const uint32_t k = me ? ct[q] : 0u;
            const uint32_t incl = wave_incl_sum(k);
            const uint32_t off = base + incl - k;
            base += readlane(incl, 63);
            const uint32_t y = sy[q];
            const uint32_t tag = me && y != 16 ? (lane + 1) << 9 | (y < 16 ? y + 1 : 1u) : 0u;
            const uint32_t mx = (uint32_t)wave_excl_max((int)tag, 0);
            const uint32_t val = mx ? (mx & 0x1FFu) : lastv;     // value + 1 (0x100: none)
            if (__any(me && y == 16 && val == 0x100u)) return -1;   // 16 with no earlier length
            const uint32_t v = (y == 16 ? val : y < 16 ? y + 1 : 1u) - 1;
            if (me && v) {
                for (uint32_t t = 0; t < k; t++) {
                    const uint32_t o = off + t;
                    S.lens[o < nlen ? o : 288 + (o - nlen)] = (uint8_t)v;
                }
            }
            // carry: the value after this block of 64 positions
            const uint32_t tall = (uint32_t)wave_max_i32((int)tag);
            lastv = tall ? (tall & 0x1FFu) : lastv;
        }
        have = base;
        last = lastv;
        if (have >= tot) {
            in_seek(I, s);
            return 0;
        }
        p0 = s;
    }
}

// the whole zlib stream; returns the decoded length, -1 invalid, -2 output
// larger than OUTMAX (host path)
template <uint32_t OUTMAX>
__device__ int64_t inflate_stream(InfSmem<OUTMAX>& S, const uint8_t* g, uint32_t plen, const uint16_t* fixed,
                                  uint32_t lane ISTAMP_PARAMS) {
    InBits I;
    I.g = g;
    I.plen = plen;
    I.buf = 0;
    I.cnt = 0;
    I.pos = 0;
    I.lane = lane;
    in_window(I, 0);
    uint32_t v;
    if (!in_take(I, 16, v)) return -1;
    const uint32_t cmf = v & 0xFF, flg = v >> 8;
    if (((cmf << 8) | flg) % 31) return -1;            // incorrect header check
    if ((cmf & 15) != 8) return -1;                    // unknown compression method
    if ((cmf >> 4) + 8 > 15) return -1;                // invalid window size
    if (flg & 0x20) return -1;                         // preset dictionary: zlib.decompress raises
    uint32_t op = 0;
    for (;;) {
        uint32_t hdr;
        if (!in_take(I, 3, hdr)) return -1;
        const uint32_t bfinal = hdr & 1, btype = hdr >> 1;
        if (btype == 0) {
            // stored: to the byte boundary, LEN, NLEN
            I.buf >>= (I.cnt & 7);
            I.cnt -= (I.cnt & 7);
            uint32_t ln, nl;
            if (!in_take(I, 16, ln) || !in_take(I, 16, nl)) return -1;
            if (ln != (~nl & 0xFFFF)) return -1;
            if (op + ln > S.cap()) return -2;
            // the buffered bytes first, then straight from the payload
            uint32_t k = 0;
            while (k < ln && I.cnt >= 8) {
                if (lane == 0) S.src()[op + k] = (inf_map_t<OUTMAX>)(inf_lit<OUTMAX> | (I.buf & 0xFF));
                I.buf >>= 8;
                I.cnt -= 8;
                k++;
            }
            if (I.pos + (ln - k) > plen) return -1;
            for (uint32_t b = 0; b < ln - k; b += 64)
                if (b + lane < ln - k) S.src()[op + k + b + lane] = (inf_map_t<OUTMAX>)(inf_lit<OUTMAX> | g[I.pos + b + lane]);
            I.pos += ln - k;
            op += ln;
        } else if (btype == 1 || btype == 2) {
            if (btype == 1 && fixed) {
                fixed_tables_in(S, fixed, lane);     // built once per device
            } else if (btype == 1) {
                fixed_tables_build(S, lane);
            } else {
                uint32_t h;
                if (!in_take(I, 14, h)) return -1;
                const uint32_t nlen = 257 + (h & 31), ndist = 1 + ((h >> 5) & 31), ncode = 4 + (h >> 10);
                if (nlen > 286 || ndist > 30) return -1;
                for (uint32_t s = lane; s < 320; s += 64) S.lens[s] = 0;
                wave_sync();
                // the ncode 3-bit code-length code lengths, at most 57 bits, in one read
                uint32_t c0, c1 = 0;
                if (!in_take(I, min(ncode, 10u) * 3, c0)) return -1;
                if (ncode > 10 && !in_take(I, (ncode - 10) * 3, c1)) return -1;
                if (lane < ncode) S.lens[c_clord2[lane]] = (uint8_t)((lane < 10 ? c0 >> (3 * lane) : c1 >> (3 * (lane - 10))) & 7u);
                wave_sync();
                if (!uniform_u32(inf_build<1>(S, 0, S.lens, 19, 0, lane))) return -1;
                wave_sync();
                for (uint32_t s = lane; s < 19; s += 64) S.lens[s] = 0;
                wave_sync();
                if (inflate_lens_par(S, I, g, plen, nlen, ndist, lane) < 0) return -1;
                wave_sync();
                // literal/length lengths live at [0, nlen) (rest 0 up to 288), distances at [288, 288+ndist)
                for (uint32_t s = nlen + lane; s < 288; s += 64) S.lens[s] = 0;
                for (uint32_t s = 288 + ndist + lane; s < 320; s += 64) S.lens[s] = 0;
                wave_sync();
                if (__builtin_amdgcn_readfirstlane(S.lens[256]) == 0) return -1;  // missing end-of-block code
                if (!uniform_u32(inf_build<5>(S, 0, S.lens, 288, 1, lane))) return -1;
                if (!uniform_u32(inf_build<1>(S, 1, S.lens + 288, 32, 1, lane))) return -1;
            }
            ISTAMP(0);
            {
                const int rc = inflate_block_par(S, I, g, plen, op, lane ISTAMP_ARGS);
                if (rc < 0) return rc;
            }
            ISTAMP(1);
        } else {
            return -1;  // invalid block type
        }
        if (bfinal) break;
    }
    // Adler-32, big-endian, after the byte boundary
    I.buf >>= (I.cnt & 7);
    I.cnt -= (I.cnt & 7);
    uint32_t a0, a1;
    if (!in_take(I, 16, a0) || !in_take(I, 16, a1)) return -1;
    const uint32_t want = ((a0 & 0xFF) << 24) | ((a0 >> 8) << 16) | ((a1 & 0xFF) << 8) | (a1 >> 8);
    wave_sync();
    // resolve the map (pointer jumping)
    for (;;) {
        bool more = false;
        for (uint32_t q0 = lane * 4; q0 < op; q0 += 256) {
            uint32_t w[4];
#pragma unroll
            for (int t = 0; t < 4; t++) w[t] = q0 + t < op ? S.src()[q0 + t] : inf_lit<OUTMAX>;
#pragma unroll
            for (int t = 0; t < 4; t++)
                if (!(w[t] & inf_lit<OUTMAX>)) {
                    w[t] = S.src()[w[t]];
                    S.src()[q0 + t] = (inf_map_t<OUTMAX>)w[t];
                    more |= !(w[t] & inf_lit<OUTMAX>);
                }
        }
        wave_sync();
        if (!__any(more)) break;
    }
    uint64_t asum = 0, bsum = 0;
    for (uint32_t q = lane; q < op; q += 64) {
        const uint32_t c = S.src()[q] & 0xFF;
        asum += c;
        bsum += (uint64_t)(op - q) * c;
    }
    ISTAMP(2);
    asum = wave_sum<uint64_t>(asum);
    bsum = wave_sum<uint64_t>(bsum);
    const uint32_t adler = (uint32_t)(((op + bsum) % 65521) << 16 | ((1 + asum) % 65521));
    if (adler != want) return -1;
    return (int64_t)op;
}

template <uint32_t OUTMAX>
__global__ __launch_bounds__(64) void k_decode_inflate(DecArgs A) {
    __shared__ InfSmem<OUTMAX> S;
    const uint32_t lane = threadIdx.x;
    const uint32_t j = uniform_u32(A.list ? A.list[blockIdx.x] : blockIdx.x);
    const DecJob J = A.jobs[j];
    uint8_t* out = uniform_ptr(A.out + J.out_off);
    const uint32_t orig = uniform_u32(J.orig);
    if constexpr (InfSmem<OUTMAX>::G) {
        S.srcg = reinterpret_cast<inf_map_t<OUTMAX>*>(A.scratch + J.scratch_off);
        S.capg = uniform_u32((uint32_t)J.scratch_cap);
    }
#ifdef AMBC_STAMPS
    uint64_t _st_t = __builtin_amdgcn_s_memtime();
    uint64_t _acc[7] = {0, 0, 0, 0, 0, 0, 0};
#endif
    const int64_t r = inflate_stream(S, uniform_ptr(A.body + J.body_off), uniform_u32(J.clen), A.inf_fixed,
                                     lane ISTAMP_ARGS);
    wave_sync();
    if (r == -2) {  // larger than the map: the host inflates it
        if (lane == 0) A.produced[j] = 0xFFFFFFFEu;
        return;
    }
    if (r < 0) {
        for (uint32_t q = lane; q < orig; q += 64) out[q] = 0;
    } else {
        const uint32_t m = min((uint32_t)r, orig);
        const uint32_t head = min((uint32_t)((4 - (reinterpret_cast<uintptr_t>(out) & 3)) & 3), m);
        if (lane < head) out[lane] = (uint8_t)(S.src()[lane] & 0xFF);
        const uint32_t nw = (m - head) >> 2;
        uint32_t* o32 = reinterpret_cast<uint32_t*>(out + head);
        for (uint32_t w = lane; w < nw; w += 64) {
            const uint32_t q = head + 4 * w;
            o32[w] = (S.src()[q] & 0xFFu) | (S.src()[q + 1] & 0xFFu) << 8 | (S.src()[q + 2] & 0xFFu) << 16 |
                     (S.src()[q + 3] & 0xFFu) << 24;
        }
        for (uint32_t q = head + (nw << 2) + lane; q < m; q += 64) out[q] = (uint8_t)(S.src()[q] & 0xFF);
        for (uint32_t q = m + lane; q < orig; q += 64) out[q] = 0;
    }
    if (lane == 0) A.produced[j] = orig;
#ifdef AMBC_STAMPS
    ISTAMP(3);
    if (lane == 0 && A.stamps) {
        for (int q = 0; q < 7; q++) A.stamps[(uint64_t)j * 8 + q] = _acc[q];
        A.stamps[(uint64_t)j * 8 + 7] = 5;
    }
#endif
}

}  // namespace

hipError_t launch_inflate_fixed_tables(uint16_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_inflate_fixed, dim3(1), dim3(64), 0, s, out);
    return hipGetLastError();
}

hipError_t launch_inflate(int kind, const DecArgs& a, hipStream_t s) {
    if (a.n_list == 0) return hipSuccess;
    if (kind == DEC_KIND_INFLATE_4K)
        hipLaunchKernelGGL(k_decode_inflate<4096>, dim3(a.n_list), dim3(64), 0, s, a);
    else if (kind == DEC_KIND_INFLATE_8K)
        hipLaunchKernelGGL(k_decode_inflate<8192>, dim3(a.n_list), dim3(64), 0, s, a);
    else if (kind == DEC_KIND_INFLATE_16K)
        hipLaunchKernelGGL(k_decode_inflate<16384>, dim3(a.n_list), dim3(64), 0, s, a);
    else if (kind == DEC_KIND_INFLATE_32K)  // 64 KB source map + tables: 2 workgroups per CU
        hipLaunchKernelGGL(k_decode_inflate<32768>, dim3(a.n_list), dim3(64), 0, s, a);
    else  // the map in device scratch
        hipLaunchKernelGGL(k_decode_inflate<65536>, dim3(a.n_list), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace ambc
