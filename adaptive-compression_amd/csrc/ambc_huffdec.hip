// ambc_huffdec.hip -- Huffman (id 3) package decoder for gfx950, one wave per
// package, every lane decoding.
//
// Reference: HuffmanCompression.decompress (compression_methods.py:407-470)
// with the tree of _build_huffman_tree / _build_tree_from_codes (:472-532):
//   [k:u8][k x (byte:u8, count:u32le)][nbits:u32le][bits, MSB first]
//   * the table is a dict: a repeated byte keeps its first slot and its last
//     count; an entry whose byte lies past the payload is an IndexError;
//   * heapq pops [weight, [byte, code], ...] lists: the smaller (weight, first
//     byte) first; lo's codes get '0', hi's '1'; fewer than two distinct bytes
//     -> IndexError (code[-1] of '' / heappop of an empty heap);
//   * nbits is capped by the bytes present; a code cut by the end of the bits
//     yields nothing; the walk stops once len(out) >= original_length, so it
//     yields min(symbols, max(orig, 1)) bytes -- one symbol when orig is 0.
// A codec exception becomes orig zero bytes (adaptive_compressor.py:440-442).
//
// Design (round 6):
//   1. table: lane-parallel parse (LDS max per byte for "last count wins");
//   2. tree: the exact heap order by repeated two-smallest reductions of
//      (weight << 8 | first byte) keys over the wave (DPP, both minima in one
//      pass); children of every merge in LDS;
//   3. a 2^HB-entry lookup table (leaf: byte + length, else the node reached
//      after HB bits), filled by 16 interleaved walks per lane;
//   4. the bits staged in LDS as big-endian words; 64 lanes decode 64 equal
//      segments at once, each starting HWARM bits early (Huffman codes resync
//      within a few codewords).  Lane l's first codeword boundary at or after
//      its segment start must equal lane l-1's first boundary at or after its
//      segment end; by induction from lane 0 (which starts at bit 0) that makes
//      every lane exact.  A lane that disagrees decodes again from its
//      predecessor's boundary (repeated until none disagrees: the lowest
//      disagreeing lane is always fixed, so at most 63 rounds; usually none);
//   5. symbol counts -> output offsets (wave prefix sum); each lane decodes
//      its segment once more into an LDS copy of the output, which goes to
//      HBM with dword stores.
// LDS at OUTMAX = 4096: 11.3 KB (14 workgroups per CU; k_decode held 25 KB).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {

namespace {

constexpr uint32_t HB = 10;               // primary lookup bits
constexpr uint32_t HWARM = 64;            // warm-up bits before a lane's segment
constexpr uint32_t TERM = 0xFFFFFFFFu;    // "no further boundary": the stream has ended

template <uint32_t OUTMAX>
struct HuffSmem {
    uint32_t bits[OUTMAX / 4 + 8];        // code bits as big-endian words, zero padded
    union {
        uint8_t out[OUTMAX];              // decoded bytes (last phase)
        struct {
            uint32_t cnt[256];            // count of byte s (its last entry's)
            uint32_t last[256];           // 1 + index of byte s's last entry, 0 = absent
        } t;                              // (table parse)
    };
    uint16_t lut[1u << HB];               // leaf: byte | len << 8; else 0x8000 | node after HB bits
    uint16_t child[256][2];               // internal node 256 + m: its '0' and '1' children
    uint32_t misc[4];
};

// the two smallest of two (a1 <= a2) pairs
__device__ __forceinline__ void pair_min(uint64_t& a1, uint64_t& a2, uint64_t b1, uint64_t b2) {
    const uint64_t lo = a1 < b1 ? a1 : b1;
    const uint64_t hi = a1 < b1 ? b1 : a1;
    const uint64_t m2 = a2 < b2 ? a2 : b2;
    a1 = lo;
    a2 = hi < m2 ? hi : m2;
}

template <int ctrl, int rm, int bm>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    const uint32_t lo = AMBC_DPP(0xFFFFFFFFu, (uint32_t)v, ctrl, rm, bm, false);
    const uint32_t hi = AMBC_DPP(0xFFFFFFFFu, (uint32_t)(v >> 32), ctrl, rm, bm, false);
    return (uint64_t)hi << 32 | lo;
}

// the two smallest keys of the wave (all lanes active); ~0 where absent
__device__ __forceinline__ void wave_two_min(uint64_t a1, uint64_t a2, uint64_t& k1, uint64_t& k2) {
#define AMBC_PAIR_STEP(ctrl, rm, bm)                                            \
    do {                                                                        \
        const uint64_t b1 = dpp_u64<ctrl, rm, bm>(a1), b2 = dpp_u64<ctrl, rm, bm>(a2); \
        pair_min(a1, a2, b1, b2);                                               \
    } while (0)
    AMBC_PAIR_STEP(0x111, 0xF, 0xF);   // row_shr:1
    AMBC_PAIR_STEP(0x112, 0xF, 0xF);   // row_shr:2
    AMBC_PAIR_STEP(0x114, 0xF, 0xF);   // row_shr:4
    AMBC_PAIR_STEP(0x118, 0xF, 0xF);   // row_shr:8
    AMBC_PAIR_STEP(0x142, 0xA, 0xF);   // row_bcast:15
    AMBC_PAIR_STEP(0x143, 0xC, 0xF);   // row_bcast:31
#undef AMBC_PAIR_STEP
    k1 = (uint64_t)readlane((uint32_t)(a1 >> 32), 63) << 32 | readlane((uint32_t)a1, 63);
    k2 = (uint64_t)readlane((uint32_t)(a2 >> 32), 63) << 32 | readlane((uint32_t)a2, 63);
}

__device__ __forceinline__ uint32_t le_part32(const uint8_t* p, uint32_t pos, uint32_t plen) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; b++)
        if (pos + b < plen) v |= (uint32_t)p[pos + b] << (8 * b);
    return v;
}

// bit reader over the staged big-endian words: buf holds `have` bits, MSB aligned
struct BitRd {
    uint64_t buf;
    uint32_t have, nw;
};

__device__ __forceinline__ void br_init(BitRd& b, const uint32_t* W, uint32_t pos) {
    const uint32_t w = pos >> 5, sh = pos & 31;
    b.buf = (((uint64_t)W[w] << 32) | W[w + 1]) << sh;
    b.have = 64 - sh;
    b.nw = w + 2;
}

__device__ __forceinline__ void br_skip(BitRd& b, const uint32_t* W, uint32_t len) {
    b.buf <<= len;
    b.have -= len;
    if (b.have <= 32) {
        b.buf |= (uint64_t)W[b.nw] << (32 - b.have);
        b.have += 32;
        b.nw++;
    }
}

__device__ __forceinline__ uint32_t bit_at(const uint32_t* W, uint32_t q) { return (W[q >> 5] >> (31 - (q & 31))) & 1u; }

// the codeword at bit pos: its byte and length; len = TERM where the bits end inside it
template <uint32_t OUTMAX>
__device__ __forceinline__ uint32_t huff_sym(const HuffSmem<OUTMAX>& S, const BitRd& b, uint32_t pos, uint32_t nbits,
                                             uint32_t& sym) {
    const uint32_t e = S.lut[(uint32_t)(b.buf >> (64 - HB))];
    if (!(e & 0x8000u)) {
        const uint32_t len = e >> 8;
        sym = e & 0xFFu;
        return len <= nbits - pos ? len : TERM;
    }
    // a code longer than HB bits: on down the tree a bit at a time (rare)
    uint32_t nd = e & 0x1FFu, len = HB;
    if (nbits - pos <= HB) return TERM;
    while (nd >= 256) {
        if (pos + len >= nbits) return TERM;
        nd = S.child[nd - 256][bit_at(S.bits, pos + len)];
        len++;
    }
    sym = nd;
    return len;
}

// One lane's decode from bit `start`: f = the first boundary >= s, cnt = the
// symbols starting in [s, e), exit = the first boundary >= e (TERM: the stream
// ended before e).  A code cut by the end of the bits is a boundary, no symbol.
template <uint32_t OUTMAX>
__device__ __forceinline__ void huff_scan(const HuffSmem<OUTMAX>& S, uint32_t start, uint32_t s, uint32_t e,
                                          uint32_t nbits, uint32_t& f, uint32_t& cnt, uint32_t& exit) {
    f = TERM;
    cnt = 0;
    exit = TERM;
    if (start >= nbits) return;
    BitRd b;
    br_init(b, S.bits, start);
    uint32_t pos = start;
    for (;;) {
        if (pos >= nbits) break;
        if (pos >= s && f == TERM) f = pos;
        if (pos >= e) { exit = pos; break; }
        uint32_t sym;
        const uint32_t len = huff_sym(S, b, pos, nbits, sym);
        if (len == TERM) break;
        cnt += pos >= s ? 1u : 0u;
        pos += len;
        if (len <= 32) br_skip(b, S.bits, len);
        else br_init(b, S.bits, pos);
    }
}

// returns the bytes produced into S.out, or -1 for a Python exception
template <uint32_t OUTMAX>
__device__ int64_t huff_decode(const uint8_t* p, uint32_t plen, uint32_t orig, HuffSmem<OUTMAX>& S, uint32_t lane,
                               unsigned long long* dbg) {
    // 1. the frequency table
    const uint32_t k = uniform_u32(p[0]);
    if (k && 1 + 5 * (k - 1) >= plen) return -1;
    for (uint32_t s = lane; s < 256; s += 64) S.t.last[s] = 0;
    __syncthreads();
    uint32_t eb[4], ec[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t e = lane + 64u * t;
        eb[t] = 0;
        ec[t] = 0;
        if (e < k) {
            eb[t] = p[1 + 5 * e];
            ec[t] = le_part32(p, 2 + 5 * e, plen);
            atomicMax(&S.t.last[eb[t]], e + 1);
        }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t e = lane + 64u * t;
        if (e < k && S.t.last[eb[t]] == e + 1) S.t.cnt[eb[t]] = ec[t];
    }
    __syncthreads();
    uint64_t key[4];
    uint32_t nid[4];
    uint32_t nf = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t s = lane + 64u * j;
        const bool have = S.t.last[s] != 0;
        key[j] = have ? ((uint64_t)S.t.cnt[s] << 8 | s) : ~0ull;
        nid[j] = s;
        nf += (uint32_t)__popcll(__ballot(have));
    }
    if (nf < 2) return -1;
    // 2. the heap's merges, exactly: the two smallest (weight, first byte) keys
    for (uint32_t m = 0; m + 1 < nf; m++) {
        uint64_t a1 = key[0], a2 = ~0ull;
#pragma unroll
        for (int j = 1; j < 4; j++) pair_min(a1, a2, key[j], ~0ull);
        uint64_t k1, k2;
        wave_two_min(a1, a2, k1, k2);
        const uint32_t s1 = (uint32_t)(k1 & 255), s2 = (uint32_t)(k2 & 255);
        const uint64_t merged = (((k1 >> 8) + (k2 >> 8)) << 8) | s1;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t s = lane + 64u * j;
            if (s == s1) {
                S.child[m][0] = (uint16_t)nid[j];
                key[j] = merged;
                nid[j] = 256 + m;
            } else if (s == s2) {
                S.child[m][1] = (uint16_t)nid[j];
                key[j] = ~0ull;
            }
        }
    }
    __syncthreads();
    const uint32_t root = 256 + nf - 2;
    // 3. the lookup table: 16 entries per lane, walked down together
    {
        uint32_t nd[16], dep[16];
#pragma unroll
        for (int i = 0; i < 16; i++) { nd[i] = root; dep[i] = 0; }
#pragma unroll
        for (uint32_t d = 0; d < HB; d++) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t v = lane + 64u * i;
                if (nd[i] >= 256) {
                    nd[i] = S.child[nd[i] - 256][(v >> (HB - 1 - d)) & 1];
                    dep[i] = d + 1;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 16; i++)
            S.lut[lane + 64u * i] = (uint16_t)(nd[i] < 256 ? (nd[i] | dep[i] << 8) : (0x8000u | nd[i]));
    }
    // 4. the bits, staged as big-endian words (bytes past the payload read as 0)
    const uint32_t b0 = 1 + 5 * k + 4;
    const uint32_t nbits_hdr = le_part32(p, 1 + 5 * k, plen);
    const uint32_t nbytes = plen > b0 ? plen - b0 : 0;
    const uint32_t nbits = (uint32_t)min((uint64_t)nbits_hdr, 8ull * nbytes);
    {
        const uint8_t* src = p + min(b0, plen);
        const uintptr_t sa = reinterpret_cast<uintptr_t>(src);
        const uint32_t sh = (uint32_t)(sa & 3);
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(sa & ~(uintptr_t)3);
        const uint32_t nw = (nbytes + 3) / 4;
        for (uint32_t w = lane; w < nw + 8; w += 64) {
            uint32_t v = 0;
            if (w < nw) {
                v = sh ? __builtin_amdgcn_alignbyte(s32[w + 1], s32[w], sh) : s32[w];
                const uint32_t valid = min(4u, nbytes - 4 * w);
                if (valid < 4) v &= (1u << (8 * valid)) - 1;
                v = __builtin_bswap32(v);
            }
            S.bits[w] = v;
        }
    }
    __syncthreads();
    // 5. 64 segments decoded at once, checked against each other
    const uint32_t seg = max(32u, ((nbits + 63) / 64 + 31) & ~31u);
    const uint32_t s = lane * seg;
    const uint32_t e = min(s + seg, nbits);
    uint32_t f, cnt, ex;
    if (s >= nbits) {
        f = TERM; cnt = 0; ex = TERM;
    } else {
        huff_scan(S, lane == 0 ? 0u : (s > HWARM ? s - HWARM : 0u), s, e, nbits, f, cnt, ex);
    }
    if (dbg) { dbg[lane * 8 + 0] = s; dbg[lane * 8 + 1] = f; dbg[lane * 8 + 2] = cnt; dbg[lane * 8 + 3] = ex; }
    int rounds = 0;
    for (int round = 0; round < 64; round++, rounds++) {
        const uint32_t prev = AMBC_DPP(TERM, ex, 0x138, 0xF, 0xF, false);   // wave_shr:1 -> lane l-1's exit
        const bool bad = lane != 0 && f != prev;
        if (!__any(bad)) break;
        if (bad) {
            if (s >= nbits) { f = TERM; cnt = 0; ex = TERM; }
            else huff_scan(S, prev, s, e, nbits, f, cnt, ex);
        }
    }
    if (dbg) { dbg[lane * 8 + 4] = f; dbg[lane * 8 + 5] = cnt; dbg[lane * 8 + 6] = ex; dbg[lane * 8 + 7] = rounds | (uint64_t)nbits << 32; }
    // 6. offsets, then every lane's symbols into the LDS output
    const uint32_t incl = wave_incl_sum(cnt);
    const uint32_t total = readlane(incl, 63);
    const uint32_t lim = max(orig, 1u);
    const uint32_t produced = min(total, lim);
    const uint32_t o = incl - cnt;
    // symbols this lane writes: those below `produced` (signed arithmetic: the
    // unsigned form `o < produced ? min(cnt, produced - o) : 0` lost its guard in
    // this kernel's code -- lanes past `produced` then wrote past the LDS output)
    const int32_t room = (int32_t)produced - (int32_t)o;
    const uint32_t n = room > 0 ? (uint32_t)min((int32_t)cnt, room) : 0u;
    if (n) {
        BitRd b;
        br_init(b, S.bits, f);
        uint32_t pos = f;
        for (uint32_t i = 0; i < n; i++) {
            uint32_t sym = 0;
            const uint32_t len = huff_sym(S, b, pos, nbits, sym);
            S.out[o + i] = (uint8_t)sym;
            pos += len;
            if (len <= 32) br_skip(b, S.bits, len);
            else br_init(b, S.bits, pos);
        }
    }
    return (int64_t)produced;
}

// Huffman packages with orig <= OUTMAX and clen <= OUTMAX (host / device walk routing)
template <uint32_t OUTMAX>
__global__ __launch_bounds__(64) void k_decode_huff(DecArgs A) {
    __shared__ HuffSmem<OUTMAX> S;
    const uint32_t lane = threadIdx.x;
    const uint32_t j = uniform_u32(A.list ? A.list[blockIdx.x] : blockIdx.x);
    const DecJob J = A.jobs[j];
    const uint8_t* p = uniform_ptr(A.body + J.body_off);
    uint8_t* out = uniform_ptr(A.out + J.out_off);
    const uint32_t orig = uniform_u32(J.orig), clen = uniform_u32(J.clen);
    int64_t produced = 0;
    if (clen) {
        const int64_t r = huff_decode<OUTMAX>(p, clen, orig, S, lane, A.stamps ? A.stamps + (uint64_t)blockIdx.x * 512 : nullptr);
        __syncthreads();
        if (r < 0) {
            for (uint32_t i = lane; i < orig; i += 64) out[i] = 0;
            produced = orig;
        } else {
            const uint32_t m = (uint32_t)r;
            // LDS -> output: dwords from the output's first aligned byte on
            const uint32_t head = min((uint32_t)((4 - (reinterpret_cast<uintptr_t>(out) & 3)) & 3), m);
            if (lane < head) out[lane] = S.out[lane];
            const uint32_t nw = (m - head) >> 2;
            uint32_t* d32 = reinterpret_cast<uint32_t*>(out + head);
            for (uint32_t w = lane; w < nw; w += 64) {
                const uint32_t q = head + 4 * w;
                d32[w] = (uint32_t)S.out[q] | (uint32_t)S.out[q + 1] << 8 | (uint32_t)S.out[q + 2] << 16 |
                         (uint32_t)S.out[q + 3] << 24;
            }
            for (uint32_t i = head + 4 * nw + lane; i < m; i += 64) out[i] = S.out[i];
            produced = r;
        }
    }
    if (lane == 0) A.produced[j] = (uint32_t)produced;
}

}  // namespace

hipError_t launch_huff(int kind, const DecArgs& a, hipStream_t s) {
    if (a.n_list == 0) return hipSuccess;
    if (kind == DEC_KIND_HUFF_4K) hipLaunchKernelGGL(k_decode_huff<4096>, dim3(a.n_list), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(k_decode_huff<8192>, dim3(a.n_list), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace ambc
