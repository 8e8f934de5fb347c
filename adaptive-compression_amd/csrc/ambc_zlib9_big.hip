// ambc_zlib9_big.hip -- zlib.compress(data, 9)'s bytes for chunks of 8193..65536 bytes.
//
// The reference's id 5 (advanced_compression.py:76-81) is eligible up to 65536
// bytes (adaptive_compressor.py:119), and its default walk tries 16 / 32 / 64 KiB
// candidates (:61-62).  ambc_zlib9.hip keeps the walkers' tables in LDS, which
// holds them up to 8 KiB; here the same algorithm (oracle/zlib9_model.c, zlib
// 1.2.11 deflate_slow + _tr_flush_block) runs with the tables in device scratch
// and adds what only long inputs reach:
//   - several blocks: zlib flushes a block with its 16383rd symbol (except the
//     final literal), so a chunk holds up to five blocks, each with its own
//     trees and stored / static / dynamic choice;
//   - distances past the window: a chain entry more than MAX_DIST = 32506 back
//     ends the search;
//   - the window slide past 65274 bytes (the NIL head at the slide step, no
//     stored block begun before 32768 once the window slid).
//
// k_z9_parse_big<CMAX>: a resident grid of 16-wave workgroups striding over the
// chunks, each with its own device scratch (Z9Big<CMAX>::BYTES):
//   1. stable counting sort of positions 1..n-3 by an 11-bit bucket of zlib's
//      15-bit hash: per-wave counters in LDS (one range of CMAX / 16 positions
//      per wave, ranks among peers by ballots), the sorted list and every
//      position's slot in scratch;
//   2. the chunk in LDS (zeros past n) and the lazy parse by 128 walkers
//      (8-lane groups, 8 candidates a step, the next step's list entries loaded
//      one step ahead); segments in scratch;
//   3. the path from 0: per 64-position window pointer doubling (exits + match
//      counts to scratch), one thread chains the windows, every window's path
//      walked on the scalar unit; the matches to the record, symbol starts and
//      coverage as LDS bitmasks;
//   4. the blocks: the 16383k-th symbols by a prefix count over the symbol-start
//      bitmask, each block's range, match rank and stored flag; per-block symbol
//      counts.
// k_z9_heap<CMAX> (ambc_z9.h): zlib's heap per (chunk, block), one per lane.
// k_z9_code_big<CMAX>: one wave per chunk.  Pass 1 builds every block's trees
// and knows the exact length; a chunk whose id 5 loses stops there.  Pass 2
// writes the package as one LSB-first bit stream (zlib header, blocks, Adler-32)
// through a 2 KB LDS ring whose finished words go to the chunk's slot after
// every 64-position round.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "ambc_internal.h"
#include "ambc_wave.h"
#include "ambc_z9.h"

namespace ambc {
namespace {

constexpr int ZB_NW = 16;                 // waves per chunk in k_z9_parse_big (64 / ZB_G walkers each)
#ifndef AMBC_Z9B_G
#define AMBC_Z9B_G 8
#endif
constexpr uint32_t ZB_G = AMBC_Z9B_G;      // lanes per walker (candidates per search step)
constexpr uint32_t ZB_GRID = 512;         // resident workgroups (2 per CU)
constexpr uint32_t Z_WSZ = 32768;         // w_size
constexpr uint32_t Z_SLIDE = 32768 + Z_MAXD;   // strstart that slides the window (65274)

#ifdef AMBC_STAMPS
// diagnostic build only: thread 0's phase cycles per parsed chunk in
// A.stamps[(2 M + k) * 8 + phase] (k_dict's slots; phase 7 = 1 marks a parse)
#define BSTAMP_DECL uint64_t _pt = __builtin_amdgcn_s_memtime(); uint64_t _pa[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define BSTAMP(ph)                                                 \
    do {                                                           \
        __builtin_amdgcn_s_waitcnt(0xC07F);                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();          \
        _pa[ph] += _t - _pt;                                       \
        _pt = _t;                                                  \
    } while (0)
#define BSTAMP_FLUSH                                                                  \
    if (threadIdx.x == 0 && A.stamps) {                                               \
        _pa[7] = 1;                                                                   \
        for (int _p = 0; _p < 8; _p++) A.stamps[(2ull * A.n_chunks + k) * 8 + _p] = _pa[_p]; \
    }
#else
#define BSTAMP_DECL
#define BSTAMP(ph) do {} while (0)
#define BSTAMP_FLUSH
#endif

template <int CMAX>
struct Z9Big {
    // 64 KiB: the sorted list takes the LDS, the chunk bytes stay in scratch
    // (zero-padded; 32 workgroups x 64 KB per XCD sit in its L2); smaller
    // chunks keep both in LDS
    static constexpr bool CHG = CMAX > 32768;
    static constexpr uint32_t RANGE = (uint32_t)CMAX / ZB_NW;   // sort positions per wave
    static constexpr uint32_t NBLK = Z9Rec<CMAX>::NBLK;
    // device scratch per resident workgroup (bytes)
    static constexpr size_t LST = 0;                        // u16 [CMAX] positions by bucket (the sort's output)
    static constexpr size_t SLOT = LST + 2ull * CMAX;       // u16 [CMAX] position -> index in the list
    static constexpr size_t SEG = SLOT + 2ull * CMAX;       // u32 [CMAX] the sort's ranks, then segments
    static constexpr size_t SD = SEG + 4ull * CMAX;         // u16 [CMAX] segment distances
    static constexpr size_t CH = SD + 2ull * CMAX;          // CHG: the chunk, zeros past n
    // CHG: the walk's byte-run starts (bitmask) and per-word run starts (u16),
    // which do not fit the LDS beside the list
    static constexpr size_t RUNB = (CH + (CHG ? (size_t)CMAX + 320 : 0) + 15) & ~(size_t)15;
    static constexpr size_t WRS = RUNB + (CHG ? (size_t)CMAX / 8 : 0);
    static constexpr size_t BYTES = WRS + (CHG ? (size_t)CMAX / 16 : 0);
};

template <int CMAX>
struct Z9BSmem {
    static constexpr bool CHG = Z9Big<CMAX>::CHG;
    static constexpr uint32_t NBLK = Z9Rec<CMAX>::NBLK;
    struct Walk {                                      // the walkers
        uint16_t lst[CMAX];                            // positions by bucket, ascending inside one
        alignas(16) uint8_t ch[CHG ? 16 : CMAX + 320]; // the chunk, zeros past n
    };
    struct Path {                                      // the path from 0
        union {
            uint16_t xit[CMAX];                        // exit offset from the window (10 bits) | matches << 10
            struct {
                uint32_t mask[CMAX / 32];              // match starts
                uint32_t cov[CMAX / 32];               // positions the matches cover
                uint32_t lf[NBLK][316];                // per-block symbol counts
            } b;
        };
        uint16_t entry[CMAX / 64], rbase[CMAX / 64];
    };
    union {
        uint16_t cnt[ZB_NW][ZNB];                      // the sort: per-wave bucket cursors
        Walk w;
        Path p;
    };
    uint32_t bend32[ZNB / 2];                          // bucket ends (u16 pairs)
    uint32_t vis[CMAX / 32];                           // clean positions some walker recorded
    uint32_t litm[CMAX / 32];                          // the walk: positions that take no match (z9b_literal_mask)
    uint32_t runb[CHG ? 1 : CMAX / 32];                //   byte-run starts, and every position >= n (CHG: scratch)
    uint16_t wrs[CHG ? 1 : CMAX / 32];                 //   the run holding position 32 w starts here (CHG: scratch)
    uint32_t bnd[8];                                   // block ends (boundary positions)
    uint32_t btop[8];                                  // the step top that flushed block b
    uint32_t nbnd, nmatch;
    __device__ __forceinline__ uint16_t* bend() { return reinterpret_cast<uint16_t*>(bend32); }
    __device__ __forceinline__ uint32_t bstart(uint32_t h) { return h ? bend()[h - 1] : 0u; }
};

// 3-gram at i of the chunk in global memory (i + 2 < n)
__device__ __forceinline__ uint32_t g_gram(const uint8_t* src, uint32_t i) {
    return (uint32_t)src[i] | (uint32_t)src[i + 1] << 8 | (uint32_t)src[i + 2] << 16;
}

// Stable counting sort of positions [1, m) by z_bucket(z_h15): wave w ranks
// the positions of its range [w RANGE, (w+1) RANGE) in order (ballots over the
// 11 bucket bits, per-wave LDS cursors); the per-bucket prefix over the waves
// and the bucket ends; then every position goes to lst[] and its index to
// slot[] (scratch; the list is copied into LDS once the cursors are dead).
template <int CMAX>
__device__ void z9b_sort(Z9BSmem<CMAX>& S, const uint8_t* src, uint32_t m, uint16_t* lst, uint16_t* slot,
                         uint32_t* loc, uint32_t wave, uint32_t lane) {
    constexpr uint32_t T = 64u * ZB_NW, RANGE = Z9Big<CMAX>::RANGE, GR = RANGE / 64;
    const uint32_t tid = wave * 64u + lane;
    uint32_t* c32 = reinterpret_cast<uint32_t*>(&S.cnt[0][0]);
    for (uint32_t b = tid; b < ZB_NW * ZNB / 2; b += T) c32[b] = 0;
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1ull;
    {
        uint16_t* c = S.cnt[wave];
#pragma unroll 2
        for (uint32_t g = 0; g < GR; g++) {
            const uint32_t i = wave * RANGE + g * 64 + lane;
            const bool v = i >= 1 && i < m;
            const uint32_t h = v ? z_bucket(z_h15(g_gram(src, i))) : 0u;
            uint64_t peers = __ballot(v);
#pragma unroll
            for (int b = 0; b < 11; b++) {
                const uint64_t mb = __ballot(v && ((h >> b) & 1u));
                peers &= ((h >> b) & 1u) ? mb : ~mb;
            }
            const uint32_t base = v ? (uint32_t)c[h] : 0u;
            loc[i] = v ? (base + (uint32_t)__popcll(peers & below)) | h << 16 : ~0u;
            if (v && (peers >> lane) == 1ull) c[h] = (uint16_t)(base + (uint32_t)__popcll(peers));
        }
    }
    __syncthreads();
    for (uint32_t h = tid; h < ZNB; h += T) {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)ZB_NW; r++) {
            const uint32_t x = S.cnt[r][h];
            S.cnt[r][h] = (uint16_t)run;
            run += x;
        }
        S.bend()[h] = (uint16_t)run;
    }
    __syncthreads();
    if (wave == 0) {
        uint32_t c[16], t = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            c[j] = S.bend32[lane * 16 + j];
            t += (c[j] & 0xFFFFu) + (c[j] >> 16);
        }
        uint32_t run = wave_incl_sum(t) - t;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t r0 = run + (c[j] & 0xFFFFu), r1 = r0 + (c[j] >> 16);
            S.bend32[lane * 16 + j] = r0 | r1 << 16;
            run = r1;
        }
    }
    __syncthreads();
#pragma unroll 2
    for (uint32_t g = 0; g < GR; g++) {
        const uint32_t i = wave * RANGE + g * 64 + lane;
        const uint32_t x = loc[i];   // (this lane's own store)
        if (x != ~0u) {
            const uint32_t h = x >> 16;
            const uint32_t idx = S.bstart(h) + S.cnt[wave][h] + (x & 0xFFFFu);
            lst[idx] = (uint16_t)i;
            slot[i] = (uint16_t)idx;
        }
    }
    __syncthreads();
}

// The lazy parse's walkers (ambc_zlib9.hip z9_walkers with the list in LDS,
// slots and segments in scratch, the chunk bytes in LDS or scratch, the
// candidates' words loaded one step ahead, the window's MAX_DIST, the slide
// step's NIL head, and the search stopped at the chain length the step needs).
// As ambc_zlib9.hip's z9_literal_mask: positions without any earlier same-hash
// position (and 0, and the last two) take no match; byte-run starts for the
// walkers' run shortcut, and per 32-position word the start of its first run.
template <int CMAX>
__device__ void z9b_literal_mask(Z9BSmem<CMAX>& S, uint32_t n, const uint16_t* slot, const uint8_t* gch,
                                 uint32_t* runb, uint16_t* wrs, uint32_t wave, uint32_t lane) {
    constexpr bool CHG = Z9Big<CMAX>::CHG;
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.w.ch);
    const uint32_t* g32 = reinterpret_cast<const uint32_t*>(gch);
    auto W32 = [&](uint32_t i) -> uint32_t {
        if constexpr (CHG) return g32[i];
        else return c32[i];
    };
    auto B8 = [&](uint32_t i) -> uint32_t {
        if constexpr (CHG) return gch[i];
        else return S.w.ch[i];
    };
    auto gram = [&](uint32_t i) -> uint32_t {
        return __builtin_amdgcn_alignbyte(W32((i >> 2) + 1), W32(i >> 2), i & 3) & 0xFFFFFFu;
    };
    for (uint32_t b = wave * 64u; b < (uint32_t)CMAX; b += 64u * ZB_NW) {
        const uint32_t p = b + lane;
        bool lit = true;
        if (p >= 1 && p + 3 <= n) {
            const uint32_t h = z_h15(gram(p));
            const uint32_t lo = S.bstart(z_bucket(h)), j = slot[p];
            if (j > lo + 4) {
                lit = false;
            } else {
                for (uint32_t t = lo; t < j; t++)
                    if (z_h15(gram(S.w.lst[t])) == h) { lit = false; break; }
            }
        }
        const uint64_t m = __ballot(lit);
        const uint64_t rm = __ballot(p == 0 || p >= n || B8(p) != B8(p - 1));
        if (lane == 0) {
            S.litm[b >> 5] = (uint32_t)m; S.litm[(b >> 5) + 1] = (uint32_t)(m >> 32);
            runb[b >> 5] = (uint32_t)rm; runb[(b >> 5) + 1] = (uint32_t)(rm >> 32);
        }
    }
    __syncthreads();
    if (wave == 0) {
        constexpr uint32_t NWD = (uint32_t)CMAX / 32, K = (NWD + 63) / 64;
        int last = -1;
#pragma unroll 1
        for (uint32_t t = 0; t < K; t++) {
            const uint32_t x = runb[lane * K + t];
            if (x) last = (int)((lane * K + t) * 32 + 31 - __builtin_clz(x));
        }
        int run = wave_excl_max(last, -1);
#pragma unroll 1
        for (uint32_t t = 0; t < K; t++) {
            const uint32_t w = lane * K + t, x = runb[w];
            wrs[w] = (uint16_t)((x & 1u) ? w * 32 : (uint32_t)max(run, 0));
            if (x) run = (int)(w * 32 + 31 - __builtin_clz(x));
        }
    }
}

template <int CMAX>
__device__ __forceinline__ void z9b_walkers(Z9BSmem<CMAX>& S, uint32_t n, const uint16_t* slot, uint32_t* seg,
                                            uint16_t* sd, const uint8_t* gch, const uint32_t* runb,
                                            const uint16_t* wrs, uint32_t wave, uint32_t lane,
                                            uint64_t* ctr = nullptr) {
#ifdef AMBC_STAMPS
    uint64_t c_it = 0, c_st = 0, c_ex = 0, c_sr = 0;   // loop iterations, chain steps, extension steps, searches
#endif
    constexpr bool CHG = Z9Big<CMAX>::CHG;
    constexpr uint32_t G = ZB_G;
    constexpr uint32_t NWK = (uint32_t)ZB_NW * (64u / G);
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(S.w.ch);
    const uint32_t* g32 = reinterpret_cast<const uint32_t*>(gch);
    auto W32 = [&](uint32_t i) -> uint32_t {
        if constexpr (CHG) return g32[i];
        else return c32[i];
    };
    auto B8 = [&](uint32_t i) -> uint32_t {
        if constexpr (CHG) return gch[i];
        else return S.w.ch[i];
    };
    const uint16_t* lst = S.w.lst;
    const uint32_t g = lane / G, r = lane % G;
    const uint32_t wid = wave * (64u / G) + g;
    // the step at which fill_window slides: the first top s >= 65274 with
    // lookahead < 262 (65275 for a 65536-byte input); at s = 65274 a hash head of
    // 32768 reads as NIL (inputs < 65536 only: later heads that far are past MAX_DIST)
    const uint32_t nil_at = n < 65536u ? Z_SLIDE : 0xFFFFFFFFu;
    uint32_t q = (uint32_t)(((uint64_t)n * wid) / NWK);
    uint32_t s = q, P = 2, Pd = 0, c = 0;
    bool clean = true, done = false;
#pragma unroll 1
    for (;;) {
        if (clean && !done && (q >= n || ((S.vis[q >> 5] >> (q & 31)) & 1u))) done = true;
        if (__all(done)) break;
#ifdef AMBC_STAMPS
        c_it++;
#endif
        // a run of match-less positions from a clean q in one step (at most 512:
        // the path's exit offsets hold 10 bits)
        bool skip = false;
        if (clean && !done && ((S.litm[q >> 5] >> (q & 31)) & 1u)) {
            uint32_t e = q;
            const uint32_t emax = min(n, q + 512u);
            for (;;) {
                const uint32_t sh = e & 31u;
                const uint32_t w = ~(S.litm[e >> 5] >> sh);
                const uint32_t t = w ? (uint32_t)__builtin_ctz(w) : 32u;
                if (t < 32u - sh) { e += t; break; }
                e += 32u - sh;
                if (e >= emax) break;
            }
            e = min(e, emax);
            if (r == 0) {
                seg[q] = 0x80000000u | (e - q);
                atomicOr(&S.vis[q >> 5], 1u << (q & 31));
            }
            q = e;
            s = q;
            skip = true;
        }
        const bool act = !done && !skip && s >= 1 && s + 3 <= n && P < 258;   // position 0 is zlib's NIL
        // ---- longest_match(s) over the first `lim` chain entries (4096, or
        // 1024 when the pending match is >= good_match); key = min(len, nice)
        // << 16 | candidate: the longest, then the most recent ----
        uint32_t k0 = 0;
        {
            uint32_t tg[4] = {0, 0, 0, 0}, h = 0, lo = 0, j = 0, nice = 0;
            const uint32_t ss = s & 3u;
            const uint32_t lim = P >= Z_GOOD ? Z_CHAIN / 4 : Z_CHAIN;
            if (act) {
                j = slot[s];
                const uint32_t a = s >> 2;
                uint32_t w[5];
#pragma unroll
                for (int t = 0; t < 5; t++) w[t] = W32(a + t);
#pragma unroll
                for (int t = 0; t < 4; t++) tg[t] = __builtin_amdgcn_alignbyte(w[t + 1], w[t], ss);
                h = z_h15(tg[0] & 0xFFFFFFu);
                lo = S.bstart(z_bucket(h));
                nice = min(Z_MAXM, n - s);
            }
            uint32_t cnt = 0;
            bool rgd = false;
            // inside a byte run (ambc_zlib9.hip): the run's earlier positions all
            // match exactly to its end, the most recent stands for them; a run
            // reaching MAX_DIST back ends the chain inside it
            if (act && s >= 2 && (tg[0] & 0xFFFFFFu) == (tg[0] & 0xFFu) * 0x010101u && B8(s - 1) == (tg[0] & 0xFFu)) {
                const uint32_t w = s >> 5, b = s & 31u;
                const uint32_t xb = runb[w] & (b == 31u ? ~0u : ((2u << b) - 1u));
                const uint32_t rs = max(1u, xb ? w * 32 + 31 - (uint32_t)__builtin_clz(xb) : (uint32_t)wrs[w]);
                uint32_t wf = w, xf = runb[w] & (b == 31u ? 0u : ~((2u << b) - 1u)), re = s + Z_MAXM + 3;
#pragma unroll 1
                for (int t = 0; t < 10; t++) {
                    if (xf) { re = wf * 32 + (uint32_t)__builtin_ctz(xf); break; }
                    if (++wf >= (uint32_t)CMAX / 32) { re = CMAX; break; }
                    xf = runb[wf];
                }
                const uint32_t B = s - rs;
                if (re >= s + 3 && B >= 8 && B <= j - lo && !(s == nil_at && s - 1 == Z_WSZ)) {
                    k0 = min(min(re - s, Z_MAXM), nice) << 16 | (s - 1);
                    cnt = B;
                    j -= B;
                    rgd = s - rs >= Z_MAXD;      // the chain's next entries lie past MAX_DIST
                }
            }
            bool gd = !act || rgd || j <= lo || cnt >= lim || (k0 >> 16) >= nice;
            int idx = (int)j - 1 - (int)r;
            // every lane loads (an index in range; lanes past the chain are masked by v)
            uint32_t cn = (uint32_t)lst[max(idx, 0)];
            uint32_t wn[5];
#pragma unroll
            for (int t = 0; t < 5; t++) wn[t] = W32((cn >> 2) + t);
#ifdef AMBC_STAMPS
            c_sr += (uint64_t)__popcll(__ballot(act && r == 0));
#endif
#pragma unroll 1
            while (__any(!gd)) {
#ifdef AMBC_STAMPS
                c_st++;
#endif
                const bool v = !gd & (idx >= (int)lo);
                const uint32_t c = cn;
                uint32_t w[5];
#pragma unroll
                for (int t = 0; t < 5; t++) w[t] = wn[t];
                // the next step's candidate and its words, issued now
                idx -= (int)G;
                cn = (uint32_t)lst[max(idx, 0)];
#pragma unroll
                for (int t = 0; t < 5; t++) wn[t] = W32((cn >> 2) + t);
                const uint32_t sh = c & 3u;
                uint32_t x[4];
#pragma unroll
                for (int t = 0; t < 4; t++) x[t] = __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
                const bool same = v & (z_h15(x[0] & 0xFFFFFFu) == h);
                const uint32_t sm = grp_bits<G>(__ballot(same), g);
                const uint32_t kidx = cnt + (uint32_t)__popc(sm & ((1u << r) - 1u)) + 1u;
                // the hash head may lie MAX_DIST back (deflate_slow's test is <=);
                // later chain entries must lie above limit = s - MAX_DIST
                const bool inwin = s - c < Z_MAXD || (s - c == Z_MAXD && kidx == 1u);
                const bool ok = same & inwin & (kidx <= lim);
                // the slide step: a head of 32768 is NIL, no search at all
                const bool nilh = grp_bits<G>(__ballot(same && kidx == 1u && c == Z_WSZ && s == nil_at), g) != 0;
                uint32_t fm = ~0u;
#pragma unroll
                for (int t = 0; t < 4; t++) fm = min(fm, ffbl_raw(x[t] ^ tg[t]) | (uint32_t)t << 5);
                uint32_t len = fm == ~0u ? 16u : fm >> 3;
                // zlib's scan_end test: only a candidate equal in its first 16
                // bytes can pass a best >= 16; it must also agree at byte best
                const uint32_t best = k0 >> 16;
                bool ext = ok && fm == ~0u && !nilh;
                if (ext && best >= 16) ext = B8(c + best) == B8(s + best);
                const bool can = fm != ~0u || best < 16 || ext;
                // the group extends its first-16-equal candidates together, most
                // recent first, 128 bytes a step, until one reaches nice
                uint32_t em = grp_bits<G>(__ballot(ext), g);
#pragma unroll 1
                while (__any(em != 0u)) {
#ifdef AMBC_STAMPS
                    c_ex++;
#endif
                    const bool gact = em != 0u;
                    const uint32_t rr = gact ? (uint32_t)__builtin_ctz(em) : 0u;
                    const uint32_t src = g * G + rr;
                    const uint32_t cc = (uint32_t)__shfl((int)c, (int)src);
                    const uint32_t ll = (uint32_t)__shfl((int)len, (int)src);
                    const uint32_t off = ll + 16u * r;
                    uint32_t f = ~0u;
                    if (gact && off < Z_MAXM) {
                        const uint32_t ac = (cc + off) >> 2, as = (s + off) >> 2, csh = cc & 3u;
                        uint32_t wc[5], ws[5];
#pragma unroll
                        for (int t = 0; t < 5; t++) { wc[t] = W32(ac + t); ws[t] = W32(as + t); }
#pragma unroll
                        for (int t = 0; t < 4; t++)
                            f = min(f, ffbl_raw(__builtin_amdgcn_alignbyte(wc[t + 1], wc[t], csh) ^
                                                __builtin_amdgcn_alignbyte(ws[t + 1], ws[t], ss)) |
                                           (uint32_t)t << 5);
                    } else if (gact) {
                        f = 0;
                    }
                    const uint32_t mm = grp_bits<G>(__ballot(gact && f != ~0u), g);
                    const uint32_t r0 = mm ? (uint32_t)__builtin_ctz(mm) : 0u;
                    const uint32_t f0 = (uint32_t)__shfl((int)f, (int)(g * G + r0));
                    const uint32_t L2 = mm ? ll + 16u * r0 + (f0 >> 3) : ll + 16u * G;
                    if (gact && r == rr) len = L2;
                    if (gact && (mm || L2 >= Z_MAXM)) {
                        em &= em - 1u;
                        if (min(L2, Z_MAXM) >= nice) em = 0;
                    }
                }
                const uint32_t Lp = min(min(len, Z_MAXM), nice);
                const uint32_t key = ok && can && !nilh ? (Lp << 16 | c) : 0u;
                k0 = nilh ? 0u : max(k0, grp_max<G>(key));
                cnt += (uint32_t)__popc(sm);
                const uint32_t far = grp_bits<G>(__ballot(v && s - c >= Z_MAXD), g);
                j = j > lo + G ? j - G : lo;
                gd = gd || nilh || j <= lo || far != 0 || cnt >= lim || (k0 >> 16) >= nice;
            }
        }
        if (!done && !skip) {
            uint32_t ML = 2, MD = 0;
            if (act) {
                const uint32_t L = k0 >> 16, d = s - (k0 & 0xFFFFu);
                if (L >= 3 && !(L == 3 && d > Z_TOOFAR)) { ML = L; MD = d; }
            }
            if (clean) {
                if (ML < 3) {
                    if (r == 0) {
                        seg[q] = 0x80000000u | 1u;
                        atomicOr(&S.vis[q >> 5], 1u << (q & 31));
                    }
                    q++;
                    s = q;
                } else {
                    P = ML;
                    Pd = MD;
                    c = 0;
                    s = q + 1;
                    clean = false;
                }
            } else if (ML <= P) {
                if (r == 0) {
                    sd[q] = (uint16_t)Pd;
                    seg[q] = 0x80000000u | P << 16 | c;
                    atomicOr(&S.vis[q >> 5], 1u << (q & 31));
                }
                q = s - 1 + P;
                s = q;
                P = 2;
                clean = true;
            } else {
                c++;
                P = ML;
                Pd = MD;
                s++;
            }
        }
    }
#ifdef AMBC_STAMPS
    if (ctr && lane == 0) *ctr = c_it | c_st << 16 | c_ex << 32 | c_sr << 48;
#endif
}


template <int CMAX>
__global__ __launch_bounds__(64 * ZB_NW) void k_z9_parse_big(EncArgs A) {
    constexpr uint32_t NW = ZB_NW, TT = 64u * NW;
    constexpr uint32_t NBLK = Z9Rec<CMAX>::NBLK;
    constexpr bool CHG = Z9Big<CMAX>::CHG;
    __shared__ Z9BSmem<CMAX> S;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1ull;
    uint8_t* scr = A.z9scr + (uint64_t)blockIdx.x * Z9Big<CMAX>::BYTES;
    uint16_t* glst = reinterpret_cast<uint16_t*>(scr + Z9Big<CMAX>::LST);
    uint16_t* slot = reinterpret_cast<uint16_t*>(scr + Z9Big<CMAX>::SLOT);
    uint32_t* seg = reinterpret_cast<uint32_t*>(scr + Z9Big<CMAX>::SEG);
    uint16_t* sd = reinterpret_cast<uint16_t*>(scr + Z9Big<CMAX>::SD);
    uint8_t* gch = scr + Z9Big<CMAX>::CH;
    uint32_t* runb = CHG ? reinterpret_cast<uint32_t*>(scr + Z9Big<CMAX>::RUNB) : S.runb;
    uint16_t* wrs = CHG ? reinterpret_cast<uint16_t*>(scr + Z9Big<CMAX>::WRS) : S.wrs;
#pragma unroll 1
    for (uint32_t k = blockIdx.x; k < A.n_chunks; k += gridDim.x) {
        __syncthreads();   // (the previous chunk's last LDS reads)
        const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
        const uint32_t n = A.coff ? (A.clen ? A.clen[k] : A.clen_all) : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
        uint32_t T = 0;
        if (n > (uint32_t)CMAX || !z9_gate(A, k, n, T)) continue;
        const uint8_t* src = A.in + pos0;
        BSTAMP_DECL
        // ---- 1. the sort (the ranks go through seg[]) ----
        z9b_sort(S, src, n - 2, glst, slot, seg, wave, lane);
        BSTAMP(0);
        // ---- 2. the list (and the chunk) in LDS, cleared segments, the walkers ----
        {
            const uint32_t m = n - 2;
            uint32_t* l32 = reinterpret_cast<uint32_t*>(S.w.lst);
            const uint32_t* g32 = reinterpret_cast<const uint32_t*>(glst);
            for (uint32_t i = threadIdx.x; i < (m + 1) / 2; i += TT) l32[i] = g32[i];
            uint8_t* dst = CHG ? gch : S.w.ch;
            if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
                const uint32_t nv = n >> 4;
                for (uint32_t q = threadIdx.x; q < nv; q += TT)
                    reinterpret_cast<uint4*>(dst)[q] = reinterpret_cast<const uint4*>(src)[q];
                for (uint32_t i = (nv << 4) + threadIdx.x; i < n; i += TT) dst[i] = src[i];
            } else {
                for (uint32_t i = threadIdx.x; i < n; i += TT) dst[i] = src[i];
            }
            for (uint32_t i = n + threadIdx.x; i < (uint32_t)CMAX + 320; i += TT) dst[i] = 0;
            for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX / 32; i += TT) S.vis[i] = 0;
        }
        __syncthreads();
        z9b_literal_mask(S, n, slot, gch, runb, wrs, wave, lane);
        __syncthreads();
        BSTAMP(1);
#ifdef AMBC_STAMPS
        uint64_t wctr = 0;
        z9b_walkers(S, n, slot, seg, sd, gch, runb, wrs, wave, lane, wave == 0 ? &wctr : nullptr);
        if (threadIdx.x == 0) _pa[6] = wctr;
#else
        z9b_walkers(S, n, slot, seg, sd, gch, runb, wrs, wave, lane);
#endif
        BSTAMP(2);
        __syncthreads();
        BSTAMP(3);
        // ---- 3. the path from 0 (as ambc_zlib9.hip): per window the exit offset
        // and the matches on the way by pointer doubling (the list is dead: LDS) ----
        const uint32_t nwin = (n + 63) / 64;
        for (uint32_t w = wave; w < nwin; w += NW) {
            const uint32_t p = w * 64 + lane;
            const uint32_t t = p < n && ((S.vis[p >> 5] >> (p & 31)) & 1u) ? seg[p] : 0u;
            uint32_t J = t ? lane + (t & 0xFFFFu) + ((t >> 16) & 0x1FFu) : lane + 1;
            uint32_t M = (t >> 16) & 0x1FFu ? 1u : 0u;
#pragma unroll
            for (int it = 0; it < 6; it++) {
                const int srcl = (int)(min(J, 63u) << 2);
                const uint32_t Jj = (uint32_t)__builtin_amdgcn_ds_bpermute(srcl, (int)J);
                const uint32_t Mj = (uint32_t)__builtin_amdgcn_ds_bpermute(srcl, (int)M);
                M = J < 64 ? M + Mj : M;
                J = J < 64 ? Jj : J;
            }
            S.p.xit[p] = (uint16_t)(J | M << 10);
        }
        for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX / 64; i += TT) S.p.entry[i] = 0xFFFFu;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t cur = 0, mr = 0;
            while (cur < n) {
                S.p.entry[cur >> 6] = (uint16_t)(cur & 63u);
                S.p.rbase[cur >> 6] = (uint16_t)mr;
                const uint32_t x = S.p.xit[cur];
                mr += x >> 10;
                cur = (cur & ~63u) + (x & 1023u);
            }
            S.nmatch = mr;
        }
        __syncthreads();
        BSTAMP(4);
        for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX / 32; i += TT) { S.p.b.mask[i] = 0; S.p.b.cov[i] = 0; }
        for (uint32_t i = threadIdx.x; i < NBLK * 316; i += TT) (&S.p.b.lf[0][0])[i] = 0;
        __syncthreads();
        uint32_t* R = A.z9rec + (uint64_t)k * Z9Rec<CMAX>::STRIDE;
        for (uint32_t w = wave; w < nwin; w += NW) {
            const uint32_t e = S.p.entry[w];
            if (e == 0xFFFFu) continue;
            const uint32_t p = w * 64 + lane;
            const uint32_t t = p < n && ((S.vis[p >> 5] >> (p & 31)) & 1u) ? seg[p] : 0u;
            const uint32_t c = t & 0xFFFFu, L = (t >> 16) & 0x1FFu;
            const uint32_t J1 = lane + max(1u, c + L);
            uint64_t on = 0;
            for (uint32_t q = e; q < 64;) {
                on |= 1ull << q;
                q = readlane(J1, q);
            }
            const bool mt = ((on >> lane) & 1u) && L != 0;
            const uint64_t mm = __ballot(mt);
            if (mt) {
                const uint32_t ms = p + c, d = sd[p];
                atomicOr(&S.p.b.mask[ms >> 5], 1u << (ms & 31));
                R[Z9Rec<CMAX>::MATCH + S.p.rbase[w] + (uint32_t)__popcll(mm & below)] = L | d << 16;
                for (uint32_t b = ms, e2 = ms + L; b < e2;) {
                    const uint32_t wd = b >> 5, hi = min(e2, (wd + 1) * 32);
                    const uint32_t bits = (hi - b == 32 ? ~0u : ((1u << (hi - b)) - 1u)) << (b & 31);
                    atomicOr(&S.p.b.cov[wd], bits);
                    b = hi;
                }
            }
        }
        __syncthreads();
        // ---- 4. the blocks: a block ends with its 16383rd symbol (a literal
        // or a match start: every position no match covers, and every match
        // start), except the final literal at n - 1 (tallied without the flush
        // check).  Wave 0 counts symbol starts 64 words at a time. ----
        if (wave == 0) {
            const uint32_t nwd = (n + 31) / 32;
            uint32_t base = 0, want = Z_BLKSYM, nb = 0, mbase = 0;
            for (uint32_t w0 = 0; w0 < nwd && nb < NBLK - 1; w0 += 64) {
                const uint32_t w = w0 + lane;
                uint32_t sym = 0, mk = 0;
                if (w < nwd) {
                    const uint32_t valid = (w + 1) * 32 <= n ? ~0u : ((1u << (n & 31)) - 1u);
                    mk = S.p.b.mask[w];
                    sym = (~S.p.b.cov[w] | mk) & valid;
                }
                const uint32_t cs = (uint32_t)__popc(sym), cm = (uint32_t)__popc(mk);
                const uint32_t incl = wave_incl_sum(cs), minc = wave_incl_sum(cm);
                while (nb < NBLK - 1) {
                    const uint64_t hit = __ballot(base + incl >= want && base + incl - cs < want);
                    if (!hit) break;
                    const uint32_t hl = (uint32_t)__builtin_ctzll(hit);
                    // the (want - before)-th set bit of that word
                    uint32_t x = readlane(sym, hl), need = want - (base + readlane(incl, hl) - readlane(cs, hl));
                    while (--need) x &= x - 1u;
                    const uint32_t bit = (uint32_t)__builtin_ctz(x);
                    const uint32_t p = (w0 + hl) * 32 + bit;
                    const uint32_t mw = readlane(mk, hl);
                    if ((mw >> bit) & 1u) {
                        const uint32_t rank = mbase + readlane(minc, hl) - readlane(cm, hl) +
                                              (uint32_t)__popc(mw & ((1u << bit) - 1u));
                        const uint32_t L = R[Z9Rec<CMAX>::MATCH + rank] & 0xFFFFu;
                        if (lane == 0) { S.bnd[nb] = p + L; S.btop[nb] = p + 1; }
                    } else {
                        if (p + 1 == n) break;   // the final literal: no flush
                        if (lane == 0) { S.bnd[nb] = p + 1; S.btop[nb] = p + 1; }
                    }
                    nb++;
                    want += Z_BLKSYM;
                }
                base += readlane(incl, 63);
                mbase += readlane(minc, 63);
            }
            if (lane == 0) S.nbnd = nb;
        }
        __syncthreads();
        const uint32_t nbnd = S.nbnd;
        // per-block symbol counts: literals (positions no match covers) by position
        for (uint32_t i = threadIdx.x; i < n; i += TT) {
            if ((S.p.b.cov[i >> 5] >> (i & 31)) & 1u) continue;
            uint32_t b = 0;
            for (uint32_t q = 0; q < nbnd; q++) b += i >= S.bnd[q] ? 1u : 0u;
            atomicAdd(&S.p.b.lf[b][src[i]], 1u);
        }
        // matches by their start: each wave takes 64 mask words at a time, ranks
        // from the popcounts of the words below
        for (uint32_t w0 = wave * 64; w0 < (n + 31) / 32; w0 += NW * 64) {
            const uint32_t w = w0 + lane;
            const uint32_t mk = w < (n + 31) / 32 ? S.p.b.mask[w] : 0u;
            uint32_t pre = 0;
            for (uint32_t q = lane; q < w0; q += 64) pre += (uint32_t)__popc(S.p.b.mask[q]);
            pre = wave_sum_u32(pre);
            const uint32_t cm = (uint32_t)__popc(mk);
            uint32_t rank = pre + wave_incl_sum(cm) - cm;
            uint32_t x = mk;
            while (x) {
                const uint32_t bit = (uint32_t)__builtin_ctz(x);
                x &= x - 1u;
                const uint32_t ms = w * 32 + bit;
                const uint32_t rc = R[Z9Rec<CMAX>::MATCH + rank++];
                const uint32_t L = rc & 0xFFFFu, d = rc >> 16;
                uint32_t b = 0;
                for (uint32_t q = 0; q < nbnd; q++) b += ms >= S.bnd[q] ? 1u : 0u;
                atomicAdd(&S.p.b.lf[b][257 + z_lcode(L)], 1u);
                atomicAdd(&S.p.b.lf[b][286 + z_dcode(d)], 1u);
            }
        }
        for (uint32_t i = threadIdx.x; i < (uint32_t)CMAX / 32; i += TT) R[Z9Rec<CMAX>::MASK + i] = S.p.b.mask[i];
        if (threadIdx.x == 0) {
            R[0] = S.nmatch;
            R[1] = nbnd + 1;
        }
        if (threadIdx.x <= nbnd) {
            // block b = threadIdx.x: [bs, be), matches before it, the stored flag
            const uint32_t b = threadIdx.x;
            const uint32_t bs = b ? S.bnd[b - 1] : 0u, be = b < nbnd ? S.bnd[b] : n;
            const uint32_t top = b < nbnd ? S.btop[b] : n;
            const uint32_t thr = n == 65536u ? Z_SLIDE + 1 : Z_SLIDE;
            uint32_t mb = 0;   // match starts below bs
            for (uint32_t q = 0; q < (bs >> 5); q++) mb += (uint32_t)__popc(S.p.b.mask[q]);
            if (bs & 31) mb += (uint32_t)__popc(S.p.b.mask[bs >> 5] & ((1u << (bs & 31)) - 1u));
            uint32_t* B = R + Z9Rec<CMAX>::BLK + 4 * b;
            B[0] = bs;
            B[1] = be;
            B[2] = mb;
            B[3] = (top >= thr && bs < Z_WSZ) ? Z9B_NOSTORE : 0u;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 158 * (nbnd + 1); i += TT) {
            const uint32_t b = i / 158, o = i % 158;
            R[Z9Rec<CMAX>::FREQ + i] = S.p.b.lf[b][2 * o] | S.p.b.lf[b][2 * o + 1] << 16;
        }
        BSTAMP(5);
        BSTAMP_FLUSH
    }
}

// ---------------------------------------------------------------------------
// k_z9_code_big: trees per block, the exact length, then the bits through a ring
constexpr uint32_t ZR_W = 512;   // ring words (2 KB): a round writes <= 96, a header <= 150

template <int CMAX>
struct Z9BCSmem {
    static constexpr uint32_t NB = Z9Rec<CMAX>::NBLK;
    alignas(16) uint32_t ring[ZR_W];
    uint32_t mstart[CMAX / 32 + 2];
    uint32_t ecl[288], ecd[32];
    uint32_t heapL[LT_N + 1], heapD[DT_N + 1];
    uint16_t lfreq[LT_N + 1], ldad[LT_N + 1];
    uint16_t dfreq[DT_N + 1], ddad[DT_N + 1];
    uint16_t bfreq[BT_N + 1], bdad[BT_N + 1];
    uint16_t blcL[16], blcD[16], blcB[16];
    uint16_t pjd[LT_N + 3], pja[LT_N + 3];
    uint32_t blc32[16], cnt32[20];
    uint32_t misc[16];
    // per block: code lengths and codes of the three trees, the header numbers
    uint8_t llen[NB][LT_N + 1], dlen[NB][DT_N + 1], blen[NB][BT_N + 1];
    uint16_t lcode[NB][288], dcode[NB][32], bcode[NB][20];
    uint32_t kind[NB], lmax[NB], dmax[NB], maxbl[NB];
};

template <int CMAX>
__global__ __launch_bounds__(64) void k_z9_code_big(EncArgs A) {
    constexpr uint32_t RM = ZR_W - 1;
    __shared__ Z9BCSmem<CMAX> S;
    const uint32_t lane = threadIdx.x;
    const uint32_t k = blockIdx.x;
    const uint64_t pos0 = A.coff ? A.coff[k] : (uint64_t)k * A.chunk_size;
    const uint32_t n = A.coff ? (A.clen ? A.clen[k] : A.clen_all) : (uint32_t)min((uint64_t)A.chunk_size, A.n_total - pos0);
    uint32_t T = 0;
    if (n > (uint32_t)CMAX || !z9_gate(A, k, n, T)) return;
    const uint8_t* src = A.in + pos0;
    const uint32_t* R = A.z9rec + (uint64_t)k * Z9Rec<CMAX>::STRIDE;
    const uint32_t* rec = R + Z9Rec<CMAX>::MATCH;
    const uint32_t nblk = uniform_u32(R[1]);
    const uint64_t below = (1ull << lane) - 1ull;
    l32* W = (l32*)S.ring;
    for (uint32_t i = lane; i < (uint32_t)CMAX / 32 + 2; i += 64)
        S.mstart[i] = i < (uint32_t)CMAX / 32 ? R[Z9Rec<CMAX>::MASK + i] : 0u;
    for (uint32_t i = lane; i < ZR_W; i += 64) S.ring[i] = 0;
    wave_sync();

    // ---- pass 1: every block's trees, kind and bits ----
    uint32_t bp = 16;   // after the zlib header
    for (uint32_t b = 0; b < nblk; b++) {
        const uint32_t* B = R + Z9Rec<CMAX>::BLK + 4 * b;
        const uint32_t bs = uniform_u32(B[0]), be = uniform_u32(B[1]), fl = uniform_u32(B[3]);
        const Z9Tree LT{(l16*)S.lfreq, (l16*)S.ldad, (l8*)S.llen[b], (l16*)S.lcode[b], (l32*)S.heapL, (l16*)S.blcL};
        const Z9Tree DT{(l16*)S.dfreq, (l16*)S.ddad, (l8*)S.dlen[b], (l16*)S.dcode[b], (l32*)S.heapD, (l16*)S.blcD};
        const Z9Tree BT{(l16*)S.bfreq, (l16*)S.bdad, (l8*)S.blen[b], (l16*)S.bcode[b], (l32*)S.heapD, (l16*)S.blcB};
        const uint16_t* F = reinterpret_cast<const uint16_t*>(R + Z9Rec<CMAX>::FREQ + 158 * b);
        const uint32_t* MG = R + Z9Rec<CMAX>::MERGE + 316 * b;
        if (lane < 20) S.cnt32[lane] = 0;
        for (uint32_t i = lane; i < 286; i += 64) S.lfreq[i] = (uint16_t)(F[i] + (i == 256 ? 1u : 0u));
        if (lane < 30) S.dfreq[lane] = F[286 + lane];
        wave_sync();
        l16* PJD = (l16*)S.pjd;
        l16* PJA = (l16*)S.pja;
        l32* BLC = (l32*)S.blc32;
        l32* MISC = (l32*)(S.misc + 12);
        uint32_t optL = 0, statL = 0, optD = 0, statD = 0, optB = 0, statB = 0;
        const int lmax = z9_build_w<5, true>(LT, PJD, PJA, BLC, MISC, 286, 15, 0, optL, statL, lane, MG);
        const int dmax = z9_build_w<1, true>(DT, PJD, PJA, BLC, MISC, 30, 15, 1, optD, statD, lane, MG + 285);
        VHeap<5> LL;
        VHeap<1> DL;
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const uint32_t x = 64u * j + lane;
            LL.h[j] = (int)x <= lmax ? (uint32_t)S.llen[b][x] : 0u;
        }
        DL.h[0] = (int)lane <= dmax ? (uint32_t)S.dlen[b][lane] : 0u;
        (void)z9_rle_par(LL, lmax, false, (l32*)S.cnt32, 0u, S.ring, 0u, lane);
        (void)z9_rle_par(DL, dmax, false, (l32*)S.cnt32, 0u, S.ring, 0u, lane);
        wave_sync();
        if (lane < 19) S.bfreq[lane] = (uint16_t)S.cnt32[lane];
        wave_sync();
        (void)z9_build_w<1, false>(BT, PJD, PJA, BLC, MISC, 19, 7, 2, optB, statB, lane);
        int maxbl;
        for (maxbl = 18; maxbl >= 3; maxbl--) if (S.blen[b][z_blord[maxbl]] != 0) break;
        const uint32_t opt = optL + optD + optB + 3u * (uint32_t)(maxbl + 1) + 5 + 5 + 4;
        const uint32_t stl = statL + statD;
        uint32_t opt_lenb = (opt + 3 + 7) >> 3;
        const uint32_t static_lenb = (stl + 3 + 7) >> 3;
        if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
        const uint32_t kind = (be - bs + 4 <= opt_lenb && !(fl & Z9B_NOSTORE)) ? 0u : (static_lenb == opt_lenb ? 1u : 2u);
        if (lane == 0) {
            S.kind[b] = kind;
            S.lmax[b] = (uint32_t)lmax;
            S.dmax[b] = (uint32_t)dmax;
            S.maxbl[b] = (uint32_t)maxbl;
        }
        if (kind == 0) bp = ((bp + 3 + 7) & ~7u) + 32 + 8 * (be - bs);
        else bp += 3 + (kind == 2 ? opt : stl);
        wave_sync();
    }
    const uint32_t total = (bp + 7) / 8 + 4;
    if (total + 18 >= T) return;
    if (A.flags & ENC_EVAL) {   // the multi-size walk's decision: pass 2 writes nothing it reads
        if (lane == 0) {
            A.ids[k] = 5;
            A.plen[k] = total;
            A.sizes[k] = 18ull + total;
        }
        return;
    }

    // ---- pass 2: the bits ----
    uint32_t* out32 = reinterpret_cast<uint32_t*>(A.slots + (uint64_t)k * A.slot_stride);
    uint32_t flushed = 0;   // words [0, flushed) are in the slot
    auto flush = [&](uint32_t upto) {
        wave_sync();
        for (uint32_t w = flushed + lane; w < upto; w += 64) {
            out32[w] = S.ring[w & RM];
            S.ring[w & RM] = 0;
        }
        wave_sync();
        flushed = upto;
    };
    if (lane == 0) z_put(W, 0, 0xDA78u, 16, RM);   // 78 DA
    bp = 16;
    for (uint32_t b = 0; b < nblk; b++) {
        const uint32_t* B = R + Z9Rec<CMAX>::BLK + 4 * b;
        const uint32_t bs = uniform_u32(B[0]), be = uniform_u32(B[1]), rank0 = uniform_u32(B[2]);
        const uint32_t last = b + 1 == nblk ? 1u : 0u;
        const uint32_t kind = uniform_u32(S.kind[b]);
        wave_sync();
        if (kind == 0) {
            // stored: 3 bits, byte alignment, LEN / NLEN, the bytes
            const uint32_t len = be - bs;
            if (lane == 0) z_put(W, bp, last, 3, RM);
            bp = (bp + 3 + 7) & ~7u;
            if (lane == 0) z_put(W, bp, len | (~len & 0xFFFFu) << 16, 32, RM);
            bp += 32;
            for (uint32_t r0 = 0; r0 < len; r0 += 64) {
                wave_sync();
                const uint32_t i = r0 + lane;
                if (i < len) z_put_atomic(S.ring, bp + 8 * i, src[bs + i], 8, RM);
                flush((bp + 8 * min(len, r0 + 64)) >> 5);
            }
            bp += 8 * len;
            flush(bp >> 5);
            continue;
        }
        if (kind == 1) {
            for (uint32_t i = lane; i < 288; i += 64) {
                uint32_t c, l;
                if (i < 144) { c = 0x30 + i; l = 8; }
                else if (i < 256) { c = 0x190 + (i - 144); l = 9; }
                else if (i < 280) { c = i - 256; l = 7; }
                else { c = 0xC0 + (i - 280); l = 8; }
                S.ecl[i] = (__builtin_bitreverse32(c) >> (32 - l)) | l << 16;
            }
            if (lane < 30) S.ecd[lane] = (__builtin_bitreverse32(lane) >> 27) | 5u << 16;
        } else {
            for (uint32_t i = lane; i < 286; i += 64) S.ecl[i] = S.lcode[b][i] | (uint32_t)S.llen[b][i] << 16;
            if (lane < 30) S.ecd[lane] = S.dcode[b][lane] | (uint32_t)S.dlen[b][lane] << 16;
        }
        wave_sync();
        {
            // the block header on the scalar unit
            SBits sb{0ull, bp & 31u, bp >> 5};
            sb.acc = sb.n ? (uint64_t)(S.ring[sb.w & RM] & ((1u << sb.n) - 1u)) : 0ull;
            sb_put(sb, W, kind << 1 | last, 3, lane, RM);
            if (kind == 2) {
                const int lmax = (int)uniform_u32(S.lmax[b]), dmax = (int)uniform_u32(S.dmax[b]);
                const int maxbl = (int)uniform_u32(S.maxbl[b]);
                sb_put(sb, W, (uint32_t)lmax + 1 - 257, 5, lane, RM);
                sb_put(sb, W, (uint32_t)dmax, 5, lane, RM);
                sb_put(sb, W, (uint32_t)maxbl + 1 - 4, 4, lane, RM);
                for (int r = 0; r <= maxbl; r++) sb_put(sb, W, S.blen[b][z_blord[r]], 3, lane, RM);
                const uint32_t bcl = lane < 19 ? (uint32_t)S.bcode[b][lane] | (uint32_t)S.blen[b][lane] << 16 : 0u;
                if (sb.n && lane == 0) W[sb.w & RM] = (uint32_t)sb.acc;
                wave_sync();
                VHeap<5> LL;
                VHeap<1> DL;
#pragma unroll
                for (int j = 0; j < 5; j++) {
                    const uint32_t x = 64u * j + lane;
                    LL.h[j] = (int)x <= lmax ? (uint32_t)S.llen[b][x] : 0u;
                }
                DL.h[0] = (int)lane <= dmax ? (uint32_t)S.dlen[b][lane] : 0u;
                uint32_t p = sb.w * 32 + sb.n;
                p += z9_rle_par(LL, lmax, true, (l32*)S.cnt32, bcl, S.ring, p, lane, RM);
                wave_sync();
                p += z9_rle_par(DL, dmax, true, (l32*)S.cnt32, bcl, S.ring, p, lane, RM);
                bp = p;
            } else {
                if (sb.n && lane == 0) W[sb.w & RM] = (uint32_t)sb.acc;
                bp = sb.w * 32 + sb.n;
            }
        }
        flush(bp >> 5);
        // the block's symbols over [bs, be), position-major, 64 positions a round
        {
            uint32_t rank = rank0;
            int carry = (int)bs;
            auto fetch = [&](uint32_t q0, uint32_t rk, uint64_t& bmo, uint32_t& xo, uint32_t& co) {
                const uint32_t pos = q0 + lane;
                const bool in = pos >= bs && pos < be;
                const bool m = in && ((S.mstart[pos >> 5] >> (pos & 31)) & 1u);
                bmo = __ballot(m);
                xo = m ? rec[rk + (uint32_t)__popcll(bmo & below)] : 0u;
                co = in ? (uint32_t)src[pos] : 0u;
            };
            uint64_t bmn = 0;
            uint32_t xn = 0, cn = 0;
            fetch(bs & ~63u, rank, bmn, xn, cn);
#pragma unroll 1
            for (uint32_t p0 = bs & ~63u; p0 < be; p0 += 64) {
                const uint64_t bm = bmn;
                const uint32_t x = xn, cb = cn;
                const uint32_t rank2 = rank + (uint32_t)__popcll(bm);
                if (p0 + 64 < be) fetch(p0 + 64, rank2, bmn, xn, cn);
                const uint32_t pos = p0 + lane;
                const bool in = pos >= bs && pos < be;
                const bool ms = (bm >> lane) & 1u;
                const uint32_t L = ms ? x & 0xFFFFu : 0u, d = x >> 16;
                const int e = ms ? (int)(pos + L) : 0;
                const int E = max(carry, wave_incl_max_i32(e));
                carry = max(carry, wave_max_i32(e));
                rank = rank2;
                const bool lit = in && !ms && E <= (int)pos;
                const uint32_t c = lit ? cb : 0u;
                const uint32_t lc = ms ? z_lcode(L) : 0u, dc = ms ? z_dcode(d) : 0u;
                uint32_t e1 = 0, e2 = 0, v1 = 0, v2 = 0;
                if (lit) {
                    e1 = S.ecl[c] >> 16;
                    v1 = S.ecl[c] & 0xFFFFu;
                } else if (ms) {
                    const uint32_t a = S.ecl[257 + lc], bb = S.ecd[dc];
                    const uint32_t la = a >> 16, lb = bb >> 16;
                    const uint32_t xl = z_xlb(lc), xd = z_xdb(dc);
                    e1 = la + xl;
                    v1 = (a & 0xFFFFu) | ((L - 3) & ((1u << xl) - 1u)) << la;
                    e2 = lb + xd;
                    v2 = (bb & 0xFFFFu) | ((d - 1) & ((1u << xd) - 1u)) << lb;
                }
                const uint32_t cost = e1 + e2;
                const uint32_t incl = wave_incl_sum(cost);
                const uint32_t q = bp + incl - cost;
                z_put_atomic(S.ring, q, v1, e1, RM);
                z_put_atomic(S.ring, q + e1, v2, e2, RM);
                bp += readlane(incl, 63);
                flush(bp >> 5);
            }
        }
        wave_sync();
        if (lane == 0) z_put(W, bp, S.ecl[256] & 0xFFFFu, S.ecl[256] >> 16, RM);
        bp += S.ecl[256] >> 16;
    }
    // ---- Adler-32 of the chunk, big-endian after the byte boundary ----
    const uint32_t adler = adler32_wave(src, n, lane);
    bp = (bp + 7) & ~7u;
    wave_sync();
    if (lane == 0)
        for (int i = 0; i < 4; i++) z_put(W, bp + 8 * i, (adler >> (24 - 8 * i)) & 0xFFu, 8, RM);
    bp += 32;
    flush((bp + 31) >> 5);
    if (lane == 0) {
        A.ids[k] = 5;
        A.plen[k] = total;
        A.sizes[k] = 18ull + total;
    }
}

template <int CMAX>
hipError_t launch_z9b_t(const EncArgs& a, hipStream_t s) {
    const uint32_t g = min(a.n_chunks, ZB_GRID);
    constexpr uint32_t NB = Z9Rec<CMAX>::NBLK;
    hipLaunchKernelGGL(k_z9_parse_big<CMAX>, dim3(g), dim3(64 * ZB_NW), 0, s, a);
    hipLaunchKernelGGL(k_z9_heap<CMAX>, dim3((a.n_chunks * NB + ZH_L - 1) / ZH_L), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_z9_code_big<CMAX>, dim3(a.n_chunks), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace

size_t z9_scratch_bytes(uint32_t cmax, uint32_t n_chunks) {
    const size_t g = std::min<size_t>(n_chunks, ZB_GRID);
    switch (cmax) {
        case 16384: return g * Z9Big<16384>::BYTES;
        case 32768: return g * Z9Big<32768>::BYTES;
        case 65536: return g * Z9Big<65536>::BYTES;
        default: return 0;
    }
}

size_t z9_rec_words_big(uint32_t cmax) {
    switch (cmax) {
        case 16384: return Z9Rec<16384>::STRIDE;
        case 32768: return Z9Rec<32768>::STRIDE;
        case 65536: return Z9Rec<65536>::STRIDE;
        default: return 0;
    }
}

hipError_t launch_zlib9_big(const EncArgs& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    if (!a.z9scr) return hipErrorInvalidValue;
    switch (z9_cmax(a.chunk_size)) {
        case 16384: return launch_z9b_t<16384>(a, s);
        case 32768: return launch_z9b_t<32768>(a, s);
        case 65536: return launch_z9b_t<65536>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace ambc
