// ambc_walk.hip -- the header walk of _adaptive_decompress on the device.
//
// The reference decodes a body by walking its chunk headers from offset 0
// (adaptive_compressor.py:399-445): an 18-byte header (marker ff ff 00 00, type,
// k, used, orig, comp_len) then comp_len payload bytes, the next header right
// after; the walk stops at a type-0 header, at a payload running past the body,
// when fewer than 18 bytes remain, or once the output reaches orig_size, and
// raises on a header without the marker.  Each position depends on the lengths
// before it -- a host walk is a chain of cache misses, one per package -- but
// the chain is a function of the body, so the device finds it without walking:
//   1. every byte position holding the marker is a candidate header, listed in
//      order (per-tile counts, a scan, a write);
//   2. each candidate links to the candidate at its successor p + 18 + comp_len
//      (binary search), or to a sink with the reason: the walk stops at it
//      (type 0, overrun), ends after it (< 18 bytes left), leaves the piece, or
//      its successor holds no marker (a mismatch if the walk gets there);
//   3. the chain from the entry candidate is marked block by block (pointer
//      doubling in LDS within blocks of 4096 candidates, one serial step per
//      block between them) -- marker bytes inside payloads are candidates too,
//      but nothing on the chain links to them;
//   4. the marked candidates, compacted in order, are the packages: each one's
//      decode job (ambc_host.cpp make_job restated), scans of the output and
//      scratch lengths, the out >= orig_size stop, per-kernel job lists.
// The body is walked piece by piece as its upload arrives (WalkState carries the
// chain's entry position and the output offset from one piece to the next), so
// the decode of a piece starts while later pieces are still on the way.  Every
// kernel is a grid-stride loop over counts the previous kernels left in device
// memory: a piece's walk is one stream of launches with no host round trip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/ambc.h"
#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {
namespace {

constexpr uint32_t WT_TILE = 65536;   // bytes of candidate positions per workgroup
constexpr uint32_t STAGE_DEC_D = 8192;   // must match ambc_decode.hip STAGE
// node flags: the walk stops at this header (no package); ends after it; leaves
// the piece after it; its successor is no marker
constexpr uint8_t F_STOP = 1, F_END = 2, F_EXIT = 4, F_BAD = 8;

__device__ __forceinline__ uint32_t rd32u(const uint8_t* p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

__device__ __forceinline__ uint32_t gtid() { return blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint32_t gsize() { return gridDim.x * blockDim.x; }

// candidate bits of the 16 positions at the 16-aligned base (w: the 16 bytes
// there and the next 4): the marker at base + t, for the positions in [a, e)
__device__ __forceinline__ uint32_t tile_bits(const uint32_t w[5], uint64_t base, uint64_t a, uint64_t e) {
    if (base >= e) return 0;
    uint32_t m = 0;
#pragma unroll
    for (int t = 0; t < 16; t++) {
        const uint32_t x = __builtin_amdgcn_alignbyte(w[(t >> 2) + 1], w[t >> 2], t & 3);
        m |= (x == 0x0000FFFFu ? 1u : 0u) << t;
    }
    const uint32_t lo = a > base ? (uint32_t)(a - base) : 0u;
    const uint32_t hi = e - base >= 16 ? 16u : (uint32_t)(e - base);
    return m & ((1u << hi) - 1u) & ~((1u << lo) - 1u);
}

// one 16-byte load per lane (coalesced), the 4 bytes after it from the next lane
// (the last lane loads them); every lane of the wave must call this
__device__ __forceinline__ void load_group(const uint8_t* body, uint64_t base, uint64_t e, uint32_t w[5]) {
    uint4 v = make_uint4(0, 0, 0, 0);
    // (the group after the last one in [a, e) too: its first bytes end the markers at e - 3 .. e - 1;
    // base + 16 <= e + 31 < blen + 64, the buffer's slack)
    if (base < e + 16) v = *reinterpret_cast<const uint4*>(body + base);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    uint32_t nx = (uint32_t)__shfl_down((int)v.x, 1);
    if ((threadIdx.x & 63) == 63 && base < e) nx = *reinterpret_cast<const uint32_t*>(body + base + 16);
    w[4] = nx;
}

// exclusive scan over a 256-thread workgroup (LDS, off the hot loops)
template <typename T>
__device__ T block_excl(T x, T* s, T& total) {
    const uint32_t t = threadIdx.x;
    s[t] = x;
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const T y = t >= o ? s[t - o] : (T)0;
        __syncthreads();
        s[t] += y;
        __syncthreads();
    }
    total = s[255];
    const T incl = s[t];
    __syncthreads();
    return incl - x;
}

// exclusive scan of v[0, n) in place by one 256-thread workgroup
template <typename T>
__device__ void serial_block_scan(T* v, uint32_t n, T* s, T* total) {
    T carry = 0;
    for (uint32_t b = 0; b < n; b += 256) {
        const uint32_t i = b + threadIdx.x;
        const T x = i < n ? v[i] : (T)0;
        T tot;
        const T ex = block_excl<T>(x, s, tot);
        if (i < n) v[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

// ---- 1. candidates -------------------------------------------------------

__global__ __launch_bounds__(256) void k_walk_count(WalkArgs A) {
    const uint64_t t0 = (A.a & ~15ull) + (uint64_t)blockIdx.x * WT_TILE;
    uint32_t c = 0;
    for (uint32_t g = threadIdx.x; g < WT_TILE / 16; g += 256) {
        const uint64_t base = t0 + 16ull * g;
        uint32_t w[5];
        load_group(A.body, base, A.e, w);
        c += (uint32_t)__popc(tile_bits(w, base, A.a, A.e));
    }
    __shared__ uint32_t red[4];
    c = wave_sum_u32(c);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) A.tcnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// tile offsets; the per-piece state reset
__global__ __launch_bounds__(256) void k_walk_tscan(WalkArgs A) {
    __shared__ uint32_t s[256];
    WalkState* st = A.st;
    serial_block_scan<uint32_t>(A.tcnt, A.ntiles, s, &st->nc);
    const uint32_t t = threadIdx.x;
    if (t < 16) { st->kcount[t] = 0; st->kfill[t] = 0; }
    if (t == 0) {
        st->nchain = 0; st->nj = 0; st->stop = ~0u; st->root = ~0u;
        st->scr = 0; st->bneed = 0; st->tot_o = 0; st->tot_s = 0;
    }
}

__global__ __launch_bounds__(256) void k_walk_list(WalkArgs A) {
    const uint64_t t0 = (A.a & ~15ull) + (uint64_t)blockIdx.x * WT_TILE;
    uint32_t at = A.tcnt[blockIdx.x];
    __shared__ uint32_t wsum[4];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t g0 = 0; g0 < WT_TILE / 16; g0 += 256) {
        const uint64_t base = t0 + 16ull * (g0 + threadIdx.x);
        uint32_t w[5];
        load_group(A.body, base, A.e, w);
        uint32_t m = tile_bits(w, base, A.a, A.e);
        const uint32_t c = (uint32_t)__popc(m);
        const uint32_t incl = wave_incl_sum(c);
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            before += (uint32_t)q < wave ? wsum[q] : 0u;
            tot += wsum[q];
        }
        uint32_t o = at + before + incl - c;
        while (m) {
            const uint32_t b = (uint32_t)__builtin_ctz(m);
            m &= m - 1u;
            A.cand[o++] = base + b;
        }
        at += tot;
        __syncthreads();
    }
}

// ---- 2. links ------------------------------------------------------------

__global__ __launch_bounds__(256) void k_walk_link(WalkArgs A) {
    WalkState* st = A.st;
    const uint32_t nc = st->nc;
    const uint64_t entry = st->entry;
    for (uint32_t i = gtid(); i <= nc; i += gsize()) {
        if (i == nc) { A.ja[nc] = nc; A.jb[nc] = nc; continue; }   // the sink
        const uint64_t p = A.cand[i];
        const uint8_t* h = A.body + p;
        const uint32_t t = h[4];
        const uint64_t q = p + 18 + rd32u(h + 14);
        uint32_t link = nc;
        uint8_t f = 0;
        if (t == 0 || q > A.blen) {
            f = F_STOP;
        } else if (q + 18 > A.blen) {
            f = F_END;
        } else if (q >= A.e) {
            f = F_EXIT;
        } else {
            uint32_t lo = i + 1, hi = nc;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (A.cand[mid] < q) lo = mid + 1;
                else hi = mid;
            }
            if (lo < nc && A.cand[lo] == q) link = lo;
            else f = F_BAD;
        }
        A.ja[i] = link;
        A.flg[i] = f;
        if (p == entry) st->root = i;
    }
}

// ---- 3. the chain --------------------------------------------------------
// Candidates in blocks of BN (links only go forward).  bexit: per block, by
// pointer doubling in LDS, where the path from each node leaves the block.
// bentry: one thread follows the chain from the entry block to block -- one
// step per block the chain visits.  bmark: per visited block, the nodes on the
// path from its entry node (pointer doubling in LDS), and their count.

constexpr uint32_t BN = 4096;           // candidates per block (1024 threads x 4)
constexpr uint32_t BT = 1024;
constexpr uint16_t LNONE = 0xFFFF;

__global__ __launch_bounds__(1024) void k_walk_bexit(WalkArgs A) {
    const uint32_t nc = A.st->nc, nb = (nc + BN - 1) / BN;
    __shared__ uint16_t v[BN];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t base = b * BN, n = min(BN, nc - base);
        for (uint32_t l = threadIdx.x; l < n; l += BT) {
            const uint32_t j = A.ja[base + l];
            v[l] = (uint16_t)(j < base + n ? j - base : l);   // the last node in the block points to itself
        }
        __syncthreads();
        for (uint32_t o = 1; o < n; o <<= 1) {
            uint16_t t[BN / BT];
#pragma unroll
            for (uint32_t q = 0; q < BN / BT; q++) {
                const uint32_t l = threadIdx.x + BT * q;
                t[q] = l < n ? v[v[l]] : (uint16_t)0;
            }
            __syncthreads();
#pragma unroll
            for (uint32_t q = 0; q < BN / BT; q++) {
                const uint32_t l = threadIdx.x + BT * q;
                if (l < n) v[l] = t[q];
            }
            __syncthreads();
        }
        for (uint32_t l = threadIdx.x; l < n; l += BT) A.jb[base + l] = A.ja[base + v[l]];
        if (threadIdx.x == 0) A.bc[b] = ~0u;             // (bentry: the block's entry node)
        __syncthreads();
    }
}

__global__ void k_walk_bentry(WalkArgs A) {
    WalkState* st = A.st;
    if (threadIdx.x) return;
    if (st->entry != WALK_ENDED && st->entry < A.e && st->root == ~0u) {
        st->err = 1;                                     // the entry lies in the piece but holds no marker
        st->entry = WALK_ENDED;
        return;
    }
    const uint32_t nc = st->nc;
    for (uint32_t x = st->root; x < nc; x = A.jb[x]) A.bc[x / BN] = x;
}

__global__ __launch_bounds__(1024) void k_walk_bmark(WalkArgs A) {
    const uint32_t nc = A.st->nc, nb = (nc + BN - 1) / BN;
    __shared__ uint16_t v[BN];
    __shared__ uint8_t m[BN];
    __shared__ uint32_t red[BT / 64];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t base = b * BN, n = min(BN, nc - base);
        if (threadIdx.x == 0) red[0] = A.bc[b];
        __syncthreads();
        const uint32_t e0 = red[0];
        __syncthreads();
        if (e0 == ~0u) {                                 // (uniform over the workgroup)
            for (uint32_t l = threadIdx.x; l < n; l += BT) A.mark[base + l] = 0;
            if (threadIdx.x == 0) A.bc[b] = 0;
            continue;
        }
        for (uint32_t l = threadIdx.x; l < n; l += BT) {
            const uint32_t j = A.ja[base + l];
            v[l] = j < base + n ? (uint16_t)(j - base) : LNONE;
            m[l] = base + l == e0 ? 1 : 0;
        }
        __syncthreads();
        // round k: the 2^k-th successors of the marked nodes, then the links doubled
        for (uint32_t o = 1; o < 2 * n; o <<= 1) {
#pragma unroll
            for (uint32_t q = 0; q < BN / BT; q++) {
                const uint32_t l = threadIdx.x + BT * q;
                if (l < n && m[l] && v[l] != LNONE) m[v[l]] = 1;
            }
            __syncthreads();
            uint16_t t[BN / BT];
#pragma unroll
            for (uint32_t q = 0; q < BN / BT; q++) {
                const uint32_t l = threadIdx.x + BT * q;
                t[q] = l < n && v[l] != LNONE ? v[v[l]] : LNONE;
            }
            __syncthreads();
#pragma unroll
            for (uint32_t q = 0; q < BN / BT; q++) {
                const uint32_t l = threadIdx.x + BT * q;
                if (l < n) v[l] = t[q];
            }
            __syncthreads();
        }
        uint32_t c = 0;
        for (uint32_t l = threadIdx.x; l < n; l += BT) {
            A.mark[base + l] = m[l];
            c += m[l];
        }
        c = wave_sum_u32(c);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            for (uint32_t w = 0; w < BT / 64; w++) tot += red[w];
            A.bc[b] = tot;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_walk_bscan(WalkArgs A) {
    __shared__ uint32_t s[256];
    serial_block_scan<uint32_t>(A.bc, (A.st->nc + BN - 1) / BN, s, &A.st->nchain);
}

// the marked candidates in order: 16 consecutive nodes per thread
__global__ __launch_bounds__(256) void k_walk_chain(WalkArgs A) {
    const uint32_t nc = A.st->nc, nb = (nc + BN - 1) / BN;
    __shared__ uint32_t s[256];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t i0 = b * BN + 16 * threadIdx.x;
        uint32_t bits = 0;
#pragma unroll
        for (int q = 0; q < 16; q++) bits |= (i0 + q < nc && A.mark[i0 + q] ? 1u : 0u) << q;
        uint32_t tot;
        uint32_t at = A.bc[b] + block_excl<uint32_t>((uint32_t)__popc(bits), s, tot);
        while (bits) {
            const uint32_t q = (uint32_t)__builtin_ctz(bits);
            bits &= bits - 1u;
            A.chain[at++] = i0 + q;
        }
    }
}

// ---- 4. jobs -------------------------------------------------------------

__device__ __forceinline__ bool reg_id(const WalkArgs& A, uint32_t t) { return (A.reg[t >> 6] >> (t & 63)) & 1ull; }

// upper bound of an LZ4 frame's decoded content (the host's lz4_content_bound)
__device__ uint64_t lz4_bound_d(const uint8_t* p, uint32_t plen) {
    if (plen < 7 || rd32u(p) != 0x184D2204u) return 0;
    const uint32_t flg = p[4], bd = p[5];
    const uint32_t bsid = (bd >> 4) & 7;
    if (bsid < 4) return 0;
    const uint64_t bmax = 1ull << (8 + 2 * bsid);
    uint64_t hp = 6, cs = 0;
    const bool has_cs = (flg >> 3) & 1;
    if (has_cs) {
        if (hp + 8 > plen) return 0;
        for (int b = 0; b < 8; b++) cs |= (uint64_t)p[hp + b] << (8 * b);
        hp += 8;
    }
    if (flg & 1) hp += 4;
    hp += 1;
    uint64_t bound = 0;
    while (hp + 4 <= plen) {
        const uint32_t bs = rd32u(p + hp);
        hp += 4;
        if (bs == 0) break;
        const uint32_t sz = bs & 0x7FFFFFFFu;
        bound += (bs & 0x80000000u) ? (uint64_t)sz : min(bmax, 255ull * sz + 16);
        hp += (uint64_t)sz + (((flg >> 4) & 1) ? 4 : 0);
    }
    return has_cs ? min(cs, bound) : bound;
}

// chain node r's decode job (ambc_host.cpp make_job / expect_len), its output
// bytes and scratch reservation; a stop node gets an empty placeholder
__device__ __forceinline__ void walk_job(const WalkArgs& A, uint32_t r, uint64_t& expect, uint64_t& sneed) {
    {
        const uint32_t i = A.chain[r];
        const uint64_t hp = A.cand[i];
        const uint8_t* h = A.body + hp;
        const uint32_t t = h[4];
        const uint32_t orig = rd32u(h + 10), clen = rd32u(h + 14);
        const bool stop = A.flg[i] & F_STOP;
        DecJob j{};
        uint32_t kind = DEC_KIND_HEAVY;
        sneed = 0;
        expect = 0;
        j.body_off = hp + 18;
        j.clen = clen;
        j.orig = orig;
        j.scratch_off = ~0ull;
        j.scratch_cap = 0;
        if (stop) {
            j.type = DEC_SKIP;
            kind = DEC_KIND_LIGHT;
        } else if (!reg_id(A, t)) {
            j.type = DEC_VERBATIM;
            kind = DEC_KIND_LIGHT;
        } else if (t == 5 && clen && orig <= AMBC_MAX_CHUNK) {
            j.type = 5;
            kind = orig <= 4096 ? DEC_KIND_INFLATE_4K : orig <= 8192 ? DEC_KIND_INFLATE_8K
                 : orig <= 16384 ? DEC_KIND_INFLATE_16K : orig <= 32768 ? DEC_KIND_INFLATE_32K : DEC_KIND_INFLATE_G;
            if (kind == DEC_KIND_INFLATE_G) {
                j.scratch_cap = orig;
                sneed = (4ull * orig + 15) & ~15ull;
            }
        } else if (t == 5 || !device_decodes(t)) {
            j.type = DEC_SKIP;
            kind = DEC_KIND_LIGHT;
        } else {
            if (t == 255 || t == 1 || t == 4) kind = DEC_KIND_LIGHT;
            if (t == 3) kind = huff_kind(orig, clen);
            j.type = t;
            if (t == 9 && clen) {
                const uint8_t* pl = h + 18;
                const uint64_t cb = lz4_bound_d(pl, clen);
                if (clen >= 7 && !((pl[4] >> 2) & 1) && cb < 0x80000000ull) {
                    if (clen <= 0x7FFF && cb <= 16384) {
                        kind = cb <= 4096 ? DEC_KIND_LZ4_4K : cb <= 8192 ? DEC_KIND_LZ4_8K : DEC_KIND_LZ4_16K;
                    } else {
                        kind = DEC_KIND_LZ4_G;
                        j.scratch_cap = cb;
                        sneed = (4 * cb + 15) & ~15ull;
                    }
                } else if (cb > STAGE_DEC_D) {
                    j.scratch_cap = cb;
                    sneed = (cb + 15) & ~15ull;
                }
            }
            if (t == 2 && clen && clen <= 0x7FFF && (uint64_t)orig + 256 <= 16640) {
                kind = orig + 256 <= 4352 ? DEC_KIND_DICT_4K : orig + 256 <= 8448 ? DEC_KIND_DICT_8K : DEC_KIND_DICT_16K;
            } else if (t == 2 && clen && (uint64_t)orig + 256 > STAGE_DEC_D) {
                j.scratch_cap = (uint64_t)orig + 256;
                sneed = (j.scratch_cap + 15) & ~15ull;
            }
        }
        if (!stop) {
            if (!reg_id(A, t)) expect = clen;
            else if (t == 255) expect = orig;
            else if (t == 4) expect = clen ? min(clen, orig) : 0u;
            else expect = clen ? orig : 0u;
        }
        j.expect = (uint32_t)expect;
        A.jobs[r] = j;
        A.kind[r] = (uint8_t)kind;
        A.olen[r] = expect;
        A.slen[r] = sneed;
    }
}

// the jobs, and per 1024 chain nodes the sums of their output / scratch bytes
__global__ __launch_bounds__(256) void k_walk_jobs(WalkArgs A) {
    const uint32_t n = A.st->nchain, nb = (n + 1023) / 1024;
    __shared__ uint64_t so[256], ss[256];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        uint64_t o = 0, s = 0;
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t r = b * 1024 + q * 256 + threadIdx.x;
            if (r < n) {
                uint64_t ex, sn;
                walk_job(A, r, ex, sn);
                o += ex;
                s += sn;
            }
        }
        uint64_t to, ts;
        (void)block_excl<uint64_t>(o, so, to);
        (void)block_excl<uint64_t>(s, ss, ts);
        if (threadIdx.x == 0) { A.bo[b] = to; A.bs[b] = ts; }
    }
}

__global__ __launch_bounds__(256) void k_walk_bscan64(WalkArgs A) {
    __shared__ uint64_t s[256];
    const uint32_t nb = (A.st->nchain + 1023) / 1024;
    serial_block_scan<uint64_t>(A.bo, nb, s, &A.st->tot_o);
    serial_block_scan<uint64_t>(A.bs, nb, s, &A.st->tot_s);
}

// offsets (output: after all earlier jobs; scratch: within the piece) and the stops
__global__ __launch_bounds__(256) void k_walk_fill(WalkArgs A) {
    WalkState* st = A.st;
    const uint32_t n = st->nchain, nb = (n + 1023) / 1024;
    const uint64_t out0 = st->out;
    __shared__ uint64_t so[256], ss[256];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t r0 = b * 1024 + 4 * threadIdx.x;
        uint64_t o = 0, s = 0;
        for (uint32_t q = 0; q < 4; q++)
            if (r0 + q < n) { o += A.olen[r0 + q]; s += A.slen[r0 + q]; }
        uint64_t to, ts;
        uint64_t po = block_excl<uint64_t>(o, so, to) + A.bo[b] + out0;
        uint64_t ps = block_excl<uint64_t>(s, ss, ts) + A.bs[b];
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t r = r0 + q;
            if (r >= n) break;
            const uint64_t ol = A.olen[r], sl = A.slen[r];
            A.jobs[r].out_off = po;
            if (sl) A.jobs[r].scratch_off = ps;
            if (A.flg[A.chain[r]] & F_STOP) atomicMin(&st->stop, r);          // the walk stops before it
            else if (po + ol >= A.orig_size) atomicMin(&st->stop, r + 1);      // the output is complete after it
            po += ol;
            ps += sl;
        }
    }
}

// the piece's outcome: jobs to decode, where the chain goes on, output so far
__global__ void k_walk_fin(WalkArgs A) {
    WalkState* st = A.st;
    const uint32_t nchain = st->nchain;
    const uint32_t nj = min(st->stop, nchain);
    st->nj = nj;
    if (st->stop != ~0u) {
        st->entry = WALK_ENDED;
    } else if (nchain) {
        const uint32_t last = A.chain[nchain - 1];
        const uint8_t f = A.flg[last];
        if (f & F_BAD) { st->err = 1; st->entry = WALK_ENDED; }
        else if (f & F_EXIT) st->entry = A.cand[last] + 18 + rd32u(A.body + A.cand[last] + 14);
        else st->entry = WALK_ENDED;                     // F_END
    }
    if (A.last) st->entry = WALK_ENDED;
    const uint64_t piece_out = nj < nchain ? A.jobs[nj].out_off - st->out : st->tot_o;
    st->out += piece_out;
    st->scr = st->tot_s;
    st->bneed = nj ? A.jobs[nj - 1].body_off + A.jobs[nj - 1].clen : 0;
}

__global__ __launch_bounds__(256) void k_walk_kcount(WalkArgs A) {
    __shared__ uint32_t hist[16];
    const uint32_t nj = A.st->nj;
    if (threadIdx.x < 16) hist[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t r = gtid(); r < nj; r += gsize()) atomicAdd(&hist[A.kind[r]], 1u);
    __syncthreads();
    if (threadIdx.x < DEC_KINDS && hist[threadIdx.x]) atomicAdd(&A.st->kcount[threadIdx.x], hist[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_walk_lists(WalkArgs A) {
    WalkState* st = A.st;
    const uint32_t nj = st->nj;
    __shared__ uint32_t cnt[16], base[16];
    for (uint32_t r0 = blockIdx.x * 256; r0 < nj; r0 += gridDim.x * 256) {
        // ranks within the workgroup by LDS atomics, one global atomic per kind
        if (threadIdx.x < 16) cnt[threadIdx.x] = 0;
        __syncthreads();
        const uint32_t r = r0 + threadIdx.x;
        const uint32_t k = r < nj ? A.kind[r] : 0u;
        const uint32_t loc = r < nj ? atomicAdd(&cnt[k], 1u) : 0u;
        __syncthreads();
        if (threadIdx.x < DEC_KINDS && cnt[threadIdx.x]) {
            uint32_t kb = 0;                              // the kind's list starts after the lists before it
            for (uint32_t q = 0; q < threadIdx.x; q++) kb += st->kcount[q];
            base[threadIdx.x] = kb + atomicAdd(&st->kfill[threadIdx.x], cnt[threadIdx.x]);
        }
        __syncthreads();
        if (r < nj) {
            A.list[base[k] + loc] = r;
            const DecJob j = A.jobs[r];
            if (j.type == DEC_SKIP) {
                const uint32_t t = A.body[j.body_off - 18 + 4];
                if (!(t == 5 && !j.clen)) {                   // (an empty zlib payload decodes to nothing)
                    const uint32_t q = atomicAdd(&st->nhost, 1u);
                    if (q < A.host_cap) A.host[q] = HostChunk{j.body_off, j.out_off, j.clen, j.orig, t, 0};
                }
            }
        }
        __syncthreads();
    }
}

// after the piece's decode: produced[] against the expected lengths
__global__ __launch_bounds__(256) void k_walk_check(WalkArgs A) {
    WalkState* st = A.st;
    for (uint32_t r = gtid(); r < A.nj; r += gsize()) {
        const uint32_t p = A.produced[r];
        const DecJob j = A.jobs[r];
        if (p == DEC_PRODUCED_HOST) {
            const uint32_t q = atomicAdd(&st->nhinf, 1u);
            if (q < A.hinf_cap) A.hinf[q] = HostChunk{j.body_off, j.out_off, j.clen, j.orig, 5, 0};
        } else if (p == 0xFFFFFFFFu) {
            st->failed = 1;
        } else if (p != j.expect) {
            st->mismatch = 1;
        }
    }
}

}  // namespace

hipError_t launch_walk_piece(WalkArgs a, hipStream_t s) {
    const uint64_t a0 = a.a & ~15ull;
    a.ntiles = a.e > a.a ? (uint32_t)((a.e - a0 + WT_TILE - 1) / WT_TILE) : 0u;
    const dim3 B(256), G(WALK_GRID);
    if (a.ntiles) hipLaunchKernelGGL(k_walk_count, dim3(a.ntiles), B, 0, s, a);
    hipLaunchKernelGGL(k_walk_tscan, dim3(1), B, 0, s, a);
    if (a.ntiles) hipLaunchKernelGGL(k_walk_list, dim3(a.ntiles), B, 0, s, a);
    hipLaunchKernelGGL(k_walk_link, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_bexit, G, dim3(BT), 0, s, a);
    hipLaunchKernelGGL(k_walk_bentry, dim3(1), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_walk_bmark, G, dim3(BT), 0, s, a);
    hipLaunchKernelGGL(k_walk_bscan, dim3(1), B, 0, s, a);
    hipLaunchKernelGGL(k_walk_chain, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_jobs, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_bscan64, dim3(1), B, 0, s, a);
    hipLaunchKernelGGL(k_walk_fill, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_fin, dim3(1), dim3(1), 0, s, a);
    hipLaunchKernelGGL(k_walk_kcount, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_lists, G, B, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_walk_check(const WalkArgs& a, hipStream_t s) {
    if (!a.nj) return hipSuccess;
    const uint32_t g = (uint32_t)std::min<uint64_t>(WALK_GRID, (a.nj + 255) / 256);
    hipLaunchKernelGGL(k_walk_check, dim3(g), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace ambc
