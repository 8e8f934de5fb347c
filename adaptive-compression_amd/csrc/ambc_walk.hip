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
//   3. the chain from the entry candidate is marked by pointer doubling (round
//      k marks the 2^k-th successors of the marked nodes; a round that marks
//      nothing new ends it) -- marker bytes inside payloads are candidates too,
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

// candidate bits of the 16 positions at the 16-aligned base: the marker at
// base + t, for the positions in [a, e)
__device__ __forceinline__ uint32_t tile_bits(const uint8_t* body, uint64_t base, uint64_t a, uint64_t e) {
    if (base >= e) return 0;
    const uint32_t* b32 = reinterpret_cast<const uint32_t*>(body + base);
    uint32_t w[5];
#pragma unroll
    for (int q = 0; q < 5; q++) w[q] = b32[q];     // (base + 20 <= e + 19 <= blen + 2: the buffer's slack)
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
    for (uint32_t g = threadIdx.x; g < WT_TILE / 16; g += 256)
        c += (uint32_t)__popc(tile_bits(A.body, t0 + 16ull * g, A.a, A.e));
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
    if (t < 16) { st->kcount[t] = 0; st->kbase[t] = 0; st->kfill[t] = 0; }
    for (uint32_t k = t; k <= WALK_ROUNDS; k += 256) st->chg[k] = 0;
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
        uint32_t m = tile_bits(A.body, base, A.a, A.e);
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
        const bool root = p == entry;
        A.mark[i] = root ? 1 : 0;
        if (root) { st->root = i; st->chg[0] = 1; }
    }
}

// the entry must be a candidate when it lies in the piece
__global__ void k_walk_root(WalkArgs A) {
    WalkState* st = A.st;
    if (st->entry != WALK_ENDED && st->entry < A.e && st->root == ~0u) {
        st->err = 1;
        st->entry = WALK_ENDED;
    }
}

// ---- 3. the chain --------------------------------------------------------

__global__ __launch_bounds__(256) void k_walk_mark(WalkArgs A) {
    WalkState* st = A.st;
    const uint32_t k = A.round;
    if (!st->chg[k]) return;
    const uint32_t* J = (k & 1) ? A.jb : A.ja;
    const uint32_t nc = st->nc;
    bool any = false;
    for (uint32_t i = gtid(); i < nc; i += gsize()) {
        if (!A.mark[i]) continue;
        const uint32_t j = J[i];
        if (j < nc && !A.mark[j]) { A.mark[j] = 1; any = true; }
    }
    if (any) st->chg[k + 1] = 1;
}

__global__ __launch_bounds__(256) void k_walk_jump(WalkArgs A) {
    WalkState* st = A.st;
    const uint32_t k = A.round;
    if (!st->chg[k + 1]) return;
    const uint32_t* src = (k & 1) ? A.jb : A.ja;
    uint32_t* dst = (k & 1) ? A.ja : A.jb;
    const uint32_t nc = st->nc;
    for (uint32_t i = gtid(); i <= nc; i += gsize()) dst[i] = src[src[i]];
}

__global__ __launch_bounds__(256) void k_walk_mcount(WalkArgs A) {
    const uint32_t nc = A.st->nc, nb = (nc + 1023) / 1024;
    __shared__ uint32_t red[4];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        uint32_t c = 0;
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t i = b * 1024 + q * 256 + threadIdx.x;
            c += i < nc && A.mark[i] ? 1u : 0u;
        }
        c = wave_sum_u32(c);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) A.bc[b] = red[0] + red[1] + red[2] + red[3];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_walk_bscan(WalkArgs A) {
    __shared__ uint32_t s[256];
    serial_block_scan<uint32_t>(A.bc, (A.st->nc + 1023) / 1024, s, &A.st->nchain);
}

__global__ __launch_bounds__(256) void k_walk_chain(WalkArgs A) {
    const uint32_t nc = A.st->nc, nb = (nc + 1023) / 1024;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ uint32_t ws[4];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        uint32_t at = A.bc[b];
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t i = b * 1024 + q * 256 + threadIdx.x;
            const bool m = i < nc && A.mark[i];
            const uint64_t bal = __ballot(m);
            const uint32_t r = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
            if (lane == 0) ws[wave] = (uint32_t)__popcll(bal);
            __syncthreads();
            uint32_t before = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < 4; w++) {
                before += (uint32_t)w < wave ? ws[w] : 0u;
                tot += ws[w];
            }
            if (m) A.chain[at + before + r] = i;
            at += tot;
            __syncthreads();
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
__global__ __launch_bounds__(256) void k_walk_jobs(WalkArgs A) {
    const uint32_t nchain = A.st->nchain;
    for (uint32_t r = gtid(); r < nchain; r += gsize()) {
        const uint32_t i = A.chain[r];
        const uint64_t hp = A.cand[i];
        const uint8_t* h = A.body + hp;
        const uint32_t t = h[4];
        const uint32_t orig = rd32u(h + 10), clen = rd32u(h + 14);
        const bool stop = A.flg[i] & F_STOP;
        DecJob j{};
        uint32_t kind = DEC_KIND_HEAVY;
        uint64_t sneed = 0, expect = 0;
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
        } else if (t == 5 || t == 6 || t == 7) {
            j.type = DEC_SKIP;
            kind = DEC_KIND_LIGHT;
        } else {
            if (t == 255 || t == 1 || t == 4) kind = DEC_KIND_LIGHT;
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

__global__ __launch_bounds__(256) void k_walk_bsum(WalkArgs A) {
    const uint32_t n = A.st->nchain, nb = (n + 1023) / 1024;
    __shared__ uint64_t so[256], ss[256];
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        uint64_t o = 0, s = 0;
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t r = b * 1024 + q * 256 + threadIdx.x;
            if (r < n) { o += A.olen[r]; s += A.slen[r]; }
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

__global__ void k_walk_kbase(WalkArgs A) {
    WalkState* st = A.st;
    uint32_t at = 0;
    for (int k = 0; k < DEC_KINDS; k++) {
        st->kbase[k] = at;
        st->kfill[k] = at;
        at += st->kcount[k];
    }
}

__global__ __launch_bounds__(256) void k_walk_lists(WalkArgs A) {
    WalkState* st = A.st;
    const uint32_t nj = st->nj;
    for (uint32_t r = gtid(); r < nj; r += gsize()) {
        A.list[atomicAdd(&st->kfill[A.kind[r]], 1u)] = r;
        const DecJob j = A.jobs[r];
        if (j.type != DEC_SKIP) continue;
        const uint32_t t = A.body[j.body_off - 18 + 4];
        if (t == 5 && !j.clen) continue;              // an empty zlib payload decodes to nothing
        const uint32_t q = atomicAdd(&st->nhost, 1u);
        if (q < A.host_cap) A.host[q] = HostChunk{j.body_off, j.out_off, j.clen, j.orig, t, 0};
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

hipError_t launch_walk_piece(WalkArgs a, uint32_t rounds, hipStream_t s) {
    const uint64_t a0 = a.a & ~15ull;
    a.ntiles = a.e > a.a ? (uint32_t)((a.e - a0 + WT_TILE - 1) / WT_TILE) : 0u;
    const dim3 B(256), G(WALK_GRID);
    if (a.ntiles) hipLaunchKernelGGL(k_walk_count, dim3(a.ntiles), B, 0, s, a);
    hipLaunchKernelGGL(k_walk_tscan, dim3(1), B, 0, s, a);
    if (a.ntiles) hipLaunchKernelGGL(k_walk_list, dim3(a.ntiles), B, 0, s, a);
    hipLaunchKernelGGL(k_walk_link, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_root, dim3(1), dim3(1), 0, s, a);
    for (uint32_t k = 0; k < rounds && k < WALK_ROUNDS; k++) {
        a.round = k;
        hipLaunchKernelGGL(k_walk_mark, G, B, 0, s, a);
        hipLaunchKernelGGL(k_walk_jump, G, B, 0, s, a);
    }
    hipLaunchKernelGGL(k_walk_mcount, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_bscan, dim3(1), B, 0, s, a);
    hipLaunchKernelGGL(k_walk_chain, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_jobs, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_bsum, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_bscan64, dim3(1), B, 0, s, a);
    hipLaunchKernelGGL(k_walk_fill, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_fin, dim3(1), dim3(1), 0, s, a);
    hipLaunchKernelGGL(k_walk_kcount, G, B, 0, s, a);
    hipLaunchKernelGGL(k_walk_kbase, dim3(1), dim3(1), 0, s, a);
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
