// ambc_dictany.hip -- DictionaryCompression(window_size, lookahead_size).compress
// for any window, lookahead and input length (the plugin path outside k_dict's
// window-4096 / lookahead-32 / 8 KiB domain).
//
// The reference's parse (compression_methods.py:195-233) is greedy: at pos the
// longest match against a start i in [max(0, pos - window), pos) -- the
// earliest i among the longest (:301-311), compared over data[pos:pos+lookahead]
// (a Python slice, :295) -- becomes (1, dist lo, dist hi, len) when len > 2,
// else the literal (0, byte).  The match at a position does not depend on how
// the parse reached it, so the work splits into:
//   k_da_match  every position's token, one wave per position: the window's
//               starts 64 at a time, a 3-byte prefix test, dword-wide extension,
//               max length then lowest lane (= earliest start); stops at the
//               first start that reaches the cap.  tok[p] = jump (1 for a
//               literal, len for a match) | DA_ERR for a longest match of >= 256
//               bytes (bytearray.append raises there, :227) | dist16 << 16;
//   k_da_block  per block of DA_BP positions, pointer doubling in LDS: for each
//               of the 256 possible entry offsets (a jump is <= 255) the exit
//               offset into the next block and the token bytes on the way;
//   k_da_group  the block tables composed per group of DA_GB blocks;
//   k_da_serial one lane over the groups: each group's entry and output base,
//               the body's length and whether the path meets a DA_ERR token;
//   k_da_fill   per group, its blocks' entries and output bases;
//   k_da_emit   per block (one wave), the path through its 64-position windows
//               (scalar walk over readlanes), token offsets by ballot prefix
//               counts, 16-bit stores (every token is 2 or 4 bytes).
// Integer work, L1/L2-resident window reads: the bound is the match search's
// VALU issue (window / 64 steps per position), not HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "ambc_internal.h"
#include "ambc_wave.h"

namespace ambc {
namespace {

constexpr uint32_t DA_ERR = 0x100u;      // tok: the longest match is longer than 255 bytes
constexpr uint32_t DA_BP = 8192;         // positions per block (k_da_block)
constexpr uint32_t DA_BT = 512;          // k_da_block threads
constexpr uint32_t DA_NE = 256;          // entry offsets per block table
constexpr uint32_t DA_GB = 64;           // blocks per group
constexpr uint64_t DA_CMASK = (1ull << 48) - 1;   // table entry: cost | exit << 48 | err << 63
constexpr uint64_t DA_EBIT = 1ull << 63;

// the dword at byte offset i (two aligned loads; the buffer is padded by 64 bytes)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* in, uint64_t i) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(in);
    const uint32_t lo = w[i >> 2], hi = w[(i >> 2) + 1];
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(i & 3));
}

// len(data[p:p + look]) with Python's slice rules (negative stops wrap once)
__device__ __forceinline__ int64_t py_slice_len(int64_t p, int64_t look, int64_t n) {
    int64_t stop = p + look;
    if (stop < 0) {
        stop += n;
        if (stop < 0) stop = 0;
    }
    if (stop > n) stop = n;
    return stop > p ? stop - p : 0;
}

__global__ __launch_bounds__(256) void k_da_match(const uint8_t* __restrict__ in, uint32_t n, int64_t window,
                                                  int64_t look, uint32_t* __restrict__ tok) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t p = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); p < n; p += nw) {
        const int64_t cap64 = py_slice_len(p, look, n);
        const uint32_t cap = (uint32_t)min<int64_t>(cap64, 256);   // >= 256: the token raises anyway
        uint32_t bl = 0, bi = 0;
        if (cap >= 3 && window > 0) {
            const uint32_t s = (int64_t)p > window ? (uint32_t)(p - window) : 0u;
            const uint32_t t4 = ld32u(in, p);
#pragma unroll 1
            for (uint32_t base = s; base < p; base += 64u) {
                const uint32_t i = base + lane;
                uint32_t L = 0;
                if (i < p) {
                    const uint32_t c = ld32u(in, i);
                    if (((c ^ t4) & 0xFFFFFFu) == 0) {
                        if (c != t4) {
                            L = 3;
                        } else {
                            uint32_t k = 4;
                            while (k < cap) {
                                const uint32_t x = ld32u(in, (uint64_t)i + k) ^ ld32u(in, (uint64_t)p + k);
                                if (x) {
                                    k += (uint32_t)__builtin_ctz(x) >> 3;
                                    break;
                                }
                                k += 4;
                            }
                            L = k;
                        }
                        L = min(L, cap);
                    }
                }
                if (__any(L > bl)) {
                    const uint32_t m = (uint32_t)wave_max_i32((int)L);
                    if (m > bl) {   // strictly longer: a later window step never wins a tie
                        const uint64_t at = __ballot(L == m);
                        bl = m;
                        bi = base + (uint32_t)__builtin_ctzll(at);
                    }
                    if (bl >= cap) break;
                }
            }
        }
        if (lane == 0) {
            uint32_t t = 1u;
            if (bl > 2) t = bl > 255 ? (DA_ERR | 1u) : (bl | ((p - bi) & 0xFFFFu) << 16);
            tok[p] = t;
        }
    }
}

// (cost, err) of a chain in LDS: low 31 bits bytes, bit 31 a DA_ERR token on the way
__device__ __forceinline__ uint32_t cost_add(uint32_t a, uint32_t b) {
    return ((a & 0x7FFFFFFFu) + (b & 0x7FFFFFFFu)) | ((a | b) & 0x80000000u);
}

__global__ __launch_bounds__(DA_BT) void k_da_block(const uint32_t* __restrict__ tok, uint32_t n,
                                                    uint64_t* __restrict__ tab) {
    __shared__ uint16_t nx[DA_BP];
    __shared__ uint32_t cs[DA_BP];
    constexpr uint32_t PER = DA_BP / DA_BT;
    const uint32_t b = blockIdx.x;
    const uint64_t b0 = (uint64_t)b * DA_BP;
    const uint32_t nloc = (uint32_t)min<uint64_t>(DA_BP, n - b0);
    for (uint32_t q = threadIdx.x; q < nloc; q += DA_BT) {
        const uint32_t t = tok[b0 + q];
        const uint32_t j = t & 0xFFu;
        nx[q] = (uint16_t)min(q + j, 0xFFFFu);
        cs[q] = (j > 2 ? 4u : 2u) | ((t & DA_ERR) ? 0x80000000u : 0u);
    }
    __syncthreads();
    // pointer doubling: after r rounds every chain has taken 2^r steps or left the block
#pragma unroll 1
    for (uint32_t r = 0; (1u << r) < DA_BP; r++) {
        uint32_t vn[PER], vc[PER];
#pragma unroll
        for (uint32_t k = 0; k < PER; k++) {
            const uint32_t q = threadIdx.x + k * DA_BT;
            vn[k] = 0xFFFFu;
            if (q < nloc) {
                vn[k] = nx[q];
                vc[k] = cs[q];
                if (vn[k] < nloc) {
                    const uint32_t a = vn[k];
                    vc[k] = cost_add(vc[k], cs[a]);
                    vn[k] = nx[a];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < PER; k++) {
            const uint32_t q = threadIdx.x + k * DA_BT;
            if (q < nloc) {
                nx[q] = (uint16_t)vn[k];
                cs[q] = vc[k];
            }
        }
        __syncthreads();
    }
    for (uint32_t e = threadIdx.x; e < DA_NE; e += DA_BT) {
        uint64_t v = 0;
        if (e < nloc) {
            const uint32_t c = cs[e];
            v = (uint64_t)(c & 0x7FFFFFFFu) | (uint64_t)(nx[e] - nloc) << 48 | ((c >> 31) ? DA_EBIT : 0ull);
        }
        tab[(uint64_t)b * DA_NE + e] = v;
    }
}

__device__ __forceinline__ uint64_t tab_step(uint64_t acc, uint64_t x) {
    return (((acc & DA_CMASK) + (x & DA_CMASK)) & DA_CMASK) | ((acc | x) & DA_EBIT);
}

// per group of DA_GB blocks and entry offset e: the composed exit | cost | err
__global__ __launch_bounds__(DA_NE) void k_da_group(const uint64_t* __restrict__ tab, uint32_t nb,
                                                    uint64_t* __restrict__ gtab) {
    const uint32_t g = blockIdx.x, e0 = threadIdx.x;
    uint32_t e = e0;
    uint64_t acc = 0;
    const uint32_t b1 = min(nb, (g + 1) * DA_GB);
    for (uint32_t b = g * DA_GB; b < b1; b++) {
        const uint64_t x = tab[(uint64_t)b * DA_NE + e];
        acc = tab_step(acc, x);
        e = (uint32_t)(x >> 48) & 0xFFu;
    }
    gtab[(uint64_t)g * DA_NE + e0] = (acc & ~(0xFFull << 48)) | (uint64_t)e << 48;
}

// one lane: every group's entry and output base; res[0] = body bytes | err << 63
__global__ void k_da_serial(const uint64_t* __restrict__ gtab, uint32_t ng, uint32_t* __restrict__ gent,
                            uint64_t* __restrict__ gbase, uint64_t* __restrict__ res) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t e = 0;
    uint64_t acc = 0;
    for (uint32_t g = 0; g < ng; g++) {
        gent[g] = e;
        gbase[g] = acc & DA_CMASK;
        const uint64_t x = gtab[(uint64_t)g * DA_NE + e];
        acc = tab_step(acc, x);
        e = (uint32_t)(x >> 48) & 0xFFu;
    }
    res[0] = acc & (DA_CMASK | DA_EBIT);
}

__global__ void k_da_fill(const uint64_t* __restrict__ tab, uint32_t nb, uint32_t ng, const uint32_t* __restrict__ gent,
                          const uint64_t* __restrict__ gbase, uint32_t* __restrict__ bent, uint64_t* __restrict__ bbase) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ng) return;
    uint32_t e = gent[g];
    uint64_t o = gbase[g];
    const uint32_t b1 = min(nb, (g + 1) * DA_GB);
    for (uint32_t b = g * DA_GB; b < b1; b++) {
        bent[b] = e;
        bbase[b] = o;
        const uint64_t x = tab[(uint64_t)b * DA_NE + e];
        o += x & DA_CMASK;
        e = (uint32_t)(x >> 48) & 0xFFu;
    }
}

// one wave per block: the path from the block's entry, tokens at their offsets
__global__ __launch_bounds__(256) void k_da_emit(const uint8_t* __restrict__ in, const uint32_t* __restrict__ tok,
                                                 uint32_t n, uint32_t nb, const uint32_t* __restrict__ bent,
                                                 const uint64_t* __restrict__ bbase, uint8_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b >= nb) return;
    const uint64_t b0 = (uint64_t)b * DA_BP;
    const uint32_t nloc = (uint32_t)min<uint64_t>(DA_BP, n - b0);
    const uint64_t below = (1ull << lane) - 1ull;
    uint16_t* o16 = reinterpret_cast<uint16_t*>(out);
    uint32_t e = bent[b];
    uint64_t ob = bbase[b];
#pragma unroll 1
    for (uint32_t w0 = 0; w0 < nloc; w0 += 64u) {
        const uint32_t q = w0 + lane;
        const uint32_t t = q < nloc ? tok[b0 + q] : 1u;
        uint64_t on = 0;
        uint32_t x = e;
        const uint32_t wl = min(64u, nloc - w0);
        while (x < wl) {
            on |= 1ull << x;
            x += __builtin_amdgcn_readlane(t, x) & 0xFFu;
        }
        e = x - 64u;   // (meaningless past the block's last window)
        const bool me = (on >> lane) & 1ull;
        const uint32_t j = t & 0xFFu;
        const bool mt = me && j > 2;
        const uint64_t mm = __ballot(mt);
        const uint64_t off = ob + 2ull * (uint64_t)(__popcll(on & below) + __popcll(mm & below));
        if (mt) {
            const uint32_t d = t >> 16;
            o16[off >> 1] = (uint16_t)(1u | (d & 0xFFu) << 8);
            o16[(off >> 1) + 1] = (uint16_t)((d >> 8) | j << 8);
        } else if (me) {
            o16[off >> 1] = (uint16_t)((uint32_t)in[b0 + q] << 8);
        }
        ob += 2ull * (uint64_t)(__popcll(on) + __popcll(mm));
    }
}

}  // namespace

uint32_t dict_any_blocks(uint64_t n) { return (uint32_t)((n + DA_BP - 1) / DA_BP); }
uint32_t dict_any_groups(uint64_t n) { return (dict_any_blocks(n) + DA_GB - 1) / DA_GB; }
uint64_t dict_any_table_bytes(uint64_t n) { return (uint64_t)dict_any_blocks(n) * DA_NE * 8; }
uint64_t dict_any_gtable_bytes(uint64_t n) { return (uint64_t)dict_any_groups(n) * DA_NE * 8; }

// the parse and the path: a.res[0] = body bytes | 1 << 63 when the reference raises
hipError_t launch_dict_any_parse(const DictAnyArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const uint32_t nb = dict_any_blocks(a.n), ng = dict_any_groups(a.n);
    const uint32_t mg = (uint32_t)std::min<uint64_t>(((uint64_t)a.n + 3) / 4, 256u * 64u);
    hipLaunchKernelGGL(k_da_match, dim3(mg), dim3(256), 0, s, a.in, a.n, a.window, a.look, a.tok);
    hipLaunchKernelGGL(k_da_block, dim3(nb), dim3(DA_BT), 0, s, a.tok, a.n, a.tab);
    hipLaunchKernelGGL(k_da_group, dim3(ng), dim3(DA_NE), 0, s, a.tab, nb, a.gtab);
    hipLaunchKernelGGL(k_da_serial, dim3(1), dim3(64), 0, s, a.gtab, ng, a.gent, a.gbase, a.res);
    hipLaunchKernelGGL(k_da_fill, dim3((ng + 63) / 64), dim3(64), 0, s, a.tab, nb, ng, a.gent, a.gbase, a.bent,
                       a.bbase);
    return hipGetLastError();
}

hipError_t launch_dict_any_emit(const DictAnyArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const uint32_t nb = dict_any_blocks(a.n);
    hipLaunchKernelGGL(k_da_emit, dim3((nb + 3) / 4), dim3(256), 0, s, a.in, a.tok, a.n, nb, a.bent, a.bbase,
                       a.out);
    return hipGetLastError();
}

}  // namespace ambc
