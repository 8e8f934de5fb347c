/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference's per-chunk selection + encode /
 * decode loop (KalharPandya/adaptive-compression, /root/reference).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the CPU baseline -- never as the
 * product path (the product is adaptive-compression_amd/csrc, HIP only).
 *
 * Pinned against the reference's own outputs: tests/golden/ JSON files and
 * tests/golden/files/ containers were produced by importing the reference
 * (tests/golden/make_golden.py); tests/test_oracle.py checks every vector.
 * The LZ4 block parse ("ambc-lz4 greedy v2") is this project's own algorithm
 * (python-lz4 is absent): its validity is pinned by the
 * system liblz4 decoding its frames, its bytes are parity-unpinned vs python-lz4.
 *
 * Build: make -C oracle   (gcc -O2 -fopenmp -shared -> oracle/_build/libambc_oracle.so)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <zlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* synthetic generator  (oracle/synth.py has the spec)                      */
/* ------------------------------------------------------------------------ */
#define GAMMA 0x9E3779B97F4A7C15ULL
#define SEG_MUL 0xD1B54A32D192ED03ULL

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static const char* VOCAB[16] = {"alpha", "beta", "gamma", "delta", "the", "quick", "brown", "fox",
                                "jumps", "over", "lazy", "dog", "data", "chunk", "marker", "stream"};

EXPORT void orc_synth(uint8_t* out, uint64_t n, uint64_t seed) {
    uint64_t s = seed, pos = 0, idx = 0;
    uint64_t cap = n / 1024 + 2;
    uint64_t* sp = (uint64_t*)malloc(cap * 3 * sizeof(uint64_t));
    uint64_t nseg = 0;
    while (pos < n) {
        s += GAMMA;
        uint64_t L = 1024 + mix64(s) % 130049ULL;
        if (L > n - pos) L = n - pos;
        sp[3 * nseg] = pos; sp[3 * nseg + 1] = L; sp[3 * nseg + 2] = idx;
        nseg++; pos += L; idx++;
    }
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t g = 0; g < (int64_t)nseg; g++) {
        uint64_t p = sp[3 * g], L = sp[3 * g + 1], id = sp[3 * g + 2];
        uint8_t* o = out + p;
        uint64_t base = mix64(seed ^ (id * SEG_MUL));
        int typ = (int)(id % 3);
        if (typ == 0) {
            memset(o, 0, L);
        } else if (typ == 1) {
            for (uint64_t j = 0; j * 8 < L; j++) {
                uint64_t w = mix64(base + (j + 1) * GAMMA);
                for (int b = 0; b < 8 && j * 8 + b < L; b++) o[j * 8 + b] = (uint8_t)(w >> (8 * b));
            }
        } else {
            uint64_t q = 0;
            for (uint64_t j = 0; q < L; j++) {
                const char* w = VOCAB[mix64(base + (j + 1) * GAMMA) >> 60];
                for (; *w && q < L; w++) o[q++] = (uint8_t)*w;
                if (q < L) o[q++] = ' ';
            }
        }
    }
    free(sp);
}

EXPORT void orc_random_bytes(uint8_t* out, uint64_t n, uint64_t seed) {
    uint64_t base = mix64(seed);
    for (uint64_t j = 0; j * 8 < n; j++) {
        uint64_t w = mix64(base + (j + 1) * GAMMA);
        for (int b = 0; b < 8 && j * 8 + b < n; b++) out[j * 8 + b] = (uint8_t)(w >> (8 * b));
    }
}

/* ------------------------------------------------------------------------ */
/* RLE  -- compression_methods.py:78-114 (enc), :116-152 (dec), :154-180    */
/* ------------------------------------------------------------------------ */
EXPORT int64_t orc_rle_encode(const uint8_t* d, uint32_t n, uint8_t* out) {
    if (n == 0) return 0;                       /* :88-89 */
    int64_t o = 0;
    uint8_t cur = d[0];
    uint32_t cnt = 1;
    for (uint32_t i = 1; i < n; i++) {          /* :95-105, runs split at 255 */
        if (d[i] == cur && cnt < 255) { cnt++; continue; }
        if (out) { out[o] = cur; out[o + 1] = (uint8_t)cnt; }
        o += 2; cur = d[i]; cnt = 1;
    }
    if (out) { out[o] = cur; out[o + 1] = (uint8_t)cnt; }
    return o + 2;
}

static int sampled_ratio_gt(const uint8_t* d, uint32_t n, int small_delta, double thr) {
    if (n < 4) return 0;                        /* :165-166 / :651-652 */
    uint32_t ss = n < 1000 ? n : 1000;
    uint32_t step = n / ss; if (step < 1) step = 1;
    uint32_t hits = 0;
    for (uint32_t i = 0; i + 1 < n; i += step) {
        if (small_delta) { int dd = (int)d[i] - (int)d[i + 1]; if (dd < 0) dd = -dd; hits += dd < 32; }
        else hits += d[i] == d[i + 1];
    }
    return ((double)hits / (double)(ss - 1)) > thr;
}
EXPORT int orc_rle_should_use(const uint8_t* d, uint32_t n) { return sampled_ratio_gt(d, n, 0, 0.3); }
/* DeltaCompression.should_use  compression_methods.py:640-667 */
EXPORT int orc_delta_should_use(const uint8_t* d, uint32_t n) { return sampled_ratio_gt(d, n, 1, 0.5); }

EXPORT int64_t orc_rle_decode(const uint8_t* p, uint32_t plen, uint32_t orig, uint8_t* out) {
    if (plen == 0) return 0;                    /* :127-128 */
    uint64_t o = 0;
    for (uint32_t i = 0; i + 1 < plen; i += 2) {   /* odd tail ignored :132-133 */
        uint32_t c = p[i + 1];
        for (uint32_t k = 0; k < c; k++) { if (o < orig) out[o] = p[i]; o++; }
    }
    if (o < orig) memset(out + o, 0, orig - o);   /* pad :145-150, truncate :142-144 */
    return orig;
}

/* ------------------------------------------------------------------------ */
/* Delta decode  compression_methods.py:610-638                              */
/* ------------------------------------------------------------------------ */
EXPORT int64_t orc_delta_decode(const uint8_t* p, uint32_t plen, uint32_t orig, uint8_t* out) {
    if (plen == 0) return 0;
    uint32_t m = plen < orig ? plen : orig;
    uint8_t prev = p[0];
    if (m > 0) out[0] = prev;
    for (uint32_t i = 1; i < m; i++) { prev = (uint8_t)(prev + p[i]); out[i] = prev; }
    return m;
}

/* ------------------------------------------------------------------------ */
/* Dictionary (simplified LZ77)  compression_methods.py:195-343             */
/* ------------------------------------------------------------------------ */
EXPORT int64_t orc_dict_encode(const uint8_t* d, uint32_t n, uint8_t* out) {
    if (n == 0) return 0;
    int64_t o = 0;
    uint32_t pos = 0;
    while (pos < n) {
        uint32_t start = pos > 4096 ? pos - 4096 : 0;     /* :294 window 4096 */
        uint32_t look = n - pos < 32 ? n - pos : 32;       /* :295 lookahead 32 */
        uint32_t best_pos = 0, best_len = 0;
        for (uint32_t i = start; i < pos; i++) {           /* :301-311 earliest wins ties */
            uint32_t l = 0;
            while (l < look && pos + l < n && d[i + l] == d[pos + l]) l++;
            if (l > best_len) { best_pos = i; best_len = l; }
        }
        if (best_len > 2) {                                 /* :215-227 */
            uint32_t dist = pos - best_pos;
            if (out) { out[o] = 1; out[o + 1] = dist & 0xFF; out[o + 2] = (dist >> 8) & 0xFF; out[o + 3] = (uint8_t)best_len; }
            o += 4; pos += best_len;
        } else {
            if (out) { out[o] = 0; out[o + 1] = d[pos]; }
            o += 2; pos += 1;
        }
    }
    return o;
}

/* DictionaryCompression(window_size, lookahead_size).compress for any window,
 * lookahead and length (compression_methods.py:187-233,279-313): the window
 * start max(0, pos - window) (:294), the lookahead as Python's slice
 * data[pos:pos + lookahead] (:295, negative stops wrap once), the earliest of
 * the longest matches (:301-311).  Returns the output length, or -2 where the
 * reference raises ValueError: a match longer than 255 bytes reaches
 * bytearray.append (:227). */
static int64_t py_slice_len(int64_t p, int64_t look, int64_t n) {
    int64_t stop = p + look;
    if (stop < 0) { stop += n; if (stop < 0) stop = 0; }
    if (stop > n) stop = n;
    return stop > p ? stop - p : 0;
}
EXPORT int64_t orc_dict_encode_wl(const uint8_t* d, uint32_t n, int64_t window, int64_t lookahead, uint8_t* out) {
    if (n == 0) return 0;
    int64_t o = 0;
    uint32_t pos = 0;
    while (pos < n) {
        int64_t st = (int64_t)pos - window;
        if (st < 0) st = 0;
        const int64_t look = py_slice_len(pos, lookahead, n);
        uint32_t best_pos = 0;
        int64_t best_len = 0;
        for (int64_t i = st; i < (int64_t)pos; i++) {
            int64_t l = 0;
            while (l < look && pos + l < n && d[i + l] == d[pos + l]) l++;
            if (l > best_len) { best_pos = (uint32_t)i; best_len = l; }
        }
        if (best_len > 2) {
            if (best_len > 255) return -2;
            const uint32_t dist = pos - best_pos;
            if (out) { out[o] = 1; out[o + 1] = dist & 0xFF; out[o + 2] = (dist >> 8) & 0xFF; out[o + 3] = (uint8_t)best_len; }
            o += 4; pos += (uint32_t)best_len;
        } else {
            if (out) { out[o] = 0; out[o + 1] = d[pos]; }
            o += 2; pos += 1;
        }
    }
    return o;
}

static int cmp_u32(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}
EXPORT int orc_dict_should_use(const uint8_t* d, uint32_t n) {   /* :315-343 */
    if (n < 100) return 0;
    uint32_t ss = n < 1000 ? n : 1000;
    uint32_t lim = n - 3 < ss ? n - 3 : ss;
    uint32_t tri[1000];
    for (uint32_t i = 0; i < lim; i++) tri[i] = (uint32_t)d[i] << 16 | (uint32_t)d[i + 1] << 8 | d[i + 2];
    qsort(tri, lim, sizeof(uint32_t), cmp_u32);
    uint32_t u = 0;
    for (uint32_t i = 0; i < lim; i++) u += (i == 0 || tri[i] != tri[i - 1]);
    return ((double)u / (double)ss) < 0.8;
}

/* returns produced length (<= orig), or -1 for a Python exception (caller zero-fills) */
EXPORT int64_t orc_dict_decode(const uint8_t* p, uint32_t plen, uint32_t orig, uint8_t* out) {
    if (plen == 0) return 0;                               /* :247-248 */
    uint64_t cap = (uint64_t)orig + 256;
    uint8_t* buf = (uint8_t*)malloc(cap ? cap : 1);
    uint64_t L = 0, pos = 0;
    int64_t ret = 0;
    while (pos < plen && L < orig) {                        /* :253 */
        uint8_t flag = p[pos++];
        if (flag == 0) {
            if (pos < plen) buf[L++] = p[pos++];
        } else if (pos + 2 < plen) {
            uint32_t dist = p[pos] | (uint32_t)p[pos + 1] << 8;
            uint32_t length = p[pos + 2];
            pos += 3;
            int64_t start = (int64_t)L - (int64_t)dist;
            for (uint32_t i = 0; i < length; i++) {         /* :273-278, Python indexing */
                int64_t idx = start + i;
                if (idx < (int64_t)L) {
                    if (idx < 0) idx += (int64_t)L;
                    if (idx < 0) { ret = -1; goto done; }   /* IndexError */
                    buf[L] = buf[idx]; L++;
                } else {
                    if (L == 0) { ret = -1; goto done; }
                    buf[L] = buf[L - 1]; L++;
                }
            }
        }
    }
    ret = (int64_t)(L < orig ? L : orig);
    memcpy(out, buf, (size_t)ret);
done:
    free(buf);
    return ret;
}

/* ------------------------------------------------------------------------ */
/* Huffman  compression_methods.py:354-574                                   */
/* ------------------------------------------------------------------------ */
/* Tree: merge the two smallest nodes ordered by (weight, first symbol of the
 * node) -- heapq order of [weight, [byte, code], ...] lists (:482-494); the
 * merged node's first symbol is lo's.  lo's leaves get '0', hi's get '1'. */
typedef struct { int16_t child[512][2]; int root; } huff_tree;

static int huff_build(int k, const uint8_t* syms, const uint64_t* w, huff_tree* t) {
    if (k == 0) return -1;            /* heappop on empty heap -> IndexError */
    if (k == 1) return -1;            /* code '' -> IndexError at :527 */
    uint64_t kw[256];
    int node[256];
    uint8_t act[256];
    memset(act, 0, sizeof act);
    for (int i = 0; i < k; i++) { kw[syms[i]] = w[i]; node[syms[i]] = syms[i]; act[syms[i]] = 1; }
    for (int m = 0; m < k - 1; m++) {
        int lo = -1, hi = -1;
        for (int s = 0; s < 256; s++) {
            if (!act[s]) continue;
            if (lo < 0 || kw[s] < kw[lo]) { hi = lo; lo = s; }
            else if (hi < 0 || kw[s] < kw[hi]) { hi = s; }
        }
        t->child[256 + m][0] = (int16_t)node[lo];
        t->child[256 + m][1] = (int16_t)node[hi];
        kw[lo] += kw[hi]; node[lo] = 256 + m; act[hi] = 0;
    }
    t->root = 256 + k - 2;
    return 0;
}

/* code lengths/values (MSB-first, <= 64 bits) for every leaf; -1 if deeper */
static int huff_codes(const huff_tree* t, uint8_t* len, uint64_t* code) {
    int stack[512], depth[512]; uint64_t val[512]; int sp = 0;
    stack[sp] = t->root; depth[sp] = 0; val[sp] = 0; sp++;
    while (sp) {
        sp--;
        int nd = stack[sp], dp = depth[sp]; uint64_t v = val[sp];
        if (nd < 256) { if (dp > 64) return -1; len[nd] = (uint8_t)dp; code[nd] = v; continue; }
        for (int b = 1; b >= 0; b--) {
            stack[sp] = t->child[nd][b]; depth[sp] = dp + 1; val[sp] = (v << 1) | (uint64_t)b; sp++;
        }
    }
    return 0;
}

/* test hook: codes for an explicit (symbol, weight) table; returns -1 on error */
EXPORT int orc_huff_code_table(int k, const uint8_t* syms, const uint64_t* w, uint8_t* len_out,
                               uint64_t* code_out) {
    huff_tree t;
    if (huff_build(k, syms, w, &t)) return -1;
    return huff_codes(&t, len_out, code_out);
}

/* first-occurrence-ordered histogram (Counter insertion order) */
static int first_order_hist(const uint8_t* d, uint32_t n, uint32_t* cnt, uint8_t* order) {
    int k = 0;
    memset(cnt, 0, 256 * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; i++) { if (cnt[d[i]]++ == 0) order[k++] = d[i]; }
    return k;
}

/* HuffmanCompression.should_use entropy, :566-574: summed in Counter order,
 * term = p*np.log2(p) with p = count/len.  tab (optional) holds numpy's term
 * for each count c (index c) at this n, so the sum is bit-exact to numpy. */
EXPORT double orc_huff_entropy(const uint8_t* d, uint32_t n, const double* tab) {
    uint32_t cnt[256]; uint8_t order[256];
    int k = first_order_hist(d, n, cnt, order);
    double e = 0.0;
    for (int i = 0; i < k; i++) {
        uint32_t c = cnt[order[i]];
        double t;
        if (tab) t = tab[c];
        else { double p = (double)c / (double)n; t = p * log2(p); }
        e = e - t;
    }
    return e;
}
EXPORT int orc_huff_should_use(const uint8_t* d, uint32_t n, const double* tab) {
    if (n < 100) return 0;
    return orc_huff_entropy(d, n, tab) < 7.0;
}

/* returns payload length, or -1 when the reference raises (k==1, k==256) */
EXPORT int64_t orc_huff_encode(const uint8_t* d, uint32_t n, uint8_t* out) {
    if (n == 0) return 0;
    uint32_t cnt[256]; uint8_t order[256];
    int k = first_order_hist(d, n, cnt, order);
    uint64_t w[256];
    for (int i = 0; i < k; i++) w[i] = cnt[order[i]];
    huff_tree t;
    if (huff_build(k, order, w, &t)) return -1;
    if (k >= 256) return -1;                         /* compressed.append(256) */
    uint8_t len[256]; uint64_t code[256];
    if (huff_codes(&t, len, code)) return -1;
    uint64_t nbits = 0;
    for (int i = 0; i < k; i++) nbits += (uint64_t)cnt[order[i]] * len[order[i]];
    int64_t total = 1 + 5 * k + 4 + (int64_t)((nbits + 7) / 8);
    if (!out) return total;
    int64_t o = 0;
    out[o++] = (uint8_t)k;
    for (int i = 0; i < k; i++) {
        uint32_t c = cnt[order[i]];
        out[o++] = order[i];
        for (int b = 0; b < 4; b++) out[o++] = (uint8_t)(c >> (8 * b));
    }
    for (int b = 0; b < 4; b++) out[o++] = (uint8_t)(nbits >> (8 * b));
    memset(out + o, 0, (size_t)(total - o));
    uint64_t bp = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t L = len[d[i]]; uint64_t v = code[d[i]];
        for (int b = L - 1; b >= 0; b--, bp++)
            if ((v >> b) & 1) out[o + (bp >> 3)] |= (uint8_t)(0x80 >> (bp & 7));
    }
    return total;
}

static uint64_t le_partial(const uint8_t* p, uint64_t pos, uint64_t plen, int nb) {
    uint64_t v = 0;
    for (int b = 0; b < nb && pos + b < plen; b++) v |= (uint64_t)p[pos + b] << (8 * b);
    return v;
}

/* :407-470; returns produced length (<= orig, may be shorter), -1 on exception */
EXPORT int64_t orc_huff_decode(const uint8_t* p, uint32_t plen, uint32_t orig, uint8_t* out) {
    if (plen == 0) return 0;
    int k = p[0];
    uint64_t pos = 1;
    uint8_t syms[256]; uint64_t w[256]; int idx[256]; int nf = 0;
    for (int s = 0; s < 256; s++) idx[s] = -1;
    for (int e = 0; e < k; e++) {
        if (pos >= plen) return -1;               /* data[pos] IndexError */
        uint8_t b = p[pos++];
        uint64_t c = le_partial(p, pos, plen, 4);
        pos += 4;
        if (idx[b] < 0) { idx[b] = nf; syms[nf] = b; nf++; }
        w[idx[b]] = c;                            /* dict: keep slot, overwrite value */
    }
    huff_tree t;
    if (huff_build(nf, syms, w, &t)) return -1;
    uint64_t nbits = le_partial(p, pos, plen, 4);
    pos += 4;
    uint64_t avail = pos < plen ? (plen - pos) * 8 : 0;
    if (nbits > avail) nbits = avail;
    int64_t o = 0;
    int nd = t.root;
    for (uint64_t bp = 0; bp < nbits; bp++) {
        int bit = (p[pos + (bp >> 3)] >> (7 - (bp & 7))) & 1;
        nd = t.child[nd][bit];
        if (nd < 256) {
            out[o++] = (uint8_t)nd;
            nd = t.root;
            if ((uint64_t)o >= orig) break;
        }
    }
    return o;
}

/* ------------------------------------------------------------------------ */
/* XXH32 (LZ4 frame header checksum)                                         */
/* ------------------------------------------------------------------------ */
#define P1 2654435761U
#define P2 2246822519U
#define P3 3266489917U
#define P4 668265263U
#define P5 374761393U
static inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t rd32(const uint8_t* p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }
EXPORT uint32_t orc_xxh32(const uint8_t* p, uint64_t len, uint32_t seed) {
    const uint8_t* e = p + len;
    uint32_t h;
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const uint8_t* lim = e - 16;
        do {
            v1 = rotl(v1 + rd32(p) * P2, 13) * P1; p += 4;
            v2 = rotl(v2 + rd32(p) * P2, 13) * P1; p += 4;
            v3 = rotl(v3 + rd32(p) * P2, 13) * P1; p += 4;
            v4 = rotl(v4 + rd32(p) * P2, 13) * P1; p += 4;
        } while (p <= lim);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    while (p + 4 <= e) { h = rotl(h + rd32(p) * P3, 17) * P4; p += 4; }
    while (p < e) { h = rotl(h + (*p) * P5, 11) * P1; p++; }
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

/* ------------------------------------------------------------------------ */
/* LZ4 ("ambc-lz4 greedy v2", this project's parse; frame = what            */
/* LZ4F_compressFrame emits for one <=64 KiB block, advanced_compression.py */
/* :272-281 calls lz4.frame.compress)                                        */
/*   hash h(i) = (u32le(d+i) * 2654435761) >> (32-10)                        */
/*   cand(i)   = max{ j < w(i) : h(j) == h(i) },  w(i) = i for i < 64, else   */
/*               64*floor(i/64) (earlier 64-position windows only);          */
/*               valid iff the 4 bytes match                                 */
/*   matchable i <= n-12; match end <= n-5 (LZ4 end-of-block rules)          */
/*   greedy: take the match at the first valid position, jump past it       */
/* ------------------------------------------------------------------------ */
#define LZ4_HB 10
static inline uint32_t lz4_hash(uint32_t v) { return (v * 2654435761U) >> (32 - LZ4_HB); }

static int64_t put_len(uint8_t* out, int64_t o, uint32_t v) {   /* ext bytes for v >= 15 */
    v -= 15;
    while (v >= 255) { if (out) out[o] = 255; o++; v -= 255; }
    if (out) out[o] = (uint8_t)v;
    return o + 1;
}

EXPORT int64_t orc_lz4_block_encode(const uint8_t* d, uint32_t n, uint8_t* out) {
    int32_t* last = (int32_t*)malloc(sizeof(int32_t) << LZ4_HB);
    for (int i = 0; i < (1 << LZ4_HB); i++) last[i] = -1;
    int64_t o = 0;
    uint32_t anchor = 0, i = 0, ins = 0;     /* ins: next position to insert */
    if (n >= 13) {
        uint32_t mlim = n - 12;
        while (i <= mlim) {
            const uint32_t w = i < 64 ? i : (i & ~63u);   /* earlier windows only */
            for (; ins < w; ins++) last[lz4_hash(rd32(d + ins))] = (int32_t)ins;
            uint32_t v = rd32(d + i);
            int32_t c = last[lz4_hash(v)];
            if (c >= 0 && rd32(d + c) == v) {
                uint32_t L = 4;
                while (i + L < n - 5 && d[c + L] == d[i + L]) L++;
                uint32_t lit = i - anchor, ml = L - 4;
                uint8_t tok = (uint8_t)((lit >= 15 ? 15 : lit) << 4 | (ml >= 15 ? 15 : ml));
                if (out) out[o] = tok;
                o++;
                if (lit >= 15) o = put_len(out, o, lit);
                if (out) memcpy(out + o, d + anchor, lit);
                o += lit;
                uint32_t off = i - (uint32_t)c;
                if (out) { out[o] = off & 0xFF; out[o + 1] = off >> 8; }
                o += 2;
                if (ml >= 15) o = put_len(out, o, ml);
                i += L; anchor = i;
            } else {
                i++;
            }
        }
    }
    uint32_t lit = n - anchor;
    if (out) out[o] = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
    o++;
    if (lit >= 15) o = put_len(out, o, lit);
    if (out) memcpy(out + o, d + anchor, lit);
    o += lit;
    free(last);
    return o;
}

/* more than 64 KiB (the single-call plugin at any length): one frame, the same
 * header with the whole content size, independent 64 KiB blocks each encoded
 * (or stored) as the one-block frame does, then the end mark */
static int64_t lz4_frame_multi(const uint8_t* d, uint32_t n, uint8_t* out) {
    int64_t o = 15;
    for (uint32_t b0 = 0; b0 < n; b0 += 65536) {
        const uint32_t m = n - b0 < 65536 ? n - b0 : 65536;
        int64_t blk = orc_lz4_block_encode(d + b0, m, NULL);
        int stored = blk >= (int64_t)m;
        if (out) {
            uint32_t bs = stored ? (m | 0x80000000U) : (uint32_t)blk;
            for (int b = 0; b < 4; b++) out[o + b] = (uint8_t)(bs >> (8 * b));
            if (stored) memcpy(out + o + 4, d + b0, m);
            else orc_lz4_block_encode(d + b0, m, out + o + 4);
        }
        o += 4 + (stored ? m : blk);
    }
    if (out) {
        uint8_t* h = out;
        h[0] = 0x04; h[1] = 0x22; h[2] = 0x4D; h[3] = 0x18;
        h[4] = 0x68; h[5] = 0x40;
        for (int b = 0; b < 8; b++) h[6 + b] = (uint8_t)((uint64_t)n >> (8 * b));
        h[14] = (uint8_t)((orc_xxh32(h + 4, 10, 0) >> 8) & 0xFF);
        memset(out + o, 0, 4);
    }
    return o + 4;
}

EXPORT int64_t orc_lz4_frame_encode(const uint8_t* d, uint32_t n, uint8_t* out) {
    if (n == 0) return 0;                  /* LZ4Compression.compress: empty -> b'' */
    if (n > 65536) return lz4_frame_multi(d, n, out);
    int64_t blk = orc_lz4_block_encode(d, n, NULL);
    int stored = blk >= (int64_t)n;
    int64_t total = 15 + 4 + (stored ? n : blk) + 4;
    if (!out) return total;
    uint8_t* h = out;
    h[0] = 0x04; h[1] = 0x22; h[2] = 0x4D; h[3] = 0x18;
    h[4] = 0x68; h[5] = 0x40;
    for (int b = 0; b < 8; b++) h[6 + b] = (uint8_t)((uint64_t)n >> (8 * b));
    h[14] = (uint8_t)((orc_xxh32(h + 4, 10, 0) >> 8) & 0xFF);
    uint32_t bs = stored ? (n | 0x80000000U) : (uint32_t)blk;
    for (int b = 0; b < 4; b++) out[15 + b] = (uint8_t)(bs >> (8 * b));
    if (stored) memcpy(out + 19, d, n);
    else orc_lz4_block_encode(d, n, out + 19);
    memset(out + total - 4, 0, 4);
    return total;
}

/* LZ4 block decode with bounds; returns produced bytes or -1 */
static int64_t lz4_block_decode(const uint8_t* s, uint64_t slen, uint8_t* dst, uint64_t dpos,
                                uint64_t dcap) {
    uint64_t ip = 0, op = dpos;
    for (;;) {
        if (ip >= slen) return -1;
        uint8_t tok = s[ip++];
        uint64_t lit = tok >> 4;
        if (lit == 15) { uint8_t b; do { if (ip >= slen) return -1; b = s[ip++]; lit += b; } while (b == 255); }
        if (ip + lit > slen || op + lit > dcap) return -1;
        memcpy(dst + op, s + ip, lit); ip += lit; op += lit;
        if (ip == slen) break;                     /* last sequence */
        if (ip + 2 > slen) return -1;
        uint64_t off = s[ip] | (uint64_t)s[ip + 1] << 8; ip += 2;
        if (off == 0 || off > op) return -1;
        uint64_t ml = tok & 15;
        if (ml == 15) { uint8_t b; do { if (ip >= slen) return -1; b = s[ip++]; ml += b; } while (b == 255); }
        ml += 4;
        if (op + ml > dcap) return -1;
        for (uint64_t k = 0; k < ml; k++) { dst[op] = dst[op - off]; op++; }
    }
    return (int64_t)(op - dpos);
}

/* lz4.frame.decompress + pad/truncate (advanced_compression.py:283-296);
 * returns orig, 0 for empty payload, -1 on a frame error (caller zero-fills). */
EXPORT int64_t orc_lz4_frame_decode(const uint8_t* p, uint32_t plen, uint32_t orig, uint8_t* out) {
    if (plen == 0) return 0;
    if (plen < 7 || rd32(p) != 0x184D2204U) return -1;
    uint8_t flg = p[4], bd = p[5];
    if ((flg >> 6) != 1 || (flg & 0x02) || (bd & 0x8F)) return -1;
    int bsid = (bd >> 4) & 7;
    if (bsid < 4) return -1;
    uint64_t bmax = 1ULL << (8 + 2 * bsid);
    uint64_t hp = 6, csize = 0;
    int has_cs = (flg >> 3) & 1, has_bck = (flg >> 4) & 1, has_cck = (flg >> 2) & 1, has_dict = flg & 1;
    if (has_cs) { if (hp + 8 > plen) return -1; csize = le_partial(p, hp, plen, 8); hp += 8; }
    if (has_dict) { if (hp + 4 > plen) return -1; hp += 4; }
    if (hp >= plen) return -1;
    if (((orc_xxh32(p + 4, hp - 4, 0) >> 8) & 0xFF) != p[hp]) return -1;
    hp++;
    uint64_t cap = has_cs ? csize : 0;
    uint64_t alloc = cap ? cap : (uint64_t)plen * 255 + 64;
    uint8_t* buf = (uint8_t*)malloc(alloc ? alloc : 1);
    uint64_t op = 0;
    int64_t ret = -1;
    for (;;) {
        if (hp + 4 > plen) goto done;
        uint32_t bs = rd32(p + hp); hp += 4;
        if (bs == 0) break;
        uint32_t sz = bs & 0x7FFFFFFFU;
        if (sz > bmax || hp + sz > plen) goto done;
        if (bs & 0x80000000U) {
            if (op + sz > alloc) goto done;
            memcpy(buf + op, p + hp, sz); op += sz;
        } else {
            uint64_t lim = op + bmax < alloc ? op + bmax : alloc;
            int64_t r = lz4_block_decode(p + hp, sz, buf, op, lim);
            if (r < 0) goto done;
            op += (uint64_t)r;
        }
        hp += sz;
        if (has_bck) {
            if (hp + 4 > plen) goto done;
            if (orc_xxh32(p + hp - sz, sz, 0) != rd32(p + hp)) goto done;
            hp += 4;
        }
    }
    if (has_cck) {
        if (hp + 4 > plen) goto done;
        if (orc_xxh32(buf, op, 0) != rd32(p + hp)) goto done;
    }
    if (has_cs && op != csize) goto done;
    {
        uint64_t m = op < orig ? op : orig;
        memcpy(out, buf, m);
        if (m < orig) memset(out + m, 0, orig - m);
        ret = orig;
    }
done:
    free(buf);
    return ret;
}

/* ------------------------------------------------------------------------ */
/* DEFLATE (id 5)   advanced_compression.py:71-107                           */
/* compress = zlib.compress(data, level=9) (CPython: deflateInit(level),     */
/* i.e. compress2), should_use = n >= 64 and calculate_entropy < 8.0 (:48-57,*/
/* :98-107; H reaches 8.0 only for an exactly uniform histogram).            */
/* ------------------------------------------------------------------------ */
EXPORT int64_t orc_deflate_encode(const uint8_t* d, uint32_t n, uint8_t* out) {
    if (n == 0) return 0;
    uLongf cap = compressBound(n);
    uint8_t* tmp = out ? NULL : (uint8_t*)malloc(cap);
    int rc = compress2(out ? out : tmp, &cap, d, n, 9);
    free(tmp);
    return rc == Z_OK ? (int64_t)cap : -1;
}

EXPORT int orc_deflate_should_use(const uint8_t* d, uint32_t n) {
    if (n < 64) return 0;
    uint32_t h[256] = {0};
    for (uint32_t i = 0; i < n; i++) h[d[i]]++;
    for (int s = 1; s < 256; s++) if (h[s] != h[0]) return 1;
    return 0;   /* exactly uniform: entropy == 8.0 */
}

/* ------------------------------------------------------------------------ */
/* "ambc-deflate v1": this project's DEFLATE (id 5) encoder, the GPU's       */
/* definition (the reference calls zlib.compress(level=9); any valid zlib    */
/* stream decodes there, and bytes are only round-trip tested).              */
/*  parse : h(i) = (u32le(d+i) * 2654435761) >> 21 for i <= n-4;             */
/*          cand(i) = last j < i with h(j) == h(i); match at p iff           */
/*          u32le(d+cand) == u32le(d+p) and p - cand <= 32768; greedy, the   */
/*          match taken at its full length capped at 258 and at n - p.       */
/*  codes : one final block, the smallest of dynamic / fixed / stored        */
/*          (ties in that order); Huffman lengths from the two-queue          */
/*          construction over (freq, symbol)-sorted leaves, limited to 15    */
/*          (7 for the code-length code) by the bl_count fix-up, assigned     */
/*          shortest-first from the most frequent (ties: higher symbol);     */
/*          code lengths run-length coded with 16/17/18 (rule in gd_rle).     */
/*  frame : zlib header 78 DA, the block, Adler-32 big-endian.               */
/* ------------------------------------------------------------------------ */
static const uint16_t GD_LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t GD_LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                    2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t GD_DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                      193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
                                      6145, 8193, 12289, 16385, 24577};
static const uint8_t GD_DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                    6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t GD_CLORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static int gd_lcode(uint32_t L) { int k = 28; while (GD_LBASE[k] > L) k--; return k; }
static int gd_dcode(uint32_t D) { int k = 29; while (GD_DBASE[k] > D) k--; return k; }

typedef struct { uint32_t pos, len, dist; } gd_seq;

EXPORT uint32_t orc_gd_parse(const uint8_t* d, uint32_t n, uint32_t* out3) {
    int32_t last[2048];
    for (int i = 0; i < 2048; i++) last[i] = -1;
    int32_t* cand = (int32_t*)malloc((size_t)(n ? n : 1) * 4);
    for (uint32_t i = 0; i < n; i++) cand[i] = -1;
    for (uint32_t i = 0; i + 4 <= n; i++) {
        uint32_t h = (rd32(d + i) * 2654435761u) >> 21;
        cand[i] = last[h];
        last[h] = (int32_t)i;
    }
    uint32_t ns = 0, p = 0;
    while (p < n) {
        int32_t c = cand[p];
        if (p + 4 <= n && c >= 0 && p - (uint32_t)c <= 32768 && rd32(d + c) == rd32(d + p)) {
            uint32_t L = 4;
            while (L < 258 && p + L < n && d[c + L] == d[p + L]) L++;
            if (out3) { out3[3 * ns] = p; out3[3 * ns + 1] = L; out3[3 * ns + 2] = p - (uint32_t)c; }
            ns++;
            p += L;
        } else {
            p++;
        }
    }
    free(cand);
    return ns;
}

/* Huffman code lengths, see the header comment */
EXPORT void orc_gd_lengths(const uint32_t* freq, int nsym, int maxbits, uint8_t* len) {
    int syms[320], k = 0;
    memset(len, 0, (size_t)nsym);
    for (int s = 0; s < nsym; s++) if (freq[s]) syms[k++] = s;
    if (k == 0) return;
    if (k == 1) { len[syms[0]] = 1; return; }
    /* sort by (freq, sym) ascending (insertion sort: k <= 320) */
    for (int i = 1; i < k; i++) {
        int s = syms[i], j = i - 1;
        while (j >= 0 && (freq[syms[j]] > freq[s] || (freq[syms[j]] == freq[s] && syms[j] > s))) {
            syms[j + 1] = syms[j];
            j--;
        }
        syms[j + 1] = s;
    }
    /* two-queue construction: leaves 0..k-1, internal nodes k..2k-2 */
    uint64_t w[640];
    int parent[640];
    for (int i = 0; i < k; i++) w[i] = freq[syms[i]];
    int a = 0, b = k, nb = k;   /* fronts of the leaf and internal queues, next internal id */
    for (int m = 0; m < k - 1; m++) {
        int pick[2];
        for (int t = 0; t < 2; t++) {
            if (a < k && (b >= nb || w[a] <= w[b])) pick[t] = a++;
            else pick[t] = b++;
        }
        w[nb] = w[pick[0]] + w[pick[1]];
        parent[pick[0]] = parent[pick[1]] = nb;
        nb++;
    }
    int depth[640];
    depth[nb - 1] = 0;
    for (int i = nb - 2; i >= 0; i--) depth[i] = depth[parent[i]] + 1;
    uint32_t blc[64] = {0};
    for (int i = 0; i < k; i++) blc[depth[i] > 63 ? 63 : depth[i]]++;
    /* limit to maxbits */
    for (int d2 = maxbits + 1; d2 < 64; d2++) { blc[maxbits] += blc[d2]; blc[d2] = 0; }
    uint64_t total = 0;
    for (int d2 = 1; d2 <= maxbits; d2++) total += (uint64_t)blc[d2] << (maxbits - d2);
    while (total > (1ull << maxbits)) {
        blc[maxbits]--;
        for (int d2 = maxbits - 1; d2 > 0; d2--)
            if (blc[d2]) { blc[d2]--; blc[d2 + 1] += 2; break; }
        total--;
    }
    /* shortest lengths to the most frequent symbols */
    int j = k;
    for (int d2 = 1; d2 <= maxbits; d2++)
        for (uint32_t c = blc[d2]; c > 0; c--) len[syms[--j]] = (uint8_t)d2;
}

/* canonical codes (RFC 1951 3.2.2), bit-reversed for LSB-first emission */
static void gd_codes(const uint8_t* len, int nsym, uint16_t* rcode) {
    uint32_t blc[16] = {0}, next[16];
    for (int s = 0; s < nsym; s++) blc[len[s]]++;
    blc[0] = 0;
    uint32_t c = 0;
    for (int b = 1; b < 16; b++) { c = (c + blc[b - 1]) << 1; next[b] = c; }
    for (int s = 0; s < nsym; s++) {
        if (!len[s]) { rcode[s] = 0; continue; }
        uint32_t v = next[len[s]]++, r = 0;
        for (int b = 0; b < len[s]; b++) r |= ((v >> b) & 1) << (len[s] - 1 - b);
        rcode[s] = (uint16_t)r;
    }
}

/* code-length RLE over the HLIT + HDIST lengths: (symbol, extra value) pairs.
 * run of zeros r: 18 x min(r,138) while r >= 11, then 17 x r if r >= 3, else
 * literal zeros; run of v != 0: v once, then 16 x min(r,6) while r >= 3, then
 * literal v for the rest. */
static int gd_rle(const uint8_t* L, int cnt, uint8_t* sym, uint8_t* ext) {
    int ns = 0, i = 0;
    while (i < cnt) {
        int v = L[i], r = 1;
        while (i + r < cnt && L[i + r] == v) r++;
        i += r;
        if (v == 0) {
            while (r >= 11) { int t = r < 138 ? r : 138; sym[ns] = 18; ext[ns++] = (uint8_t)(t - 11); r -= t; }
            if (r >= 3) { sym[ns] = 17; ext[ns++] = (uint8_t)(r - 3); r = 0; }
            while (r-- > 0) { sym[ns] = 0; ext[ns++] = 0; }
        } else {
            sym[ns] = (uint8_t)v; ext[ns++] = 0; r--;
            while (r >= 3) { int t = r < 6 ? r : 6; sym[ns] = 16; ext[ns++] = (uint8_t)(t - 3); r -= t; }
            while (r-- > 0) { sym[ns] = (uint8_t)v; ext[ns++] = 0; }
        }
    }
    return ns;
}

typedef struct { uint8_t* p; uint64_t bit; } gd_bits;
static void gd_put(gd_bits* o, uint32_t v, int nb) {
    for (int i = 0; i < nb; i++) {
        if ((v >> i) & 1) o->p[(o->bit + i) >> 3] |= (uint8_t)(1u << ((o->bit + i) & 7));
    }
    o->bit += nb;
}

static uint32_t gd_adler(const uint8_t* d, uint32_t n) {
    uint32_t a = 1, b = 0;
    for (uint32_t i = 0; i < n; i++) { a = (a + d[i]) % 65521; b = (b + a) % 65521; }
    return b << 16 | a;
}

/* returns the zlib stream length; writes it to out when out != NULL
 * (out must hold n + 5 * (n / 65535 + 1) + 6 bytes) */
EXPORT int64_t orc_gd_encode(const uint8_t* d, uint32_t n, uint8_t* out) {
    uint32_t* sq = (uint32_t*)malloc(((size_t)n / 4 + 2) * 12);
    uint32_t ns = orc_gd_parse(d, n, sq);
    uint32_t lf[286] = {0}, df[30] = {0};
    uint64_t extra = 0;
    uint32_t p = 0;
    for (uint32_t s = 0; s <= ns; s++) {
        uint32_t mp = s < ns ? sq[3 * s] : n;
        for (; p < mp; p++) lf[d[p]]++;
        if (s < ns) {
            int lc = gd_lcode(sq[3 * s + 1]), dc = gd_dcode(sq[3 * s + 2]);
            lf[257 + lc]++; df[dc]++;
            extra += GD_LEXT[lc] + GD_DEXT[dc];
            p += sq[3 * s + 1];
        }
    }
    lf[256] = 1;
    /* dynamic: at least two distance codes carry a length (zlib's convention) */
    uint32_t dfx[30];
    memcpy(dfx, df, sizeof dfx);
    { int used = 0; for (int i = 0; i < 30; i++) used += dfx[i] != 0;
      for (int i = 0; used < 2 && i < 2; i++) if (!dfx[i]) { dfx[i] = 1; used++; } }
    uint8_t ll[286], dl[30];
    orc_gd_lengths(lf, 286, 15, ll);
    orc_gd_lengths(dfx, 30, 15, dl);
    int hlit = 286; while (hlit > 257 && !ll[hlit - 1]) hlit--;
    int hdist = 30; while (hdist > 1 && !dl[hdist - 1]) hdist--;
    uint8_t cat[316], rs[316], re[316];
    memcpy(cat, ll, (size_t)hlit);
    memcpy(cat + hlit, dl, (size_t)hdist);
    int nr = gd_rle(cat, hlit + hdist, rs, re);
    uint32_t cf[19] = {0};
    for (int i = 0; i < nr; i++) cf[rs[i]]++;
    uint8_t cl[19];
    orc_gd_lengths(cf, 19, 7, cl);
    int hclen = 19; while (hclen > 4 && !cl[GD_CLORD[hclen - 1]]) hclen--;
    uint64_t dyn = 3 + 5 + 5 + 4 + 3ull * hclen;
    for (int i = 0; i < nr; i++) dyn += cl[rs[i]] + (rs[i] == 16 ? 2 : rs[i] == 17 ? 3 : rs[i] == 18 ? 7 : 0);
    uint64_t fix = 3;
    for (int s = 0; s < 286; s++) {
        dyn += (uint64_t)lf[s] * ll[s];
        fix += (uint64_t)lf[s] * (s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
    }
    for (int s = 0; s < 30; s++) { dyn += (uint64_t)df[s] * dl[s]; fix += (uint64_t)df[s] * 5; }
    dyn += extra; fix += extra;
    uint64_t nblk = n ? (n + 65534) / 65535 : 1;
    uint64_t by_dyn = (dyn + 7) / 8, by_fix = (fix + 7) / 8, by_sto = (uint64_t)n + 5 * nblk;
    int kind = by_dyn <= by_fix && by_dyn <= by_sto ? 2 : by_fix <= by_sto ? 1 : 0;
    uint64_t body = kind == 2 ? by_dyn : kind == 1 ? by_fix : by_sto;
    int64_t total = (int64_t)(2 + body + 4);
    if (out) {
        memset(out, 0, (size_t)total);
        out[0] = 0x78; out[1] = 0xDA;
        gd_bits o = {out + 2, 0};
        if (kind == 0) {
            uint8_t* q = out + 2;
            for (uint64_t b = 0, pos = 0; b < nblk; b++) {
                uint32_t L = (uint32_t)((n - pos) < 65535 ? (n - pos) : 65535);
                *q++ = b + 1 == nblk ? 1 : 0;
                q[0] = (uint8_t)L; q[1] = (uint8_t)(L >> 8); q[2] = (uint8_t)~L; q[3] = (uint8_t)(~L >> 8);
                q += 4;
                memcpy(q, d + pos, L); q += L; pos += L;
            }
        } else {
            uint8_t fl[288], fd[30];
            const uint8_t* LL = ll;
            const uint8_t* DL = dl;
            uint16_t lc[288], dcd[30];
            gd_put(&o, 1, 1);
            gd_put(&o, (uint32_t)kind, 2);
            if (kind == 1) {
                for (int s = 0; s < 288; s++) fl[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
                for (int s = 0; s < 30; s++) fd[s] = 5;
                LL = fl; DL = fd;
                gd_codes(fl, 288, lc);
                gd_codes(fd, 30, dcd);
            } else {
                gd_codes(ll, 286, lc);
                gd_codes(dl, 30, dcd);
                uint16_t cc[19];
                gd_codes(cl, 19, cc);
                gd_put(&o, (uint32_t)(hlit - 257), 5);
                gd_put(&o, (uint32_t)(hdist - 1), 5);
                gd_put(&o, (uint32_t)(hclen - 4), 4);
                for (int i = 0; i < hclen; i++) gd_put(&o, cl[GD_CLORD[i]], 3);
                for (int i = 0; i < nr; i++) {
                    gd_put(&o, cc[rs[i]], cl[rs[i]]);
                    if (rs[i] >= 16) gd_put(&o, re[i], rs[i] == 16 ? 2 : rs[i] == 17 ? 3 : 7);
                }
            }
            p = 0;
            for (uint32_t s = 0; s <= ns; s++) {
                uint32_t mp = s < ns ? sq[3 * s] : n;
                for (; p < mp; p++) gd_put(&o, lc[d[p]], LL[d[p]]);
                if (s < ns) {
                    uint32_t L = sq[3 * s + 1], D = sq[3 * s + 2];
                    int lcd = gd_lcode(L), dcc = gd_dcode(D);
                    gd_put(&o, lc[257 + lcd], LL[257 + lcd]);
                    gd_put(&o, L - GD_LBASE[lcd], GD_LEXT[lcd]);
                    gd_put(&o, dcd[dcc], DL[dcc]);
                    gd_put(&o, D - GD_DBASE[dcc], GD_DEXT[dcc]);
                    p += L;
                }
            }
            gd_put(&o, lc[256], LL[256]);
        }
        uint32_t ad = gd_adler(d, n);
        uint8_t* t = out + total - 4;
        t[0] = (uint8_t)(ad >> 24); t[1] = (uint8_t)(ad >> 16); t[2] = (uint8_t)(ad >> 8); t[3] = (uint8_t)ad;
    }
    free(sq);
    return total;
}

/* ------------------------------------------------------------------------ */
/* per-chunk selection   adaptive_compressor.py:537-590 (single candidate)  */
/* + _process_chunk :631-700                                                 */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint32_t chunk_size;
    uint32_t mode;          /* 0 native (per-chunk), 1 reference (remainder-raw) */
    uint32_t method_mask;   /* bit i -> method id i enabled (ids 1..15) */
    uint32_t flags;         /* ORC_GDEFLATE: id 5 = "ambc-deflate v1" (GPU engine), else zlib-9 */
    uint32_t pref_min[16];
    uint32_t pref_max[16];
    const double* ent_full; /* optional numpy entropy terms for n == chunk_size */
    const double* ent_tail; /* optional numpy entropy terms for n == N % chunk_size */
} orc_params;

#define ORC_GDEFLATE 1u

typedef struct {
    uint64_t method_usage[256];
    uint64_t total_chunks, compressed_chunks, raw_chunks;
    uint64_t bytes_saved, payload_bytes, overhead_bytes;
} orc_stats;

static int pref_ok(const orc_params* p, int id, uint32_t n) {
    return (p->method_mask >> id & 1) && p->pref_min[id] <= n && n <= p->pref_max[id];
}

/* returns winning id (255 = raw); *plen = payload length */
EXPORT int orc_select(const uint8_t* d, uint32_t n, const orc_params* p, const double* tab,
                      int64_t* plen) {
    int64_t best = n;            /* (len+18)/n < 1.0  <=>  len+18 < n */
    int win = 255;
    int64_t wl = n;
    if (pref_ok(p, 1, n) && orc_rle_should_use(d, n)) {
        int64_t l = orc_rle_encode(d, n, NULL);
        if (l + 18 < best) { best = l + 18; win = 1; wl = l; }
    }
    if (pref_ok(p, 2, n) && orc_dict_should_use(d, n)) {
        int64_t l = orc_dict_encode(d, n, NULL);
        if (l + 18 < best) { best = l + 18; win = 2; wl = l; }
    }
    if (pref_ok(p, 3, n) && orc_huff_should_use(d, n, tab)) {
        int64_t l = orc_huff_encode(d, n, NULL);
        if (l >= 0 && l + 18 < best) { best = l + 18; win = 3; wl = l; }
    }
    /* id 4 (Delta): payload length == n, can never satisfy len+18 < n */
    if (pref_ok(p, 5, n) && orc_deflate_should_use(d, n)) {
        int64_t l = (p->flags & ORC_GDEFLATE) ? orc_gd_encode(d, n, NULL) : orc_deflate_encode(d, n, NULL);
        if (l >= 0 && l + 18 < best) { best = l + 18; win = 5; wl = l; }
    }
    if (pref_ok(p, 9, n) && n >= 1024) {          /* LZ4 should_use :298-307 */
        int64_t l = orc_lz4_frame_encode(d, n, NULL);
        if (l + 18 < best) { best = l + 18; win = 9; wl = l; }
    }
    *plen = wl;
    return win;
}

static void put_hdr(uint8_t* o, int type, uint32_t used, uint32_t orig, uint32_t clen) {
    o[0] = 0xFF; o[1] = 0xFF; o[2] = 0; o[3] = 0;        /* marker, :303-310 */
    o[4] = (uint8_t)type; o[5] = 0;
    for (int b = 0; b < 4; b++) {
        o[6 + b] = (uint8_t)(used >> (8 * b));
        o[10 + b] = (uint8_t)(orig >> (8 * b));
        o[14 + b] = (uint8_t)(clen >> (8 * b));
    }
}

static int64_t encode_payload(int id, const uint8_t* d, uint32_t n, uint8_t* out, uint32_t flags) {
    if (id == 5 && (flags & ORC_GDEFLATE)) return orc_gd_encode(d, n, out);
    switch (id) {
    case 1: return orc_rle_encode(d, n, out);
    case 2: return orc_dict_encode(d, n, out);
    case 3: return orc_huff_encode(d, n, out);
    case 5: return orc_deflate_encode(d, n, out);
    case 9: return orc_lz4_frame_encode(d, n, out);
    default: memcpy(out, d, n); return n;
    }
}

/* ids of every chunk (native decisions) -> used by tests as well */
EXPORT void orc_decide_all(const uint8_t* in, uint64_t n, const orc_params* p, uint8_t* ids,
                           uint32_t* plens, int nthreads) {
    uint64_t C = p->chunk_size, M = (n + C - 1) / C;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    (void)nthreads;
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t k = 0; k < (int64_t)M; k++) {
        uint64_t pos = (uint64_t)k * C;
        uint32_t len = (uint32_t)(n - pos < C ? n - pos : C);
        const double* tab = len == C ? p->ent_full : p->ent_tail;
        int64_t pl;
        ids[k] = (uint8_t)orc_select(in + pos, len, p, tab, &pl);
        plens[k] = (uint32_t)pl;
    }
}

/* _adaptive_compress (:363-394) with CHUNK_SIZE_CANDIDATES=[C].
 * Returns body length (incl. 16-B end chunk), -1 if out_cap too small,
 * -2 if a reference-mode raw remainder does not fit the u32 fields. */
EXPORT int64_t orc_compress_body(const uint8_t* in, uint64_t n, const orc_params* p, uint8_t* out,
                                 uint64_t out_cap, orc_stats* st, int nthreads) {
    uint64_t C = p->chunk_size, M = (n + C - 1) / C;
    uint8_t* ids = (uint8_t*)malloc(M ? M : 1);
    uint32_t* pl = (uint32_t*)malloc((M ? M : 1) * sizeof(uint32_t));
    orc_decide_all(in, n, p, ids, pl, nthreads);
    uint64_t R = M;                                  /* first chunk with no winner */
    if (p->mode == 1) for (uint64_t k = 0; k < M; k++) if (ids[k] == 255) { R = k; break; }
    uint64_t* off = (uint64_t*)malloc((M + 1) * sizeof(uint64_t));
    off[0] = 0;
    for (uint64_t k = 0; k < M; k++) {
        uint64_t len = n - k * C < C ? n - k * C : C;
        uint64_t sz;
        if (k < R) sz = 18 + (ids[k] == 255 ? len : pl[k]);
        else if (k == R) sz = 18 + (n - k * C);
        else sz = 0;
        off[k + 1] = off[k] + sz;
    }
    int64_t total = (int64_t)off[M] + 16;
    if (R < M && n - R * C > 0xFFFFFFFFULL) { total = -2; goto out; }
    if ((uint64_t)total > out_cap) { total = -1; goto out; }
    memset(st, 0, sizeof *st);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t k = 0; k < (int64_t)(R < M ? R : M); k++) {
        uint64_t pos = (uint64_t)k * C;
        uint32_t len = (uint32_t)(n - pos < C ? n - pos : C);
        uint8_t* o = out + off[k];
        int id = ids[k];
        uint32_t clen = id == 255 ? len : pl[k];
        put_hdr(o, id, len, len, clen);
        encode_payload(id, in + pos, len, o + 18, p->flags);
    }
    for (uint64_t k = 0; k < (R < M ? R : M); k++) {
        uint64_t len = n - k * C < C ? n - k * C : C;
        st->total_chunks++;
        if (ids[k] == 255) st->raw_chunks++;
        else {
            st->compressed_chunks++;
            st->method_usage[ids[k]]++;
            st->payload_bytes += pl[k];
            st->overhead_bytes += 18;
            st->bytes_saved += len - (pl[k] + 18);
        }
    }
    if (R < M) {
        uint64_t rem = n - R * C;
        put_hdr(out + off[R], 255, (uint32_t)rem, (uint32_t)rem, (uint32_t)rem);
        memcpy(out + off[R] + 18, in + R * C, rem);
        st->total_chunks++; st->raw_chunks++;
    }
    {
        uint8_t* e = out + off[M];              /* _create_end_chunk :595-607 (u16 used) */
        e[0] = 0xFF; e[1] = 0xFF; memset(e + 2, 0, 14);
        st->overhead_bytes += 16;
    }
out:
    free(ids); free(pl); free(off);
    return total;
}
