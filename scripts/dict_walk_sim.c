/* Dictionary walkers: how many tokens NW greedy-parse walkers visit beyond the
 * single parse (parses from different starts meet quickly).  CPU simulation with
 * the reference rule (longest, then earliest match of up to 32 in a 4096 window).
 *   gcc -O2 -o /tmp/walk scripts/dict_walk_sim.c && /tmp/walk chunks.bin 4096 24
 * (chunks.bin: raw bytes, e.g. the ASCII class of scripts/kbench.py)  */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
// greedy-parse walker overshoot: M(p) per position (oracle rule), then NW walkers
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb"); size_t cs = atoi(argv[2]); int nchunks = atoi(argv[3]);
    uint8_t* buf = malloc(cs * nchunks); size_t got = fread(buf, 1, cs * nchunks, f); (void)got;
    int nws[] = {1, 2, 4, 8, 16, 32, 64};
    long tot_path = 0, tot_vis[7] = {0};
    for (int c = 0; c < nchunks; c++) {
        uint8_t* d = buf + c * cs; uint32_t n = cs;
        uint32_t* Lp = malloc(4 * n);
        for (uint32_t pos = 0; pos < n; pos++) {
            uint32_t start = pos > 4096 ? pos - 4096 : 0, look = n - pos < 32 ? n - pos : 32, bl = 0;
            for (uint32_t i = start; i < pos; i++) { uint32_t l = 0; while (l < look && d[i + l] == d[pos + l]) l++; if (l > bl) bl = l; }
            Lp[pos] = bl > 2 ? bl : 1;
        }
        for (uint32_t p = 0; p < n; p += Lp[p]) tot_path++;
        for (int w = 0; w < 7; w++) {
            int NW = nws[w]; uint8_t* vis = calloc(n, 1); long cnt = 0;
            // lock-step: each walker advances one token per round
            uint32_t P[64]; int act[64];
            for (int k = 0; k < NW; k++) { P[k] = (uint32_t)((uint64_t)n * k / NW); act[k] = 1; }
            for (int any = 1; any;) {
                any = 0;
                for (int k = 0; k < NW; k++) {
                    if (!act[k]) continue;
                    if (P[k] >= n || vis[P[k]]) { act[k] = 0; continue; }
                    vis[P[k]] = 1; cnt++; P[k] += Lp[P[k]]; any = 1;
                }
            }
            tot_vis[w] += cnt; free(vis);
        }
        free(Lp);
    }
    printf("path tokens/chunk %.1f\n", (double)tot_path / nchunks);
    for (int w = 0; w < 7; w++) printf("NW=%2d visited/chunk %.1f overhead %.1f%%\n", nws[w], (double)tot_vis[w] / nchunks, 100.0 * (tot_vis[w] - tot_path) / tot_path);
}
