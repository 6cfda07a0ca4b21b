/* gen_edgelist.c -- write a benchmark config's synthetic power-law graph as a
 * text edge list "v<a> v<b> 1" (one line per undirected line), for the loader
 * benchmark (tools/loader_bench.py).  Uses smore_gen_powerlaw (the same graph
 * bench.py builds in memory).
 *   gcc -O2 -Iinclude -o tools/gen_edgelist tools/gen_edgelist.c -Lsmore_amd/lib -lsmore_hip
 *   tools/gen_edgelist <V> <lines> <seed> <out.txt> */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "smore_hip.h"

static char* put_u(char* p, uint32_t x) {
    char t[12];
    int n = 0;
    do { t[n++] = (char)('0' + x % 10); x /= 10; } while (x);
    while (n) *p++ = t[--n];
    return p;
}

int main(int argc, char** argv) {
    if (argc != 5) { fprintf(stderr, "usage: gen_edgelist V lines seed out.txt\n"); return 1; }
    const int64_t V = atoll(argv[1]), lines = atoll(argv[2]);
    const uint64_t seed = strtoull(argv[3], 0, 10);
    int32_t* src = malloc(sizeof(int32_t) * lines);
    int32_t* dst = malloc(sizeof(int32_t) * lines);
    if (!src || !dst || smore_gen_powerlaw(V, lines, 0, 0.8, seed, src, dst) != SMORE_OK) return 2;
    FILE* f = fopen(argv[4], "wb");
    if (!f) return 3;
    char* buf = malloc(1 << 24);
    char* p = buf;
    for (int64_t l = 0; l < lines; ++l) {
        *p++ = 'v'; p = put_u(p, (uint32_t)src[l]); *p++ = ' ';
        *p++ = 'v'; p = put_u(p, (uint32_t)dst[l]); *p++ = ' '; *p++ = '1'; *p++ = '\n';
        if (p - buf > (1 << 24) - 64) { fwrite(buf, 1, (size_t)(p - buf), f); p = buf; }
    }
    fwrite(buf, 1, (size_t)(p - buf), f);
    fclose(f);
    return 0;
}
