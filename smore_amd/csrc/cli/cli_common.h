// cli_common.h -- argv handling shared by the flag-compatible CLIs
// (cli/line.cpp:4-14 ArgPos semantics: "-flag value", last flag wins nothing,
// missing value is an error).
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "smore_hip.h"

static int ArgPos(const char* str, int argc, char** argv) {
    for (int a = 1; a < argc; a++)
        if (!strcmp(str, argv[a])) {
            if (a == argc - 1) {
                printf("Argument missing for %s\n", str);
                exit(1);
            }
            return a;
        }
    return -1;
}

static int mode_of(const char* s) {
    if (!strcmp(s, "hogwild")) return SMORE_HOGWILD;
    if (!strcmp(s, "serial")) return SMORE_SERIAL;
    if (!strcmp(s, "atomic")) return SMORE_ATOMIC;
    return SMORE_HYBRID;
}

#define SMORE_CLI_CHECK(ctx, expr)                                                    \
    do {                                                                              \
        int rc_ = (expr);                                                             \
        if (rc_ != SMORE_OK) {                                                        \
            fprintf(stderr, "%s failed (%d): %s\n", #expr, rc_, smore_last_error(ctx)); \
            exit(2);                                                                  \
        }                                                                             \
    } while (0)

static smore_ctx* open_context(int device) {
    smore_ctx* ctx = nullptr;
    if (smore_create(device, &ctx) != SMORE_OK) {
        fprintf(stderr, "cannot create a context on device %d\n", device);
        exit(2);
    }
    return ctx;
}

static int64_t print_graph(smore_ctx* ctx) {
    int64_t V = 0, E = 0;
    smore_graph_info(ctx, &V, &E);
    printf("Connections:\n\t# of connection:\t%lld\n\t# of vertex:\t\t%lld\n", (long long)E, (long long)V);
    return V;
}

// run samples [0, n) of a run of `total` in launches of 2^26 with progress
static void train_chunks(smore_ctx* ctx, int model, unsigned long long total, unsigned long long n, int K,
                         double alpha, double reg, unsigned long long seed, int mode) {
    const unsigned long long chunk = 1ull << 26;
    for (unsigned long long done = 0; done < n;) {
        unsigned long long c = n - done < chunk ? n - done : chunk;
        SMORE_CLI_CHECK(ctx, smore_train_edges(ctx, model, done, c, total, K, alpha, reg, seed, mode));
        done += c;
        printf("\tProgress: %.3f %%%c", (double)done / total * 100, 13);
        fflush(stdout);
    }
    printf("\tProgress: 100.00 %%\n");
}

static void save(smore_ctx* ctx, const char* path, int fmt) {
    printf("Save Model:\n");
    SMORE_CLI_CHECK(ctx, smore_save_weights(ctx, SMORE_W, path, fmt));
    printf("\tSave to <%s>\n", path);
}
