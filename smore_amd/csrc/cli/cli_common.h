// cli_common.h -- argv handling shared by the flag-compatible CLIs
// (cli/line.cpp:4-14 ArgPos semantics: "-flag value", last flag wins nothing,
// missing value is an error).
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

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

// One training run on one GPU (a context) or on -gpus N GPUs (a replica group
// on devices device .. device+N-1, smore_group_*): replica 0 is the primary
// that loads, initialises and saves; its tables are broadcast before training
// and every replica agrees again when a training call returns.
struct Run {
    smore_group* g = nullptr;
    smore_ctx* ctx = nullptr;
    // -gpus N: the replicas' exchange rule, SMORE_SYNC=adaptive (the default:
    // per row the sum of the deltas for rows updated a few times per exchange,
    // towards their mean for the hub rows), mean, or sum (every update applied
    // once, with the hub rows synced between launches; it diverges at 4 and
    // more replicas at the default exchange period), DESIGN.md 10
    int mean = SMORE_SYNC_ADAPTIVE;
};

static Run open_run(int device, int gpus) {
    Run r;
    if (gpus <= 1) {
        r.ctx = open_context(device);
        return r;
    }
    std::vector<int> devs;
    for (int i = 0; i < gpus; ++i) devs.push_back(device + i);
    if (smore_group_create(devs.data(), gpus, &r.g) != SMORE_OK) {
        fprintf(stderr, "cannot create a %d-GPU group from device %d\n", gpus, device);
        exit(2);
    }
    r.ctx = smore_group_ctx(r.g, 0);
    if (const char* e = getenv("SMORE_SYNC"))
        r.mean = !strcmp(e, "sum") ? SMORE_SYNC_SUM : !strcmp(e, "mean") ? SMORE_SYNC_MEAN : SMORE_SYNC_ADAPTIVE;
    return r;
}

#define SMORE_RUN_CHECK(run, expr)                                                                   \
    do {                                                                                             \
        int rc_ = (expr);                                                                            \
        if (rc_ != SMORE_OK) {                                                                       \
            fprintf(stderr, "%s failed (%d): %s\n", #expr, rc_,                                      \
                    (run).g ? smore_group_last_error((run).g) : smore_last_error((run).ctx));         \
            exit(2);                                                                                 \
        }                                                                                            \
    } while (0)

static void run_load(Run& r, const char* path, int undirected, int vm, int nm) {
    if (r.g) SMORE_RUN_CHECK(r, smore_group_load_edgelist(r.g, path, undirected, vm, nm));
    else SMORE_RUN_CHECK(r, smore_load_edgelist(r.ctx, path, undirected, vm, nm));
}

static void run_alloc(Run& r, int dim, int ntables) {
    if (r.g) SMORE_RUN_CHECK(r, smore_group_alloc_tables(r.g, dim, ntables));
    else SMORE_RUN_CHECK(r, smore_alloc_tables(r.ctx, dim, ntables));
}

// after the primary's tables are initialised / warm-started
static void run_replicate(Run& r) {
    if (r.g) SMORE_RUN_CHECK(r, smore_group_broadcast_tables(r.g));
}

static void run_close(Run& r) {
    if (r.g) smore_group_destroy(r.g);
    else smore_destroy(r.ctx);
    r.g = nullptr;
    r.ctx = nullptr;
}

static int64_t print_graph(smore_ctx* ctx) {
    int64_t V = 0, E = 0;
    smore_graph_info(ctx, &V, &E);
    printf("Connections:\n\t# of connection:\t%lld\n\t# of vertex:\t\t%lld\n", (long long)E, (long long)V);
    return V;
}

// run samples [0, n) of a run of `total` in launches of 2^26 per GPU with
// progress (the edge-model CLIs line / mf / bpr; inline: the walk-model CLIs
// include this header without calling it)
inline void train_chunks(Run& r, int model, unsigned long long total, unsigned long long n, int K, double alpha,
                         double reg, unsigned long long seed, int mode) {
    const int gpus = r.g ? smore_group_size(r.g) : 1;
    const unsigned long long chunk = (1ull << 26) * (unsigned long long)gpus;
    for (unsigned long long done = 0; done < n;) {
        unsigned long long c = n - done < chunk ? n - done : chunk;
        if (r.g) SMORE_RUN_CHECK(r, smore_group_train_edges(r.g, model, done, c, total, K, alpha, reg, seed, mode, 0, r.mean));
        else SMORE_RUN_CHECK(r, smore_train_edges(r.ctx, model, done, c, total, K, alpha, reg, seed, mode));
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
