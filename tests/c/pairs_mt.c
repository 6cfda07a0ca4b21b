/* The Go UpdatePairs hook under the reference's concurrency (go/pkg/pronet/
 * hip.go updatePairsHIP; the reference's callers run UpdatePairs from
 * `workers` goroutines, internal/models/deepwalk/deepwalk.go:96-120): T host
 * threads, each issuing B one-walk batches of P random pairs against SHARED
 * host tables (Hogwild, as the Go caller's [][]float64), exactly as the hook
 * does per call: smore_pairs_rows lists the touched rows, they are gathered
 * from the shared tables, smore_train_pairs_rows_mt trains them (concurrent
 * calls combined into one device call), the rows are scattered back.
 *
 *   pairs_mt <edges.bin> <threads> <batches> <pairs> <dim> <K> <mt:0|1>
 *
 * edges.bin: int64 V, int64 E, then E int32 src, E int32 dst (directed slots).
 * Prints one JSON line: threads, pairs in total, seconds, pairs per second,
 * the device calls and the requests they served. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "smore_hip.h"

static smore_ctx* ctx;
static float *W, *C;
static int64_t V;
static int B, P, D, K, MT;
static volatile int failed;

static uint64_t next_rand(uint64_t* s) {
    uint64_t x = *s;
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return *s = x;
}

static void* worker(void* arg) {
    const int tid = (int)(intptr_t)arg;
    uint64_t st = 0x9E3779B97F4A7C15ull * (uint64_t)(tid + 1);
    int32_t* v = malloc(sizeof(int32_t) * P);
    int32_t* c = malloc(sizeof(int32_t) * P);
    int32_t* wi = malloc(sizeof(int32_t) * P);
    int32_t* ci = malloc(sizeof(int32_t) * P * (K + 1));
    float* wr = malloc(sizeof(float) * (size_t)P * D);
    float* cr = malloc(sizeof(float) * (size_t)P * (K + 1) * D);
    for (int b = 0; b < B && !failed; ++b) {
        for (int i = 0; i < P; ++i) {
            v[i] = (int32_t)(next_rand(&st) % (uint64_t)V);
            c[i] = (int32_t)(next_rand(&st) % (uint64_t)V);
        }
        const uint64_t unit = (uint64_t)tid * 1000003ull + (uint64_t)b;
        int64_t nw = 0, nc = 0;
        if (smore_pairs_rows(ctx, v, c, P, K, 7, unit, wi, &nw, ci, &nc) != SMORE_OK) {
            failed = 1;
            break;
        }
        for (int64_t i = 0; i < nw; ++i) memcpy(wr + i * D, W + (int64_t)wi[i] * D, sizeof(float) * D);
        for (int64_t i = 0; i < nc; ++i) memcpy(cr + i * D, C + (int64_t)ci[i] * D, sizeof(float) * D);
        const int rc = MT ? smore_train_pairs_rows_mt(ctx, v, c, P, K, 0.025, 7, unit, SMORE_ATOMIC, wi, nw, wr, ci,
                                                      nc, cr)
                          : smore_train_pairs_rows(ctx, v, c, P, K, 0.025, 7, unit, SMORE_ATOMIC, wi, nw, wr, ci, nc,
                                                   cr);
        if (rc != SMORE_OK) {
            fprintf(stderr, "train_pairs_rows: %s\n", smore_last_error(ctx));
            failed = 1;
            break;
        }
        for (int64_t i = 0; i < nw; ++i) memcpy(W + (int64_t)wi[i] * D, wr + i * D, sizeof(float) * D);
        for (int64_t i = 0; i < nc; ++i) memcpy(C + (int64_t)ci[i] * D, cr + i * D, sizeof(float) * D);
    }
    free(v);
    free(c);
    free(wi);
    free(ci);
    free(wr);
    free(cr);
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: pairs_mt edges.bin threads batches pairs dim K mt\n");
        return 2;
    }
    const int T = atoi(argv[2]);
    B = atoi(argv[3]);
    P = atoi(argv[4]);
    D = atoi(argv[5]);
    K = atoi(argv[6]);
    MT = atoi(argv[7]);
    FILE* f = fopen(argv[1], "rb");
    int64_t E = 0;
    if (!f || fread(&V, 8, 1, f) != 1 || fread(&E, 8, 1, f) != 1) return 2;
    int32_t* src = malloc(sizeof(int32_t) * E);
    int32_t* dst = malloc(sizeof(int32_t) * E);
    if (fread(src, 4, E, f) != (size_t)E || fread(dst, 4, E, f) != (size_t)E) return 2;
    fclose(f);
    double* wts = malloc(sizeof(double) * E);
    for (int64_t e = 0; e < E; ++e) wts[e] = 1.0;
    if (smore_create(0, &ctx) != SMORE_OK) return 3;
    if (smore_set_graph_edges(ctx, V, E, src, dst, wts, SMORE_VM_OUT_DEGREES, SMORE_NM_DEGREES) != SMORE_OK ||
        smore_set_semantics(ctx, SMORE_SEM_GO) != SMORE_OK ||
        smore_alloc_tables(ctx, D, 2) != SMORE_OK) {
        fprintf(stderr, "setup: %s\n", smore_last_error(ctx));
        return 3;
    }
    free(src);
    free(dst);
    free(wts);
    W = malloc(sizeof(float) * (size_t)V * D);
    C = calloc((size_t)V * D, sizeof(float));
    uint64_t st = 12345;
    for (int64_t i = 0; i < V * D; ++i) W[i] = ((float)(next_rand(&st) % 1000000) / 1e6f - 0.5f) / D;
    pthread_t* th = malloc(sizeof(pthread_t) * T);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
    for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    uint64_t calls = 0, reqs = 0;
    smore_pairs_combine_stats(ctx, &calls, &reqs);
    int finite = 1;
    for (int64_t i = 0; i < V * D && finite; ++i) finite = W[i] == W[i] && C[i] == C[i];
    printf("{\"threads\": %d, \"batches_per_thread\": %d, \"pairs_per_batch\": %d, \"dim\": %d, \"mt\": %d, "
           "\"pairs\": %lld, \"seconds\": %.4f, \"pairs_per_s\": %.1f, \"device_calls\": %llu, \"requests\": %llu, "
           "\"finite\": %d, \"failed\": %d}\n",
           T, B, P, D, MT, (long long)T * B * P, sec, (double)T * B * P / sec, (unsigned long long)calls,
           (unsigned long long)reqs, finite, failed);
    smore_destroy(ctx);
    return failed ? 1 : 0;
}
