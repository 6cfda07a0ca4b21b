/* go_shape.c -- the exact C call sequence of the Go cgo shim
 * (go/pkg/pronet/hip.go: NewHIP, TrainEdges, TrainDeepWalk), as a C program
 * the GPU tests can run (no Go toolchain in this image).  TEST
 * INFRASTRUCTURE: built by `make goshape`, driven by tests/test_gpu_goshape.py.
 *
 * input (little-endian): int64 V, E, dim, model (-1 = DeepWalk), K, total,
 * gpus, mode; double alpha, lambda; uint64 seed; int32 src[E], dst[E];
 * double w[E]; double nprob[V]; int64 nalias[V]; double W0[V*dim],
 * C0[V*dim]; DeepWalk only: int64 walk_times, walk_steps, window, n,
 * order[n]; node2vec (model -2): double p, q; metapath2vec (model -3, the
 * calls of metapath2vec_hip.go: NewHIPEdges, SetNodeTypes, TrainMetapath2Vec):
 * int64 ntypes, int32 type[V], int64 npaths, total, int32 lens[npaths],
 * paths[total]; CTDNE (model -4, ctdne_hip.go: NewHIPEdges, SetTemporalEdges,
 * TrainCTDNE): double time_window, int64 Et, int32 tsrc[Et], tdst[Et], double
 * ts[Et]; UpdatePairs (model -5, hip.go updatePairsHIP: NewHIP on one GPU,
 * BeginPairs, Pairs, EndPairs): int64 n, uint64 unit, int32 v[n], c[n].
 * output: double W[V*dim], C[V*dim] (C = C0 when not trained). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "smore_hip.h"

static void* rd(FILE* f, size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p || fread(p, 1, bytes, f) != bytes) {
        fprintf(stderr, "go_shape: short input\n");
        exit(3);
    }
    return p;
}

static int64_t rd64(FILE* f) {
    int64_t x;
    if (fread(&x, 8, 1, f) != 1) exit(3);
    return x;
}

static smore_group* G;
#define CHECK(what, expr)                                                                       \
    do {                                                                                        \
        if ((expr) != SMORE_OK) {                                                               \
            fprintf(stderr, "go_shape: %s: %s\n", what, G ? smore_group_last_error(G) : "?");   \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: go_shape <in.bin> <out.bin>\n");
        return 1;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 3;
    const int64_t V = rd64(f), E = rd64(f), dim = rd64(f), model = rd64(f), K = rd64(f), total = rd64(f),
                  gpus = rd64(f), mode = rd64(f);
    double ad[2];
    if (fread(ad, 8, 2, f) != 2) return 3;
    uint64_t seed;
    if (fread(&seed, 8, 1, f) != 1) return 3;
    int32_t* src = rd(f, 4 * E);
    int32_t* dst = rd(f, 4 * E);
    double* w = rd(f, 8 * E);
    double* nprob = rd(f, 8 * V);
    int64_t* nalias = rd(f, 8 * V);
    double* T[2] = {rd(f, 8 * V * dim), rd(f, 8 * V * dim)};
    int64_t walk_times = 0, walk_steps = 0, window = 0, n_order = 0;
    int64_t* order = NULL;
    if (model < 0 && model != -5) {
        walk_times = rd64(f);
        walk_steps = rd64(f);
        window = rd64(f);
        n_order = rd64(f);
        order = rd(f, 8 * n_order);
    }
    double pq[2] = {1.0, 1.0};   /* node2vec (model -2): p, q */
    if (model == -2 && fread(pq, 8, 2, f) != 2) return 3;
    int64_t ntypes = 0, npaths = 0, ptotal = 0, Et = 0;
    int32_t *types = NULL, *plens = NULL, *paths = NULL, *tsrc = NULL, *tdst = NULL;
    double twin = 0.0, *ts = NULL;
    if (model == -3) {
        ntypes = rd64(f);
        types = rd(f, 4 * V);
        npaths = rd64(f);
        ptotal = rd64(f);
        plens = rd(f, 4 * npaths);
        paths = rd(f, 4 * ptotal);
    }
    int64_t npairs = 0;
    uint64_t unit = 0;
    int32_t *pv = NULL, *pc = NULL;
    if (model == -5) {
        npairs = rd64(f);
        if (fread(&unit, 8, 1, f) != 1) return 3;
        pv = rd(f, 4 * npairs);
        pc = rd(f, 4 * npairs);
    }
    if (model == -4) {
        if (fread(&twin, 8, 1, f) != 1) return 3;
        Et = rd64(f);
        tsrc = rd(f, 4 * Et);
        tdst = rd(f, 4 * Et);
        ts = rd(f, 8 * Et);
    }
    fclose(f);

    /* NewHIP */
    int devs[64];
    for (int i = 0; i < gpus; ++i) devs[i] = i;
    if (smore_group_create(devs, (int)gpus, &G) != SMORE_OK) return 2;
    CHECK("set_graph_edges", smore_group_set_graph_edges(G, V, E, src, dst, w, SMORE_VM_OUT_DEGREES, SMORE_NM_DEGREES));
    CHECK("set_semantics", smore_group_set_semantics(G, SMORE_SEM_GO));
    for (int r = 0; r < gpus; ++r)
        CHECK("set_alias", smore_set_alias(smore_group_ctx(G, r), SMORE_AT_NEGATIVE, nprob, nalias, V));
    if (model == -3) CHECK("set_node_types", smore_group_set_node_types(G, types, (int)ntypes));    /* SetNodeTypes */
    if (model == -4) CHECK("set_temporal", smore_group_set_temporal_edges(G, Et, tsrc, tdst, ts)); /* SetTemporalEdges */
    /* TrainEdges / TrainDeepWalk: alloc, put + broadcast, chunked train, get */
    const int ntab = model == SMORE_LINE1 ? 1 : 2;
    CHECK("alloc_tables", smore_group_alloc_tables(G, (int)dim, ntab));
    smore_ctx* c0 = smore_group_ctx(G, 0);
    if (model == -5) {   /* (*HIP).PairsRows: list the touched rows, gather, train, scatter back */
        int32_t* wi = malloc(4 * npairs + 4);
        int32_t* ci = malloc(4 * npairs * (K + 1) + 4);
        int64_t nw = 0, nc = 0;
        CHECK("pairs_rows", smore_pairs_rows(c0, pv, pc, npairs, (int)K, seed, unit, wi, &nw, ci, &nc));
        float* wr = malloc(4 * nw * dim + 4);
        float* cr = malloc(4 * nc * dim + 4);
        for (int64_t i = 0; i < nw; ++i)
            for (int64_t k = 0; k < dim; ++k) wr[i * dim + k] = (float)T[0][wi[i] * dim + k];
        for (int64_t i = 0; i < nc; ++i)
            for (int64_t k = 0; k < dim; ++k) cr[i * dim + k] = (float)T[1][ci[i] * dim + k];
        CHECK("train_pairs_rows", smore_train_pairs_rows(c0, pv, pc, npairs, (int)K, ad[0], seed, unit, (int)mode,
                                                         wi, nw, wr, ci, nc, cr));
        for (int64_t i = 0; i < nw; ++i)
            for (int64_t k = 0; k < dim; ++k) T[0][wi[i] * dim + k] = (double)wr[i * dim + k];
        for (int64_t i = 0; i < nc; ++i)
            for (int64_t k = 0; k < dim; ++k) T[1][ci[i] * dim + k] = (double)cr[i * dim + k];
        smore_group_destroy(G);
        FILE* o = fopen(argv[2], "wb");
        if (!o) return 3;
        fwrite(T[0], 8, V * dim, o);
        fwrite(T[1], 8, V * dim, o);
        fclose(o);
        return 0;
    }
    float* buf = malloc(4 * V * dim + 4);
    for (int t = 0; t < ntab; ++t) {
        for (int64_t i = 0; i < V * dim; ++i) buf[i] = (float)T[t][i];
        CHECK("set_table", smore_set_table(c0, t, buf, V, (int)dim));
    }
    CHECK("broadcast", smore_group_broadcast_tables(G));
    if (model >= 0) {
        const uint64_t step = ((uint64_t)1 << 27) * (uint64_t)gpus;
        for (uint64_t done = 0; done < (uint64_t)total;) {
            uint64_t n = (uint64_t)total - done;
            if (n > step) n = step;
            CHECK("train_edges", smore_group_train_edges(G, (int)model, done, n, (uint64_t)total, (int)K, ad[0], ad[1],
                                                         seed, (int)mode, 0, 0));
            done += n;
        }
    } else {
        const uint64_t step = ((uint64_t)1 << 20) * (uint64_t)gpus;
        for (uint64_t done = 0; done < (uint64_t)n_order;) {
            uint64_t n = (uint64_t)n_order - done;
            if (n > step) n = step;
            if (model == -3)   /* TrainMetapath2Vec */
                CHECK("train_metapath2vec",
                      smore_group_train_metapath2vec(G, done, done + n, (int)walk_times, (int)walk_steps, (int)window,
                                                     (int)K, ad[0], paths, plens, (int)npaths, seed, order,
                                                     (int)mode, 0, 0));
            else if (model == -4)   /* TrainCTDNE */
                CHECK("train_ctdne", smore_group_train_ctdne(G, done, done + n, (int)walk_times, (int)walk_steps,
                                                             (int)window, (int)K, ad[0], twin, seed, order,
                                                             (int)mode, 0, 0));
            else if (model == -2)   /* TrainNode2Vec */
                CHECK("train_node2vec", smore_group_train_node2vec(G, done, done + n, (int)walk_times, (int)walk_steps,
                                                                   (int)window, (int)K, ad[0], pq[0], pq[1], seed,
                                                                   order, (int)mode, 0, 0));
            else
                CHECK("train_deepwalk", smore_group_train_deepwalk(G, done, done + n, (int)walk_times,
                                                                   (int)walk_steps, (int)window, (int)K, ad[0], seed,
                                                                   order, (int)mode, 0, 0));
            done += n;
        }
    }
    for (int t = 0; t < ntab; ++t) {
        CHECK("get_table", smore_get_table(c0, t, buf, V, (int)dim));
        for (int64_t i = 0; i < V * dim; ++i) T[t][i] = (double)buf[i];
    }
    smore_group_destroy(G);
    FILE* o = fopen(argv[2], "wb");
    if (!o) return 3;
    fwrite(T[0], 8, V * dim, o);
    fwrite(T[1], 8, V * dim, o);
    fclose(o);
    return 0;
}
