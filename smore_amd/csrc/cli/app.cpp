// app -- flag-compatible replacement of cli/app.cpp (APP) on one MI355X
// or -gpus N.  Extra flags: -device, -gpus, -mode hogwild|atomic|hybrid|serial, -seed, -format cpp|go.
#include <vector>

#include "cli_common.h"

int main(int argc, char** argv) {
    int i;
    if (argc == 1) {
        printf("[smore-mi355x] APP\n\nOptions Description:\n");
        printf("\t-train <string>\n\t-save <string>\n\t-undirected <int> (1)\n\t-dimensions <int> (64)\n");
        printf("\t-walk_times <int> (10)\n\t-sample_times <int> (10)\n\t-jump <double> (0.15)\n");
        printf("\t-negative_samples <int> (5)\n\t-alpha <float> (0.025)\n\t-threads <int>\n");
        printf("\t-device <int> -gpus <int> -mode hogwild|atomic|hybrid|serial -seed <int> -format cpp|go\n");
        printf("Usage:\n./app -train net.txt -save rep.txt -undirected 1 -dimensions 64 -walk_times 10 "
               "-sample_times 10 -jump 0.15 -negative_samples 5 -alpha 0.025 -threads 1\n");
        return 0;
    }
    char network_file[4096] = "", rep_file[4096] = "";
    // defaults of cli/app.cpp:52-53
    int dimensions = 64, undirected = 1, negative_samples = 5, walk_times = 10, sample_times = 10, threads = 1;
    int device = 0, gpus = 1, fmt = 0, mode = SMORE_HYBRID;
    unsigned long long seed = 1;
    double init_alpha = 0.025, jump = 0.15;
    if ((i = ArgPos("-train", argc, argv)) > 0) snprintf(network_file, sizeof network_file, "%s", argv[i + 1]);
    if ((i = ArgPos("-save", argc, argv)) > 0) snprintf(rep_file, sizeof rep_file, "%s", argv[i + 1]);
    if ((i = ArgPos("-undirected", argc, argv)) > 0) undirected = atoi(argv[i + 1]);
    if ((i = ArgPos("-dimensions", argc, argv)) > 0) dimensions = atoi(argv[i + 1]);
    if ((i = ArgPos("-negative_samples", argc, argv)) > 0) negative_samples = atoi(argv[i + 1]);
    if ((i = ArgPos("-walk_times", argc, argv)) > 0) walk_times = atoi(argv[i + 1]);
    if ((i = ArgPos("-sample_times", argc, argv)) > 0) sample_times = atoi(argv[i + 1]);
    if ((i = ArgPos("-jump", argc, argv)) > 0) jump = atof(argv[i + 1]);
    if ((i = ArgPos("-alpha", argc, argv)) > 0) init_alpha = atof(argv[i + 1]);
    if ((i = ArgPos("-threads", argc, argv)) > 0) threads = atoi(argv[i + 1]);
    if ((i = ArgPos("-device", argc, argv)) > 0) device = atoi(argv[i + 1]);
    if ((i = ArgPos("-gpus", argc, argv)) > 0) gpus = atoi(argv[i + 1]);
    if ((i = ArgPos("-mode", argc, argv)) > 0) mode = mode_of(argv[i + 1]);
    if ((i = ArgPos("-seed", argc, argv)) > 0) seed = strtoull(argv[i + 1], 0, 10);
    if ((i = ArgPos("-format", argc, argv)) > 0) fmt = !strcmp(argv[i + 1], "go");

    Run run = open_run(device, gpus);
    smore_ctx* ctx = run.ctx;
    run_load(run, network_file, undirected, SMORE_VM_OUT_DEGREES, SMORE_NM_DEGREES);
    int64_t V = print_graph(ctx);
    printf("Model Setting:\n\tdimension:\t\t%d\n", dimensions);
    run_alloc(run, dimensions, 2);
    // APP::Init: W then C from one rand() stream (src/model/APP.cpp:35-58)
    SMORE_CLI_CHECK(ctx, smore_init_table_glibc(ctx, SMORE_W, 0));
    SMORE_CLI_CHECK(ctx, smore_init_table_glibc(ctx, SMORE_C, (uint64_t)V * dimensions));
    run_replicate(run);
    printf("Model:\n\t[APP]\nLearning Parameters:\n\twalk_times:\t\t%d\n\tsample_times:\t\t%d\n"
           "\tjumping factor:\t\t%g\n\tnegative_samples:\t%d\n\talpha:\t\t\t%g\n\tworkers:\t\t%d\nStart Training:\n",
           walk_times, sample_times, jump, negative_samples, init_alpha, threads);
    // start order: the per-walk_time rand() Fisher-Yates after Init's draws (src/model/APP.cpp:83-91)
    std::vector<int64_t> order((size_t)V * walk_times);
    smore_deepwalk_order(V, walk_times, 2ull * V * dimensions, order.data());
    const uint64_t units = (uint64_t)V * walk_times * sample_times;
    const uint64_t chunk = (((uint64_t)1 << 24) / sample_times * sample_times + sample_times) * (gpus > 1 ? gpus : 1);
    for (uint64_t b = 0; b < units; b += chunk) {
        uint64_t e = b + chunk < units ? b + chunk : units;
        if (run.g)
            SMORE_RUN_CHECK(run, smore_group_train_app(run.g, b, e, walk_times, sample_times, jump, negative_samples,
                                                       init_alpha, seed, order.data(), mode, 0, run.mean));
        else
            SMORE_RUN_CHECK(run, smore_train_app(ctx, b, e, walk_times, sample_times, jump, negative_samples,
                                                 init_alpha, seed, order.data(), mode));
        printf("\tProgress: %.3f %%%c", (double)e / units * 100, 13);
        fflush(stdout);
    }
    printf("\tProgress: 100.00 %%\n");
    save(ctx, rep_file, fmt);
    run_close(run);
    return 0;
}
