// deepwalk -- flag-compatible replacement of cli/deepwalk.cpp (DeepWalk) on one
// MI355X, including -load_v / -load_c warm starts in the SaveWeights format
// (proNet::LoadPreTrain, src/proNet.cpp:238-286).  Extra flags: -device,
// -mode hogwild|atomic|hybrid|serial, -seed, -format cpp|go.
#include <vector>

#include "cli_common.h"

int main(int argc, char** argv) {
    int i;
    if (argc == 1) {
        printf("[smore-mi355x] DeepWalk\n\nOptions Description:\n");
        printf("\t-train <string>\n\t-save <string>\n\t-load_v <string>\n\t-load_c <string>\n");
        printf("\t-undirected <int> (1)\n\t-dimensions <int> (64)\n\t-window_size <int> (5)\n");
        printf("\t-negative_samples <int> (5)\n\t-walk_times <int> (10)\n\t-walk_steps <int> (40)\n");
        printf("\t-alpha <float> (0.025)\n\t-threads <int>\n");
        printf("\t-device <int> -gpus <int> -mode hogwild|atomic|hybrid|serial -seed <int> -format cpp|go\n");
        printf("Usage:\n./deepwalk -train net.txt -save rep.txt -undirected 1 -dimensions 64 -walk_times 10 "
               "-walk_steps 40 -window_size 5 -negative_samples 5 -alpha 0.025 -threads 1\n");
        return 0;
    }
    char network_file[4096] = "", rep_file[4096] = "", load_v[4096] = "", load_c[4096] = "";
    // defaults of cli/deepwalk.cpp:56-57 (walk_steps 5 in the C++ CLI)
    int dimensions = 64, undirected = 1, window_size = 5, negative_samples = 5, walk_times = 10, walk_steps = 5;
    int threads = 1, device = 0, gpus = 1, fmt = 0, mode = SMORE_HYBRID;
    unsigned long long seed = 1;
    double init_alpha = 0.025;
    if ((i = ArgPos("-train", argc, argv)) > 0) snprintf(network_file, sizeof network_file, "%s", argv[i + 1]);
    if ((i = ArgPos("-save", argc, argv)) > 0) snprintf(rep_file, sizeof rep_file, "%s", argv[i + 1]);
    if ((i = ArgPos("-load_v", argc, argv)) > 0) snprintf(load_v, sizeof load_v, "%s", argv[i + 1]);
    if ((i = ArgPos("-load_c", argc, argv)) > 0) snprintf(load_c, sizeof load_c, "%s", argv[i + 1]);
    if ((i = ArgPos("-undirected", argc, argv)) > 0) undirected = atoi(argv[i + 1]);
    if ((i = ArgPos("-dimensions", argc, argv)) > 0) dimensions = atoi(argv[i + 1]);
    if ((i = ArgPos("-window_size", argc, argv)) > 0) window_size = atoi(argv[i + 1]);
    if ((i = ArgPos("-negative_samples", argc, argv)) > 0) negative_samples = atoi(argv[i + 1]);
    if ((i = ArgPos("-walk_times", argc, argv)) > 0) walk_times = atoi(argv[i + 1]);
    if ((i = ArgPos("-walk_steps", argc, argv)) > 0) walk_steps = atoi(argv[i + 1]);
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
    // DeepWalk::Init: W then C from one rand() stream (src/model/DeepWalk.cpp:43-55)
    SMORE_CLI_CHECK(ctx, smore_init_table_glibc(ctx, SMORE_W, 0));
    SMORE_CLI_CHECK(ctx, smore_init_table_glibc(ctx, SMORE_C, (uint64_t)V * dimensions));
    if (load_v[0]) { printf("\tload vertex pretrain:\t%s\n", load_v); SMORE_CLI_CHECK(ctx, smore_load_pretrain(ctx, SMORE_W, load_v)); }
    if (load_c[0]) { printf("\tload context pretrain:\t%s\n", load_c); SMORE_CLI_CHECK(ctx, smore_load_pretrain(ctx, SMORE_C, load_c)); }
    run_replicate(run);
    printf("Model:\n\t[DeepWalk]\nLearning Parameters:\n\twalk_times:\t\t%d\n\twalk_steps:\t\t%d\n"
           "\twindow_size:\t\t%d\n\tnegative_samples:\t%d\n\talpha:\t\t\t%g\n\tworkers:\t\t%d\nStart Training:\n",
           walk_times, walk_steps, window_size, negative_samples, init_alpha, threads);
    std::vector<int64_t> order((size_t)V * walk_times);
    smore_deepwalk_order(V, walk_times, 2ull * V * dimensions, order.data());
    const uint64_t total = (uint64_t)V * walk_times, chunk = (uint64_t)(1 << 20) * (gpus > 1 ? gpus : 1);
    for (uint64_t b = 0; b < total; b += chunk) {
        uint64_t e = b + chunk < total ? b + chunk : total;
        if (run.g)
            SMORE_RUN_CHECK(run, smore_group_train_deepwalk(run.g, b, e, walk_times, walk_steps, window_size,
                                                            negative_samples, init_alpha, seed, order.data(), mode, 0, run.mean));
        else
            SMORE_RUN_CHECK(run, smore_train_deepwalk(ctx, b, e, walk_times, walk_steps, window_size, negative_samples,
                                                      init_alpha, seed, order.data(), mode));
        printf("\tProgress: %.3f %%%c", (double)e / total * 100, 13);
        fflush(stdout);
    }
    printf("\tProgress: 100.00 %%\n");
    save(ctx, rep_file, fmt);
    run_close(run);
    return 0;
}
