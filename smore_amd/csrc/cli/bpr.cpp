// bpr -- flag-compatible replacement of cli/bpr.cpp (BPR, UpdateBPRPair, 5
// rounds; `-negative_samples` and `-reg` are accepted and ignored by the
// update rule exactly as in src/proNet.cpp:1406-1455).  Extra flags: -device,
// -mode hogwild|atomic|hybrid|serial, -seed, -format cpp|go.
#include "cli_common.h"

int main(int argc, char** argv) {
    int i;
    if (argc == 1) {
        printf("[smore-mi355x] BPR\n\nOptions Description:\n");
        printf("\t-train <string>\n\t-save <string>\n\t-dimensions <int> (64)\n\t-sample_times <int> (10, x10^6)\n");
        printf("\t-alpha <float> (0.025)\n\t-threads <int>\n");
        printf("\t-device <int> -gpus <int> -mode hogwild|atomic|hybrid|serial -seed <int> -format cpp|go\n");
        printf("Usage:\n./bpr -train net.txt -save rep.txt -dimensions 64 -sample_times 10 -alpha 0.025 -threads 1\n");
        return 0;
    }
    char network_file[4096] = "", rep_file[4096] = "";
    int dimensions = 64, negative_samples = 5, sample_times = 10, threads = 1, device = 0, gpus = 1, fmt = 0;
    int mode = SMORE_HYBRID;
    unsigned long long seed = 1;
    double init_alpha = 0.025, reg = 0.01;
    if ((i = ArgPos("-train", argc, argv)) > 0) snprintf(network_file, sizeof network_file, "%s", argv[i + 1]);
    if ((i = ArgPos("-save", argc, argv)) > 0) snprintf(rep_file, sizeof rep_file, "%s", argv[i + 1]);
    if ((i = ArgPos("-dimensions", argc, argv)) > 0) dimensions = atoi(argv[i + 1]);
    if ((i = ArgPos("-negative_samples", argc, argv)) > 0) negative_samples = atoi(argv[i + 1]);
    if ((i = ArgPos("-sample_times", argc, argv)) > 0) sample_times = atoi(argv[i + 1]);
    if ((i = ArgPos("-reg", argc, argv)) > 0) reg = atof(argv[i + 1]);
    if ((i = ArgPos("-alpha", argc, argv)) > 0) init_alpha = atof(argv[i + 1]);
    if ((i = ArgPos("-threads", argc, argv)) > 0) threads = atoi(argv[i + 1]);
    if ((i = ArgPos("-device", argc, argv)) > 0) device = atoi(argv[i + 1]);
    if ((i = ArgPos("-gpus", argc, argv)) > 0) gpus = atoi(argv[i + 1]);
    if ((i = ArgPos("-mode", argc, argv)) > 0) mode = mode_of(argv[i + 1]);
    if ((i = ArgPos("-seed", argc, argv)) > 0) seed = strtoull(argv[i + 1], 0, 10);
    if ((i = ArgPos("-format", argc, argv)) > 0) fmt = !strcmp(argv[i + 1], "go");
    (void)negative_samples; (void)reg;

    Run run = open_run(device, gpus);
    smore_ctx* ctx = run.ctx;
    // BPR() sets negative_method "no_degrees" (src/model/BPR.cpp:4-7); LoadEdgeList(file, 0)
    run_load(run, network_file, 0, SMORE_VM_OUT_DEGREES, SMORE_NM_NO_DEGREES);
    print_graph(ctx);
    printf("Model Setting:\n\tdimension:\t\t%d\n", dimensions);
    run_alloc(run, dimensions, 1);
    SMORE_CLI_CHECK(ctx, smore_init_table_glibc(ctx, SMORE_W, 0));
    run_replicate(run);
    printf("Model:\n\t[BPR]\nLearning Parameters:\n\tsample_times:\t\t%d\n\talpha:\t\t\t%g\n\tworkers:\t\t%d\n"
           "Start Training:\n", sample_times, init_alpha, threads);
    const unsigned long long total = (unsigned long long)sample_times * 1000000ull;
    train_chunks(run, SMORE_BPR, total, total, 5, init_alpha, 0.0, seed, mode);
    save(ctx, rep_file, fmt);
    run_close(run);
    return 0;
}
