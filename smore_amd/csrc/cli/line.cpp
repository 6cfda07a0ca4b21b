// line -- flag-compatible replacement of cli/line.cpp (LINE 1st/2nd order) on
// one MI355X.  Extra flags: -device <int>, -mode hogwild|atomic|hybrid|serial,
// -seed <int>, -format cpp|go (SaveWeights number format).
#include <string>

#include "cli_common.h"

int main(int argc, char** argv) {
    int i;
    if (argc == 1) {
        printf("[smore-mi355x] LINE\n\n");
        printf("Options Description:\n");
        printf("\t-train <string>\n\t\tTrain the Network data\n");
        printf("\t-save <string>\n\t\tSave the representation data\n");
        printf("\t-dimensions <int>\n\t\tDimension of vertex representation; default is 64\n");
        printf("\t-undirected <int>\n\t\tWhether the edge is undirected; default is 1\n");
        printf("\t-order <int>\n\t\tLearning with 1st/2nd order; default is 2\n");
        printf("\t-negative_samples <int>\n\t\tNumber of negative examples; default is 5\n");
        printf("\t-sample_times <int>\n\t\tNumber of training samples *Million; default is 10\n");
        printf("\t-threads <int>\n\t\tAccepted for compatibility (the GPU runs one Hogwild stream)\n");
        printf("\t-alpha <float>\n\t\tInit learning rate; default is 0.025\n");
        printf("\t-device <int> -gpus <int> -mode hogwild|atomic|hybrid|serial -seed <int> -format cpp|go\n");
        printf("Usage:\n./line -train net.txt -save rep.txt -undirected 1 -order 2 -dimensions 64 "
               "-sample_times 10 -negative_samples 5 -alpha 0.025 -threads 1\n");
        return 0;
    }
    char network_file[4096] = "", rep_file[4096] = "";
    int dimensions = 64, undirected = 1, negative_samples = 5, sample_times = 10, threads = 1, order = 2;
    int device = 0, gpus = 1, mode = SMORE_HYBRID, fmt = 0;
    unsigned long long seed = 1;
    double init_alpha = 0.025;
    if ((i = ArgPos("-train", argc, argv)) > 0) snprintf(network_file, sizeof network_file, "%s", argv[i + 1]);
    if ((i = ArgPos("-save", argc, argv)) > 0) snprintf(rep_file, sizeof rep_file, "%s", argv[i + 1]);
    if ((i = ArgPos("-undirected", argc, argv)) > 0) undirected = atoi(argv[i + 1]);
    if ((i = ArgPos("-order", argc, argv)) > 0) order = atoi(argv[i + 1]);
    if ((i = ArgPos("-dimensions", argc, argv)) > 0) dimensions = atoi(argv[i + 1]);
    if ((i = ArgPos("-negative_samples", argc, argv)) > 0) negative_samples = atoi(argv[i + 1]);
    if ((i = ArgPos("-sample_times", argc, argv)) > 0) sample_times = atoi(argv[i + 1]);
    if ((i = ArgPos("-alpha", argc, argv)) > 0) init_alpha = atof(argv[i + 1]);
    if ((i = ArgPos("-threads", argc, argv)) > 0) threads = atoi(argv[i + 1]);
    if ((i = ArgPos("-device", argc, argv)) > 0) device = atoi(argv[i + 1]);
    if ((i = ArgPos("-gpus", argc, argv)) > 0) gpus = atoi(argv[i + 1]);
    if ((i = ArgPos("-mode", argc, argv)) > 0) mode = mode_of(argv[i + 1]);
    if ((i = ArgPos("-seed", argc, argv)) > 0) seed = strtoull(argv[i + 1], 0, 10);
    if ((i = ArgPos("-format", argc, argv)) > 0) fmt = !strcmp(argv[i + 1], "go");
    order = order == 1 ? 1 : 2;

    Run run = open_run(device, gpus);
    smore_ctx* ctx = run.ctx;
    run_load(run, network_file, undirected, SMORE_VM_OUT_DEGREES, SMORE_NM_DEGREES);
    print_graph(ctx);
    printf("Model Setting:\n\tdimension:\t\t%d\n", dimensions);
    run_alloc(run, dimensions, order == 1 ? 1 : 2);
    SMORE_CLI_CHECK(ctx, smore_init_table_glibc(ctx, SMORE_W, 0));
    run_replicate(run);
    printf("Model:\n\t[LINE]\nLearning Parameters:\n\torder:\t\t\t%d%s\n", order, order == 1 ? "st" : "nd");
    printf("\tsample_times:\t\t%d\n\tnegative_samples:\t%d\n\talpha:\t\t\t%g\n\tworkers:\t\t%d\n", sample_times,
           negative_samples, init_alpha, threads);
    printf("Start Training:\n");
    const unsigned long long total = (unsigned long long)sample_times * 1000000ull;
    // one worker runs counts 1 .. total-1 (src/model/LINE.cpp:166-170)
    train_chunks(run, order == 1 ? SMORE_LINE1 : SMORE_LINE2, total, total ? total - 1 : 0, negative_samples,
                 init_alpha, 0.0, seed, mode);
    save(ctx, rep_file, fmt);
    run_close(run);
    return 0;
}
