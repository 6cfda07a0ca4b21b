// mf -- flag-compatible replacement of cli/mf.cpp (MF, UpdateFactorizedPair)
// on one MI355X.  Extra flags: -device, -mode hogwild|atomic|hybrid|serial,
// -seed, -format cpp|go.
#include "cli_common.h"

int main(int argc, char** argv) {
    int i;
    if (argc == 1) {
        printf("[smore-mi355x] MF\n\nOptions Description:\n");
        printf("\t-train <string>\n\t-save <string>\n\t-dimensions <int> (64)\n\t-negative_samples <int> (5)\n");
        printf("\t-sample_times <int> (10, x10^6)\n\t-alpha <float> (0.025)\n\t-reg <float> (0.01)\n\t-threads <int>\n");
        printf("\t-device <int> -gpus <int> -mode hogwild|atomic|hybrid|serial -seed <int> -format cpp|go\n");
        printf("Usage:\n./mf -train net.txt -save rep.txt -dimensions 64 -sample_times 10 -negative_samples 5 "
               "-alpha 0.025 -reg 0.01 -threads 1\n");
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
    if ((i = ArgPos("-alpha", argc, argv)) > 0) init_alpha = atof(argv[i + 1]);
    if ((i = ArgPos("-reg", argc, argv)) > 0) reg = atof(argv[i + 1]);
    if ((i = ArgPos("-threads", argc, argv)) > 0) threads = atoi(argv[i + 1]);
    if ((i = ArgPos("-device", argc, argv)) > 0) device = atoi(argv[i + 1]);
    if ((i = ArgPos("-gpus", argc, argv)) > 0) gpus = atoi(argv[i + 1]);
    if ((i = ArgPos("-mode", argc, argv)) > 0) mode = mode_of(argv[i + 1]);
    if ((i = ArgPos("-seed", argc, argv)) > 0) seed = strtoull(argv[i + 1], 0, 10);
    if ((i = ArgPos("-format", argc, argv)) > 0) fmt = !strcmp(argv[i + 1], "go");

    Run run = open_run(device, gpus);
    smore_ctx* ctx = run.ctx;
    // MF() sets negative_method "no_degrees" (src/model/MF.cpp:4-7); LoadEdgeList(file, 0)
    run_load(run, network_file, 0, SMORE_VM_OUT_DEGREES, SMORE_NM_NO_DEGREES);
    print_graph(ctx);
    printf("Model Setting:\n\tdimension:\t\t%d\n", dimensions);
    run_alloc(run, dimensions, 1);
    SMORE_CLI_CHECK(ctx, smore_init_table_glibc(ctx, SMORE_W, 0));
    run_replicate(run);
    printf("Model:\n\t[MF]\nLearning Parameters:\n\tsample_times:\t\t%d\n\tnegative_samples:\t%d\n"
           "\talpha:\t\t\t%g\n\tregularization:\t\t%g\n\tworkers:\t\t%d\nStart Training:\n",
           sample_times, negative_samples, init_alpha, reg, threads);
    const unsigned long long total = (unsigned long long)sample_times * 1000000ull;
    train_chunks(run, SMORE_MF, total, total, negative_samples, init_alpha, reg, seed, mode);
    save(ctx, rep_file, fmt);
    run_close(run);
    return 0;
}
