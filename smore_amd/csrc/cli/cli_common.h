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

#define SMORE_CLI_CHECK(ctx, expr)                                                    \
    do {                                                                              \
        int rc_ = (expr);                                                             \
        if (rc_ != SMORE_OK) {                                                        \
            fprintf(stderr, "%s failed (%d): %s\n", #expr, rc_, smore_last_error(ctx)); \
            exit(2);                                                                  \
        }                                                                             \
    } while (0)
