// The RCCL failure watch (smore_amd/csrc/comm_watch.h) against a FAKE RCCL
// table: no GPU, no RCCL.  Each scenario prints "name status abort_calls why".
//   async   the communicator reports an asynchronous error after 5 polls
//   stuck   never completes, no error: the deadline (0.2 s) ends the wait
//   stream  the stream reports a failure
//   ok      completes after 5 polls: no abort
//   inprog  RCCL says ncclInProgress (not an error) until completion
#include <cstdio>
#include <cstring>

#include "../../smore_amd/csrc/comm_watch.h"

using smore_host::Rccl;

static int g_polls = 0, g_aborts = 0, g_destroys = 0, g_bad_destroys = 0;
static ncclComm_t g_aborted[2];
static ncclResult_t g_async = ncclSuccess;
static int g_async_after = 1 << 30;

static ncclResult_t fake_async(ncclComm_t, ncclResult_t* r) {
    *r = g_polls >= g_async_after ? g_async : ncclSuccess;
    return ncclSuccess;
}
static ncclResult_t fake_abort(ncclComm_t c) {
    g_aborted[g_aborts++ % 2] = c;
    return ncclSuccess;
}
static ncclResult_t fake_destroy(ncclComm_t c) {
    ++g_destroys;
    for (int i = 0; i < g_aborts && i < 2; ++i)
        if (g_aborted[i] == c) ++g_bad_destroys;   // a use after free in the real library
    return ncclSuccess;
}
static const char* fake_string(ncclResult_t r) { return r == ncclRemoteError ? "remote process exited" : "fake"; }

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    Rccl L;
    L.async_error = fake_async;
    L.abort = fake_abort;
    L.destroy = fake_destroy;
    L.error_string = fake_string;
    ncclComm_t comms[2] = {reinterpret_cast<ncclComm_t>(0x10), reinterpret_cast<ncclComm_t>(0x20)};
    const char* s = argv[1];
    int ready_after = 1 << 30, stream_fail = 0;
    if (!strcmp(s, "async")) { g_async = ncclRemoteError; g_async_after = 5; }
    else if (!strcmp(s, "ok")) ready_after = 5;
    else if (!strcmp(s, "stream")) stream_fail = 3;
    else if (!strcmp(s, "inprog")) { g_async = ncclInProgress; g_async_after = 0; ready_after = 7; }
    std::string why;
    auto ready = [&]() -> int {
        ++g_polls;
        if (stream_fail && g_polls >= stream_fail) return -1;
        return g_polls >= ready_after ? 1 : 0;
    };
    const int rc = smore_host::comm_watch(&L, comms, 2, ready, 0.2, why);
    smore_host::comm_release(&L, comms, 2);
    if (g_bad_destroys) {
        printf("%s destroyed-after-abort %d\n", s, g_bad_destroys);
        return 1;
    }
    printf("%s %d %d %d %s\n", s, rc, g_aborts, g_destroys, why.c_str());
    return 0;
}
