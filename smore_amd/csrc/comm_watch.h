// comm_watch.h -- RCCL failure detection of the multi-GPU paths (SURVEY.md 5
// "failure detection: RCCL ncclCommGetAsyncError polling").
//
// The reference has no failure path at all (one process, shared memory;
// src/proNet.cpp:143 even ignores a failed fopen).  Here a host wait on work
// that depends on a collective -- a group call's final synchronisation, or
// smore_synchronize on a context with its own communicator -- must not hang
// forever on a dead or stuck peer.  comm_watch polls the work's completion;
// between polls it asks RCCL for the communicator's asynchronous error
// (ncclCommGetAsyncError) and bounds the total wait.  On an error, a failed
// stream or the deadline it aborts the communicator (ncclCommAbort: the
// in-flight collective kernels return, so the GPU is left usable for a
// clean exit) and reports why; the caller returns SMORE_EHIP.  No in-process
// restart: a multi-GPU run that lost a peer exits non-zero.
//
// Internal; the RCCL entry points come from the dlopen'ed table (Rccl) so
// tests can hand in a fake one (tests/c/comm_watch_test.cpp).
#pragma once
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <string>
#include <thread>

namespace smore_host {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string err;
};

// the wait bound (seconds): $SMORE_COMM_TIMEOUT, else 1800 -- long enough for
// any queued training call, short enough that a stuck peer ends the job
inline double comm_timeout_default() {
    const char* e = getenv("SMORE_COMM_TIMEOUT");
    const double t = e ? atof(e) : 0.0;
    return t > 0.0 ? t : 1800.0;
}

// Wait until ready() returns 1 (0: not yet, < 0: the stream failed).  Between
// polls: every communicator in comms[0 .. n) is asked for its asynchronous
// error.  Returns 0, or -1 with `why` set after aborting every communicator.
// ncclCommAbort frees a communicator, so an aborted handle is set to null
// here: the caller's teardown (comm_release) must not destroy it again.
template <class Ready>
int comm_watch(const Rccl* L, ncclComm_t* comms, int n, Ready&& ready, double timeout_s, std::string& why) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto abort_all = [&] {
        for (int i = 0; L && L->abort && i < n; ++i)
            if (comms[i]) {
                (void)L->abort(comms[i]);
                comms[i] = nullptr;
            }
    };
    for (long poll = 0;; ++poll) {
        const int r = ready();
        if (r > 0) return 0;
        if (r < 0) {
            why = "a stream waiting on a collective failed";
            abort_all();
            return -1;
        }
        for (int i = 0; L && L->async_error && i < n; ++i) {
            if (!comms[i]) continue;
            ncclResult_t a = ncclSuccess;
            const ncclResult_t q = L->async_error(comms[i], &a);
            if (q != ncclSuccess || (a != ncclSuccess && a != ncclInProgress)) {
                const ncclResult_t bad = q != ncclSuccess ? q : a;
                why = std::string("RCCL asynchronous error on communicator ") + std::to_string(i) + ": " +
                      (L->error_string ? L->error_string(bad) : "unknown");
                abort_all();
                return -1;
            }
        }
        const double el = std::chrono::duration<double>(clk::now() - t0).count();
        if (el > timeout_s) {
            why = "collective not complete after " + std::to_string((long)timeout_s) +
                  " s (a stuck peer?); communicators aborted";
            abort_all();
            return -1;
        }
        if (poll < 200) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// teardown: destroy the communicators still held (an aborted one is null)
inline void comm_release(const Rccl* L, ncclComm_t* comms, int n) {
    for (int i = 0; i < n; ++i) {
        if (comms[i] && L && L->destroy) (void)L->destroy(comms[i]);
        comms[i] = nullptr;
    }
}

}  // namespace smore_host
