"""RCCL failure detection (smore_amd/csrc/comm_watch.h) with a
fake RCCL table, on the CPU: an asynchronous communicator error, a stuck
peer (deadline) and a failed stream each end the wait with a failure and
abort every communicator once, and the teardown that follows destroys none
of the aborted (freed) handles; a completing wait (also through RCCL's
ncclInProgress state) aborts nothing and the teardown destroys every one.
The library's group_sync and smore_synchronize (own communicator) wait
through this function."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

SRC = os.path.join(ROOT, "tests", "c", "comm_watch_test.cpp")


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("cw") / "comm_watch_test")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-o", exe, SRC,
                    "-pthread"], check=True)
    return exe


def _run(prog, scenario):
    out = subprocess.run([prog, scenario], check=True, capture_output=True, text=True, timeout=30).stdout.split(" ", 4)
    rc, aborts, destroys = int(out[1]), int(out[2]), int(out[3])
    assert destroys == 2 - aborts   # no aborted communicator is destroyed again
    return rc, aborts, out[4].strip()


def test_async_error_aborts(prog):
    rc, aborts, why = _run(prog, "async")
    assert rc == -1 and aborts == 2 and "remote process exited" in why and "communicator 0" in why


def test_stuck_peer_times_out(prog):
    rc, aborts, why = _run(prog, "stuck")
    assert rc == -1 and aborts == 2 and "not complete after" in why


def test_failed_stream_aborts(prog):
    rc, aborts, why = _run(prog, "stream")
    assert rc == -1 and aborts == 2 and "stream" in why


@pytest.mark.parametrize("scenario", ["ok", "inprog"])
def test_completion_aborts_nothing(prog, scenario):
    rc, aborts, why = _run(prog, scenario)
    assert rc == 0 and aborts == 0 and why == ""
