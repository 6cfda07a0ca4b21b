"""bench.py host logic without a GPU: the live-PMC CSV reduction against the
committed round-3 rocprofv3 passes of the same config (profiles/r03), which
profiles/pmc_traffic.json summarised with tools/pmc_summary.py."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_pmc_per_launch_matches_committed_summary():
    prof = os.path.join(ROOT, "profiles", "r03")
    f = bench.pmc_per_launch(os.path.join(prof, "c4_hybrid_pmc_fetch.csv"), "FETCH_SIZE")
    w = bench.pmc_per_launch(os.path.join(prof, "c4_hybrid_pmc_write.csv"), "WRITE_SIZE")
    ref = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    for k in bench.PMC_KERNELS:
        assert abs(f[k] + w[k] - ref["kernels"][k]["hbm_bytes_per_launch"]) <= 1e-6 * ref["kernels"][k]["hbm_bytes_per_launch"]
    assert abs(sum(f.values()) + sum(w.values()) - ref["hbm_bytes_per_step"]) <= 1e-6 * ref["hbm_bytes_per_step"]


def test_pmc_per_launch_ignores_other_counters(tmp_path):
    p = tmp_path / "c.csv"
    p.write_text('"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n'
                 '1,"void smore::draw_kernel<5, 0>(x)","FETCH_SIZE",10\n'
                 '1,"void smore::draw_kernel<5, 0>(x)","FETCH_SIZE",6\n'
                 '2,"void smore::draw_kernel<5, 0>(x)","FETCH_SIZE",12\n'
                 '3,"void smore::draw_kernel<5, 0>(x)","WRITE_SIZE",99\n'
                 '4,"other","FETCH_SIZE",1000\n')
    got = bench.pmc_per_launch(str(p), "FETCH_SIZE")
    assert list(got) == ["draw_kernel"]
    assert got["draw_kernel"] == (16 + 12) / 2 * 1024 * bench.FETCH_CORRECTION


def test_samples_to_loss_interpolation(tmp_path):
    """tools/samples_to_loss.py: the N-replica total that reaches one
    replica's loss, by log-linear interpolation, and the effective speed-up
    N x sample efficiency x exchange time efficiency."""
    import json
    import subprocess
    import sys
    rows = [{"ranks": 1, "c0": 1.0, "period": 1.0, "log2_total": t, "loss": l} for t, l in ((29, 3.0), (30, 2.0))]
    rows += [{"ranks": 4, "c0": 1.0, "period": 0.5, "log2_total": t, "loss": l}
             for t, l in ((29, 4.0), (30, 3.0), (31, 2.0))]
    p = tmp_path / "s.jsonl"
    p.write_text("".join(json.dumps(r) + "\n" for r in rows))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "samples_to_loss.py"), str(p),
                          "--step-ms", "100", "--exchange-ms", "5"], capture_output=True, text=True, check=True)
    got = {r["target_log2_total"]: r for r in map(json.loads, out.stdout.split("\n")[:-1])}
    # one replica reaches 3.0 at 2^29 and 2.0 at 2^30; four do at 2^30 and 2^31
    assert got[29]["n_ranks_log2_total"] == 30.0 and got[29]["sample_eff"] == 0.5
    assert got[30]["n_ranks_log2_total"] == 31.0
    assert abs(got[29]["time_eff"] - 100 / 110) < 1e-3
    assert abs(got[29]["effective_speedup"] - 4 * 0.5 * 100 / 110) < 0.01


def test_gpus_flag_must_match_launcher_world(monkeypatch):
    """--gpus N under a launcher whose WORLD_SIZE differs exits non-zero
    before anything touches the GPU."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "--gpus 1 but WORLD_SIZE=2" in p.stderr
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "--gpus 8 but WORLD_SIZE=2" in p.stderr


def test_gpus_flag_without_launcher_starts_ranks(monkeypatch):
    """--gpus N > 1 with no WORLD_SIZE: bench.py must start N ranks itself
    (world_from_env -> None) and pass its own arguments to them."""
    import types
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.world_from_env(types.SimpleNamespace(gpus=1)) == 1
    assert bench.world_from_env(types.SimpleNamespace(gpus=4)) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.world_from_env(types.SimpleNamespace(gpus=4)) == 4
    seen = {}

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return types.SimpleNamespace(returncode=3)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    assert bench.launch_ranks(types.SimpleNamespace(gpus=4)) == 3
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4" and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
