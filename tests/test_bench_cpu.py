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
