import sys, json, time, numpy as np
sys.path.insert(0, "/root/repo")
import smore_amd
from smore_amd import graphgen
sys.path.insert(0, "/root/repo/tools")
from replica_study import heldout_loss
cfg = sys.argv[1]; T = 1 << int(sys.argv[2])
V, (src, dst, w) = graphgen.config_edges(cfg)
pn = smore_amd.ProNet(0)
pn.set_graph_edges(V, src, dst, w)
held = pn.sample_edges("line2", (1 << 40) + 17, 100_000, 5, 20251015 + 1)
pn.alloc_tables(64, 2)
for chunk in [int(x) for x in sys.argv[3:]]:
    pn.init_table_glibc(0, 0); pn.zero_table(1)
    t0 = time.perf_counter()
    for b in range(0, T, chunk):
        pn.train_edges("line2", b, min(chunk, T - b), T, 5, 0.025, 0.0, 20251015, "hybrid", sync=False)
    pn.synchronize()
    print(json.dumps({"config": cfg, "total": T, "launch": chunk, "loss": round(heldout_loss(pn.get_table(0), pn.get_table(1), held), 5), "s": round(time.perf_counter() - t0, 2)}), flush=True)
