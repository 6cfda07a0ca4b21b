"""Writes tests/golden/temporal.txt: a synthetic timestamped edge list in the
pkg/temporal format ("src dst timestamp", temporal_graph.go:60-130): 80
vertices, power-law-ish sources, distinct timestamps per source (Go's
sort.Slice is unstable, so equal timestamps of one source have no defined
order), one malformed timestamp and one short line (both skipped).  Seeded."""
import numpy as np

rng = np.random.default_rng(5)
N, E = 80, 600
src = (rng.zipf(1.6, E) - 1) % N
dst = rng.integers(0, N, E)
ts = rng.permutation(np.arange(E)) * 0.37 + rng.random(E) * 0.1   # distinct everywhere
lines = ["n%d n%d %.4f" % (a, b, t) for a, b, t in zip(src, dst, ts)]
lines.insert(17, "n3 n4 notatime")
lines.insert(40, "n5 n6")
open("tests/golden/temporal.txt", "w").write("\n".join(lines) + "\n")
