"""Writes tests/golden/hetero.txt: a synthetic heterogeneous edge list in the
pkg/hetero format ("src srcType dst dstType edgeType [weight]",
hetero_graph.go:60-110) -- users buy items, items belong to categories, some
item-item links, one user linked only to a category.  Seeded."""
import numpy as np

rng = np.random.default_rng(11)
lines = []
U, I, Cc = 60, 40, 6
cat = rng.integers(0, Cc, I)
for u in range(U):
    for i in rng.choice(I, size=rng.integers(1, 6), replace=False):
        lines.append(f"u{u} User i{i} Item buy {1 + rng.integers(0, 3)}")
for i in range(I):
    lines.append(f"i{i} Item c{cat[i]} Category in")
for _ in range(15):
    a, b = rng.integers(0, I, 2)
    lines.append(f"i{a} Item i{b} Item sim")
lines.append("u999 User c0 Category likes")
rng.shuffle(lines)
open("tests/golden/hetero.txt", "w").write("\n".join(lines) + "\n")
