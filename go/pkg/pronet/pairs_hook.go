package pronet

import "math/rand"

// pairs_hook.go -- the dispatch point of UpdatePairs (optimizer.go, patched by
// go/patches/train_dispatch.patch).  Nil in a plain build, so UpdatePairs runs
// its own CPU loop; hip.go (-tags smore_hip) sets it to the GPU batch
// (smore_train_pairs).  Copy this file into pkg/pronet with hip.go.
var hipUpdatePairs func(pn *ProNet, wVertex, wContext [][]float64, vertices, contexts []int64, dim,
	negativeSamples int, alpha float64, rng *rand.Rand)
