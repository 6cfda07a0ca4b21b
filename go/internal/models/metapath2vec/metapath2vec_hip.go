//go:build smore_hip

package metapath2vec

import (
	"fmt"
	"math/rand"
	"os"
	"time"

	"github.com/cnclabs/smore/pkg/pronet"
)

const hipEnabled = true

// trainHIP is (*Metapath2Vec).Train (internal/models/metapath2vec/
// metapath2vec.go:106-200) on MI355X GPUs.  Go keeps pkg/hetero's loader;
// what it built is handed over once: the adjacency of hg.Edges (with
// hg.EdgeWeights) in vertex order, every node's type id (hg.TypeHash of
// hg.NodeTypes), the meta-paths as type ids, and the negative table Train
// builds (BuildAliasMethod over ones, :140-145).  The walk start order is
// shuffled here as Train does it; walks, SkipGrams and UpdatePairs run on
// the GPU with the Go learning-rate schedule over walkTimes * NumNodes walks.
func (mp *Metapath2Vec) trainHIP(walkTimes, walkSteps, windowSize, negativeSamples int, alpha float64, workers int) {
	hg := mp.hg
	V := hg.NumNodes
	var src, dst []int64
	var wts []float64
	for v := int64(0); v < V; v++ {
		ws := hg.EdgeWeights[v]
		for i, t := range hg.Edges[v] {
			src, dst, wts = append(src, v), append(dst, t), append(wts, ws[i])
		}
	}
	types := make([]int64, V)
	for v := int64(0); v < V; v++ {
		types[v] = hg.TypeHash[hg.NodeTypes[v]]
	}
	paths := make([][]int64, len(mp.metaPaths))
	for i, p := range mp.metaPaths {
		for _, t := range p {
			paths[i] = append(paths[i], hg.TypeHash[t])
		}
	}
	negDistribution := make([]float64, V)
	for i := range negDistribution {
		negDistribution[i] = 1.0
	}
	negativeAT := pronet.BuildAliasMethod(negDistribution, 0.75)
	order := make([]int64, 0, int64(walkTimes)*V)
	for t := 0; t < walkTimes; t++ {
		keys := make([]int64, V)
		for i := int64(0); i < V; i++ {
			keys[i] = i
		}
		for i := int64(0); i < V; i++ {
			j := i + rand.Int63n(V-i)
			keys[i], keys[j] = keys[j], keys[i]
		}
		order = append(order, keys...)
	}
	cfg := pronet.HIPConfigFromEnv(uint64(time.Now().UnixNano()))
	h, err := pronet.NewHIPEdges(V, src, dst, wts, negativeAT, cfg)
	if err == nil {
		defer h.Close()
		err = h.SetNodeTypes(types, len(hg.TypeKeys))
	}
	if err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	total := uint64(len(order))
	report := func(done uint64) {
		fmt.Printf("\tProgress: %.3f %%\r", float64(done)/float64(total)*100)
	}
	if err := h.TrainMetapath2Vec(mp.embeddings, mp.contextEmbeddings, mp.dim, order, paths, walkTimes, walkSteps,
		windowSize, negativeSamples, alpha, report); err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	fmt.Printf("\tAlpha: %.6f\tProgress: 100.00 %%\n", alpha*0.0001)
}
