//go:build smore_hip

package node2vec

import (
	"fmt"
	"math/rand"
	"os"
	"time"

	"github.com/cnclabs/smore/pkg/pronet"
)

const hipEnabled = true

// trainHIP is (*Node2Vec).Train (internal/models/node2vec/node2vec.go:178-258)
// on MI355X GPUs: the start order is shuffled here as Train does it, then the
// biased walks (p, q), fixed-window SkipGrams and UpdatePairs run on the GPU
// with the Go learning-rate schedule over walkTimes * MaxVid walks.
func (n2v *Node2Vec) trainHIP(walkTimes, walkSteps, windowSize, negativeSamples int, alpha float64, workers int) {
	V := n2v.pnet.MaxVid
	order := make([]int64, 0, int64(walkTimes)*V)
	for t := 0; t < walkTimes; t++ {
		keys := make([]int64, V)
		for vid := int64(0); vid < V; vid++ {
			keys[vid] = vid
		}
		for vid := int64(0); vid < V; vid++ {
			j := vid + rand.Int63n(V-vid)
			keys[vid], keys[j] = keys[j], keys[vid]
		}
		order = append(order, keys...)
	}
	cfg := pronet.HIPConfigFromEnv(uint64(time.Now().UnixNano()))
	h, err := n2v.pnet.NewHIP(cfg)
	if err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	defer h.Close()
	total := uint64(len(order))
	report := func(done uint64) {
		fmt.Printf("\tProgress: %.3f %%\r", float64(done)/float64(total)*100)
	}
	if err := h.TrainNode2Vec(n2v.wVertex, n2v.wContext, n2v.dim, order, walkTimes, walkSteps, windowSize,
		negativeSamples, alpha, n2v.p, n2v.q, report); err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	fmt.Printf("\tAlpha: %.6f\tProgress: 100.00 %%\n", alpha*0.0001)
}
