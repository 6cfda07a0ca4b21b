//go:build smore_hip

package ctdne

import (
	"fmt"
	"math/rand"
	"os"
	"time"

	"github.com/cnclabs/smore/pkg/pronet"
)

const hipEnabled = true

// trainHIP is (*CTDNE).Train (internal/models/ctdne/ctdne.go:80-200) on
// MI355X GPUs.  Go keeps pkg/temporal's loader; what it built is handed over
// once: tg.OutEdges of every node in vertex order (already sorted by
// timestamp by the loader's sort.Slice, so ties keep Go's own order), as the
// graph (unit weights) and as the temporal edges, and the negative table Train
// builds (BuildAliasMethod over node activity, :110-121).  The walk start
// order is shuffled here as Train does it; active-range start times, temporal
// walks, SkipGrams and UpdatePairs run on the GPU with the Go learning-rate
// schedule over walkTimes * NumNodes walks.
func (ctdne *CTDNE) trainHIP(walkTimes, walkSteps, windowSize, negativeSamples int, alpha float64, workers int) {
	tg := ctdne.tg
	V := tg.NumNodes
	var src, dst []int64
	var ones, ts []float64
	for v := int64(0); v < V; v++ {
		for _, e := range tg.OutEdges[v] {
			src, dst = append(src, v), append(dst, e.To)
			ones, ts = append(ones, 1.0), append(ts, e.Timestamp)
		}
	}
	negDistribution := make([]float64, V)
	for i := int64(0); i < V; i++ {
		if activity := tg.GetNodeActivity(i); activity > 0 {
			negDistribution[i] = float64(activity)
		} else {
			negDistribution[i] = 1.0
		}
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
	h, err := pronet.NewHIPEdges(V, src, dst, ones, negativeAT, cfg)
	if err == nil {
		defer h.Close()
		err = h.SetTemporalEdges(src, dst, ts)
	}
	if err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	total := uint64(len(order))
	report := func(done uint64) {
		fmt.Printf("\tProgress: %.3f %%\r", float64(done)/float64(total)*100)
	}
	if err := h.TrainCTDNE(ctdne.embeddings, ctdne.contextEmbeddings, ctdne.dim, order, walkTimes, walkSteps,
		windowSize, negativeSamples, alpha, ctdne.timeWindow, report); err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	fmt.Printf("\tAlpha: %.6f\tProgress: 100.00 %%\n", alpha*0.0001)
}
