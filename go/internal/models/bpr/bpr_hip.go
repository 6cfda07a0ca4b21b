//go:build smore_hip

package bpr

import (
	"fmt"
	"os"
	"time"

	"github.com/cnclabs/smore/pkg/pronet"
)

const hipEnabled = true

// trainHIP is (*BPR).Train's sample loop (internal/models/bpr/bpr.go:82-130)
// on MI355X GPUs: total = sampleTimes * MaxLine samples of SourceSample ->
// TargetSample -> one NegativeSample -> UpdateBPRPair(wVertex users,
// wContext items, lambda) with the Go learning-rate schedule.
func (b *BPR) trainHIP(sampleTimes int, alpha, lambda float64, workers int) {
	cfg := pronet.HIPConfigFromEnv(uint64(time.Now().UnixNano()))
	h, err := b.pnet.NewHIP(cfg)
	if err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	defer h.Close()
	total := uint64(sampleTimes) * uint64(b.pnet.MaxLine)
	report := func(done uint64) {
		fmt.Printf("\tProgress: %.3f %%\r", float64(done)/float64(total)*100)
	}
	if err := h.TrainEdges(pronet.HIPBPR, b.wVertex, b.wContext, b.dim, total, 1, alpha, lambda, report); err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	fmt.Printf("\tAlpha: %.6f\tProgress: 100.00 %%\n", alpha*0.0001)
}
