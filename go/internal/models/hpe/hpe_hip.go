//go:build smore_hip

package hpe

import (
	"fmt"
	"os"
	"time"

	"github.com/cnclabs/smore/pkg/pronet"
)

const hipEnabled = true

// trainHIP is (*HPE).Train's sample loop (internal/models/hpe/hpe.go:72-124)
// on MI355X GPUs.  The Go HPE loop is SourceSample -> TargetSample ->
// UpdatePair(wVertex, wContext) over sampleTimes * MaxLine samples with the
// Go learning-rate schedule -- the Go LINE-2 edge rule, so it runs on
// HIPLine2 (pkg/pronet/hip.go TrainEdges).  GPUs and scatter mode:
// SMORE_HIP_DEVICE, SMORE_HIP_GPUS, SMORE_HIP_MODE, SMORE_HIP_SEED.
func (h *HPE) trainHIP(sampleTimes, negativeSamples int, alpha float64, workers int) {
	cfg := pronet.HIPConfigFromEnv(uint64(time.Now().UnixNano()))
	g, err := h.pnet.NewHIP(cfg)
	if err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	defer g.Close()
	total := uint64(sampleTimes) * uint64(h.pnet.MaxLine)
	report := func(done uint64) {
		a := alpha * (1.0 - float64(done/pronet.Monitor*pronet.Monitor)/float64(total))
		if a < alpha*0.0001 {
			a = alpha * 0.0001
		}
		fmt.Printf("\tAlpha: %.6f\tProgress: %.3f %%\r", a, float64(done)/float64(total)*100)
	}
	if err := g.TrainEdges(pronet.HIPLine2, h.wVertex, h.wContext, h.dim, total, negativeSamples, alpha, 0,
		report); err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	fmt.Printf("\tAlpha: %.6f\tProgress: 100.00 %%\n", alpha*0.0001)
}
