//go:build smore_hip

package line

import (
	"fmt"
	"os"
	"time"

	"github.com/cnclabs/smore/pkg/pronet"
)

const hipEnabled = true

// trainHIP is (*LINE).Train's sample loop (internal/models/line/line.go:87-146)
// on MI355X GPUs: total = sampleTimes * MaxLine samples, Go learning-rate
// schedule, order 2 -> UpdatePair(wVertex, wContext), order 1 ->
// updateFirstOrder(wVertex).  GPUs and scatter mode: SMORE_HIP_DEVICE,
// SMORE_HIP_GPUS, SMORE_HIP_MODE, SMORE_HIP_SEED (pkg/pronet/hip.go).
func (l *LINE) trainHIP(sampleTimes, negativeSamples int, alpha float64, workers int) {
	cfg := pronet.HIPConfigFromEnv(uint64(time.Now().UnixNano()))
	h, err := l.pnet.NewHIP(cfg)
	if err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	defer h.Close()
	total := uint64(sampleTimes) * uint64(l.pnet.MaxLine)
	model := pronet.HIPLine2
	if l.order == First {
		model = pronet.HIPLine1
	}
	report := func(done uint64) {
		a := alpha * (1.0 - float64(done/pronet.Monitor*pronet.Monitor)/float64(total))
		if a < alpha*0.0001 {
			a = alpha * 0.0001
		}
		fmt.Printf("\tAlpha: %.6f\tProgress: %.3f %%\r", a, float64(done)/float64(total)*100)
	}
	if err := h.TrainEdges(model, l.wVertex, l.wContext, l.dim, total, negativeSamples, alpha, 0, report); err != nil {
		fmt.Fprintln(os.Stderr, "smore_hip:", err)
		os.Exit(1)
	}
	fmt.Printf("\tAlpha: %.6f\tProgress: 100.00 %%\n", alpha*0.0001)
}
