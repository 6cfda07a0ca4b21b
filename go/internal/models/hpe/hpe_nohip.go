//go:build !smore_hip

package hpe

const hipEnabled = false

func (h *HPE) trainHIP(sampleTimes, negativeSamples int, alpha float64, workers int) {}
