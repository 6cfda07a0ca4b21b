//go:build !smore_hip

package ctdne

const hipEnabled = false

func (ctdne *CTDNE) trainHIP(walkTimes, walkSteps, windowSize, negativeSamples int, alpha float64, workers int) {}
