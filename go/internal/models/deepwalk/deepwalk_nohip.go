//go:build !smore_hip

package deepwalk

const hipEnabled = false

func (dw *DeepWalk) trainHIP(walkTimes, walkSteps, windowSize, negativeSamples int, alpha float64, workers int) {}
