//go:build !smore_hip

package line

const hipEnabled = false

func (l *LINE) trainHIP(sampleTimes, negativeSamples int, alpha float64, workers int) {}
