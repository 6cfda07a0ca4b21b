//go:build !smore_hip

package bpr

const hipEnabled = false

func (b *BPR) trainHIP(sampleTimes int, alpha, lambda float64, workers int) {}
