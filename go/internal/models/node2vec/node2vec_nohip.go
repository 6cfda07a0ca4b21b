//go:build !smore_hip

package node2vec

const hipEnabled = false

func (n2v *Node2Vec) trainHIP(walkTimes, walkSteps, windowSize, negativeSamples int, alpha float64, workers int) {}
