//go:build !smore_hip

package metapath2vec

const hipEnabled = false

func (mp *Metapath2Vec) trainHIP(walkTimes, walkSteps, windowSize, negativeSamples int, alpha float64, workers int) {
}
