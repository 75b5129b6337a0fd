//go:build !gpu

// scan_cpu.go -- the miner's search without the gpu build tag: the
// reference's own loop (bitcoin/miner/miner.go:58-65 over bitcoin.Hash,
// hash.go:11-15) behind the same scan() signature as gpu.go, with the
// inclusive bounds of README:329 (the reference loop stops at i < Upper) and
// no wrap at upper = 2^64-1.

package main

import "github.com/minhtrangvy/distributed_bitcoin_miner/project2/bitcoin"

func scan(data string, lower, upper uint64) (uint64, uint64, error) {
	bestHash, bestNonce := uint64(maxUint64), uint64(maxUint64)
	if lower > upper {
		return bestHash, bestNonce, nil
	}
	for n := lower; ; n++ {
		if h := bitcoin.Hash(data, n); h < bestHash { // strict '<': ties keep the smaller nonce
			bestHash, bestNonce = h, n
		}
		if n == upper {
			return bestHash, bestNonce, nil
		}
	}
}
