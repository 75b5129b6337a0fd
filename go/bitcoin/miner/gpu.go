//go:build gpu

// gpu.go -- the GPU backend of the reference miner's search loop, bound to
// libbtcminer.so through cgo (include/btcminer.h).
//
// It replaces bitcoin/miner/miner.go:58-65 of the reference
// (/root/reference/project2; that loop calls bitcoin.Hash, hash.go:11-15, once
// per nonce and keeps a strict-'<' minimum).  Drop this file and scan_cpu.go
// into project2/bitcoin/miner/, apply miner_go.patch, and check this
// repository out as btcminer/ next to project2/ (the #cgo paths below are
// relative to this file there).  `go build -tags gpu` then links the GPU
// library; a build without the tag keeps the reference's own loop
// (scan_cpu.go).  examples/bm_c_client.c makes the same calls from C, with
// the same preamble, and is what the tests compile (this image has no Go).

package main

/*
#cgo CFLAGS: -I${SRCDIR}/../../../btcminer/include
#cgo LDFLAGS: -L${SRCDIR}/../../../btcminer/distributed_bitcoin_minter_amd -lbtcminer -Wl,-rpath,${SRCDIR}/../../../btcminer/distributed_bitcoin_minter_amd
#include <stdlib.h>
#include "btcminer.h"
*/
import "C"

import (
	"errors"
	"runtime"
	"unsafe"
)

// gpuMiner owns one context over every visible GPU: one process driving up
// to 8 MI355X, whose per-GPU partials the library combines with one RCCL
// allgather (host copies if RCCL fails at run time).
type gpuMiner struct{ ctx *C.bm_ctx_t }

var theGPU *gpuMiner

func bmError(rc C.int) error { return errors.New(C.GoString(C.bm_strerror(rc))) }

func newGPUMiner() (*gpuMiner, error) {
	// the HIP device is per OS thread: keep this goroutine's calls on one
	runtime.LockOSThread()
	var ctx *C.bm_ctx_t
	if rc := C.bm_ctx_create(0, &ctx); rc != C.BM_OK {
		return nil, bmError(rc)
	}
	var n C.int
	if rc := C.bm_ctx_num_devices(ctx, &n); rc == C.BM_OK && n > 1 {
		C.bm_ctx_set_balance(ctx, 1) // pieces follow each GPU's measured rate
	}
	return &gpuMiner{ctx: ctx}, nil
}

// search returns min over n in [lower, upper] of (bitcoin.Hash(data, n), n),
// ties to the smallest n: bit-exact with the loop it replaces.  Bounds are
// inclusive (README:329); lower > upper gives (2^64-1, 2^64-1), as
// miner.go:45-46 does when its loop runs zero times.
func (g *gpuMiner) search(data string, lower, upper uint64) (uint64, uint64, error) {
	var out C.bm_result_t
	var p *C.uint8_t
	if len(data) > 0 {
		cs := C.CBytes([]byte(data)) // Go's %s: the string's raw bytes, copied by the library
		defer C.free(cs)
		p = (*C.uint8_t)(unsafe.Pointer(cs))
	}
	rc := C.bm_search_gpu(g.ctx, p, C.size_t(len(data)), C.uint64_t(lower), C.uint64_t(upper), &out)
	if rc != C.BM_OK {
		return 0, 0, bmError(rc)
	}
	return uint64(out.hash), uint64(out.nonce), nil
}

func (g *gpuMiner) close() { C.bm_ctx_destroy(g.ctx) }

// scan is what miner.go's job loop calls (miner_go.patch).  The context is
// opened on the first job and kept for the life of the process; an error
// (no gfx950 GPU: BM_ENODEV -- there is no CPU fallback in the library)
// makes the miner leave, so the server reassigns the job (README:413).
func scan(data string, lower, upper uint64) (uint64, uint64, error) {
	if theGPU == nil {
		g, err := newGPUMiner()
		if err != nil {
			return 0, 0, err
		}
		theGPU = g
	}
	return theGPU.search(data, lower, upper)
}
