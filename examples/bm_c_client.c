/*
 * bm_c_client.c -- a plain C consumer of libbtcminer.so: the calls the Go
 * miner's cgo shim (go/bitcoin/miner/gpu.go) makes, in the same order and
 * under the same preamble, minus Go (this image has no Go toolchain).
 * tests/test_abi.py extracts the preamble and the #cgo flags from gpu.go,
 * checks the block below matches it line for line, and builds this file with
 * exactly those flags.  __graft_entry__.build() also builds it in-tree:
 *
 *   gcc -O2 -Iinclude examples/bm_c_client.c -Ldistributed_bitcoin_minter_amd -lbtcminer \
 *       -Wl,-rpath,'$ORIGIN/../distributed_bitcoin_minter_amd' -o examples/bm_c_client
 *
 * Usage: bm_c_client <msg> <lower> <upper> [num_gpus (default 0: every visible GPU, as gpu.go)]
 * Prints "Result <hash> <nonce>" (the client's format, README:395-401), or
 * "error <status> <bm_strerror>" and exits 2 -- e.g. BM_ENODEV on a host
 * without a gfx950 GPU, since the library has no CPU fallback.
 */
/* ---- cgo preamble of go/bitcoin/miner/gpu.go (verbatim) ---- */
#include <stdlib.h>
#include "btcminer.h"
/* ---- end of the cgo preamble ---- */
#include <inttypes.h>
#include <stdio.h>
#include <string.h>

static int fail(int rc) {
    printf("error %d %s\n", rc, bm_strerror(rc));
    return 2;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <msg> <lower> <upper> [num_gpus]\n", argv[0]);
        return 1;
    }
    const char* msg = argv[1];
    const size_t len = strlen(msg);
    const uint64_t lower = strtoull(argv[2], NULL, 10);
    const uint64_t upper = strtoull(argv[3], NULL, 10);
    const int ngpu = argc > 4 ? atoi(argv[4]) : 0;
    if (bm_abi_version() != BM_ABI_VERSION) {
        printf("error abi %d != %d\n", bm_abi_version(), BM_ABI_VERSION);
        return 2;
    }
    /* newGPUMiner: every visible GPU, balanced pieces when there are several */
    bm_ctx_t* ctx = NULL;
    int rc = bm_ctx_create(ngpu, &ctx);
    if (rc != BM_OK) return fail(rc);
    int n = 0;
    if (bm_ctx_num_devices(ctx, &n) == BM_OK && n > 1) bm_ctx_set_balance(ctx, 1);
    /* gpuMiner.search: the message bytes in C memory (C.CBytes), one call */
    uint8_t* cs = NULL;
    if (len > 0) {
        cs = (uint8_t*)malloc(len);
        if (!cs) return fail(BM_ENOMEM);
        memcpy(cs, msg, len);
    }
    bm_result_t r;
    rc = bm_search_gpu(ctx, cs, len, lower, upper, &r);
    free(cs);
    if (rc != BM_OK) {
        bm_ctx_destroy(ctx);
        return fail(rc);
    }
    /* not in gpu.go: bitcoin.Hash for the winning nonce must give the winning hash back */
    uint64_t h = 0;
    rc = bm_hash_gpu(ctx, (const uint8_t*)msg, len, &r.nonce, 1, &h);
    /* gpuMiner.close */
    bm_ctx_destroy(ctx);
    if (rc != BM_OK) return fail(rc);
    if (h != r.hash && !(r.hash == UINT64_MAX && r.nonce == UINT64_MAX)) {
        printf("error rehash %" PRIu64 " != %" PRIu64 "\n", h, r.hash);
        return 2;
    }
    printf("Result %" PRIu64 " %" PRIu64 "\n", r.hash, r.nonce);
    return 0;
}
