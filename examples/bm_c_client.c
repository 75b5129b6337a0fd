/*
 * bm_c_client.c -- a plain C consumer of libbtcminer.so, using nothing but
 * include/btcminer.h: what the Go miner's cgo shim does,
 * minus Go.  Built with gcc against the in-tree library:
 *
 *   gcc -O2 -Iinclude examples/bm_c_client.c -Ldistributed_bitcoin_minter_amd -lbtcminer \
 *       -Wl,-rpath,'$ORIGIN/../distributed_bitcoin_minter_amd' -o examples/bm_c_client
 *
 * Usage: bm_c_client <msg> <lower> <upper> [num_gpus]
 * Prints "Result <hash> <nonce>" (the client's format, README:395-401), or
 * "error <status> <bm_strerror>" and exits 2 -- e.g. BM_ENODEV on a host
 * without a gfx950 GPU, since the library has no CPU fallback.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "btcminer.h"

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
    const uint64_t lower = strtoull(argv[2], NULL, 10);
    const uint64_t upper = strtoull(argv[3], NULL, 10);
    const int ngpu = argc > 4 ? atoi(argv[4]) : 1;
    if (bm_abi_version() != BM_ABI_VERSION) {
        printf("error abi %d != %d\n", bm_abi_version(), BM_ABI_VERSION);
        return 2;
    }
    bm_ctx_t* ctx = NULL;
    int rc = bm_ctx_create(ngpu, &ctx);
    if (rc != BM_OK) return fail(rc);
    bm_result_t r;
    rc = bm_search_gpu(ctx, (const uint8_t*)msg, strlen(msg), lower, upper, &r);
    if (rc != BM_OK) {
        bm_ctx_destroy(ctx);
        return fail(rc);
    }
    /* bitcoin.Hash for the winning nonce must give the winning hash back */
    uint64_t h = 0;
    rc = bm_hash_gpu(ctx, (const uint8_t*)msg, strlen(msg), &r.nonce, 1, &h);
    bm_ctx_destroy(ctx);
    if (rc != BM_OK) return fail(rc);
    if (h != r.hash && !(r.hash == UINT64_MAX && r.nonce == UINT64_MAX)) {
        printf("error rehash %" PRIu64 " != %" PRIu64 "\n", h, r.hash);
        return 2;
    }
    printf("Result %" PRIu64 " %" PRIu64 "\n", r.hash, r.nonce);
    return 0;
}
