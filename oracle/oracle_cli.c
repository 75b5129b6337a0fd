/*
 * oracle_cli -- command-line front end of the CPU oracle (test infra only).
 *   oracle_cli hash   <msg-hex> <nonce>
 *   oracle_cli search <msg-hex> <lower> <upper> [threads] [openssl:0|1]
 *   oracle_cli search16 <msg-hex> <lower> <upper> [threads]   (AVX-512, bm_scan16.c)
 * Prints "<hash> <nonce>" (decimal), the same pair the reference client
 * prints as "Result <hash> <nonce>" (bitcoin/client/client.go:76-78).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bm_oracle.h"

static size_t unhex(const char* s, uint8_t* out, size_t cap) {
    size_t n = strlen(s) / 2;
    if (n > cap) return (size_t)-1;
    for (size_t i = 0; i < n; ++i) {
        unsigned v;
        if (sscanf(s + 2 * i, "%2x", &v) != 1) return (size_t)-1;
        out[i] = (uint8_t)v;
    }
    return n;
}

int main(int argc, char** argv) {
    static uint8_t msg[1 << 16];
    if (argc < 4) {
        fprintf(stderr, "usage: %s hash <msg-hex> <nonce> | search <msg-hex> <lo> <hi> [threads] [openssl]\n",
                argv[0]);
        return 2;
    }
    size_t len = unhex(argv[2], msg, sizeof msg);
    if (len == (size_t)-1) return 2;
    if (!strcmp(argv[1], "hash")) {
        printf("%llu\n", (unsigned long long)oracle_hash(msg, len, strtoull(argv[3], NULL, 10)));
        return 0;
    }
    if (!strcmp(argv[1], "search") && argc >= 5) {
        uint64_t lo = strtoull(argv[3], NULL, 10), hi = strtoull(argv[4], NULL, 10), h, n;
        int th = argc > 5 ? atoi(argv[5]) : 1, ossl = argc > 6 ? atoi(argv[6]) : 0;
        if (oracle_search_mt(msg, len, lo, hi, th, ossl, &h, &n)) return 1;
        printf("%llu %llu\n", (unsigned long long)h, (unsigned long long)n);
        return 0;
    }
    if (!strcmp(argv[1], "search16") && argc >= 5) {
        uint64_t lo = strtoull(argv[3], NULL, 10), hi = strtoull(argv[4], NULL, 10), h, n;
        int th = argc > 5 ? atoi(argv[5]) : 1;
        if (oracle_search_x16(msg, len, lo, hi, th, &h, &n)) return 1;
        printf("%llu %llu\n", (unsigned long long)h, (unsigned long long)n);
        return 0;
    }
    return 2;
}
