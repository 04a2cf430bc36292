/* host_bench.c -- the host entry points as a plain-C caller (what a cgo Serializer adapter is) would
 * use them: sym_encode_host + sym_decode_host on a bench-config-2-shaped batch (2^20 kv
 * SetRequests, 64-byte keys, 256-byte values, pseudo-random bytes) in pinned memory from
 * sym_host_alloc, after `warm` seconds of the same calls.  No torch in the process.
 *
 *   make -C tests bin/host_bench && tests/bin/host_bench [calls] [warm seconds]
 *
 * A torch process loads torch's own HIP runtime (torch/lib/libamdhip64.so), whose D2H copies run as
 * blit kernels that do not overlap the SDMA H2D copies; a Go (cgo) or C process linking
 * /opt/rocm's runtime gets SDMA both ways -- bench.py's host-inclusive leg runs this driver for
 * that reason (host entry points).
 */
#define _POSIX_C_SOURCE 199309L /* clock_gettime under -std=c11 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/symphony_hip.h"

#define DIE(what)                                                          \
    do {                                                                   \
        fprintf(stderr, "%s failed: %s\n", what, sym_last_error());        \
        exit(1);                                                           \
    } while (0)

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void* halloc(sym_ctx* ctx, uint64_t bytes) {
    void* p = NULL;
    if (sym_host_alloc(ctx, bytes, &p) != SYM_OK) DIE("sym_host_alloc");
    return p;
}

int main(int argc, char** argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 6;
    const double warm = argc > 2 ? atof(argv[2]) : 2.0;
    const uint64_t n = 1u << 20, K = 64, V = 256;
    sym_ctx* ctx = NULL;
    if (sym_ctx_create(0, &ctx) != SYM_OK) DIE("sym_ctx_create");
    uint8_t* kb = halloc(ctx, n * K);
    uint8_t* vb = halloc(ctx, n * V);
    uint64_t* ko = halloc(ctx, 8 * (n + 1));
    uint64_t* vo = halloc(ctx, 8 * (n + 1));
    uint64_t x = 0x5eed0001ull;
    for (uint64_t i = 0; i < n * K; i += 8) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        memcpy(kb + i, &x, 8);
    }
    for (uint64_t i = 0; i < n * V; i += 8) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        memcpy(vb + i, &x, 8);
    }
    for (uint64_t i = 0; i <= n; ++i) {
        ko[i] = i * K;
        vo[i] = i * V;
    }
    const uint64_t total = n * (sym_record_overhead(SYM_SCHEMA_KV_SET_REQUEST) + K + V);
    uint8_t* out = halloc(ctx, total + 16);
    uint64_t* off = halloc(ctx, 8 * (n + 1));
    uint8_t* dk = halloc(ctx, n * K + 16);
    uint8_t* dv = halloc(ctx, n * V + 16);
    uint64_t* dko = halloc(ctx, 8 * (n + 1));
    uint64_t* dvo = halloc(ctx, 8 * (n + 1));
    uint8_t* st = halloc(ctx, n);
    const uint8_t* bytes[2] = {kb, vb};
    const uint64_t* offs[2] = {ko, vo};
    uint8_t* dbytes[2] = {dk, dv};
    uint64_t* doffs[2] = {dko, dvo};
    const uint64_t caps[2] = {n * K + 16, n * V + 16};
    const double t_w = now();
    int first = 1;
    double te = 0, td = 0;
    for (int i = 0; first || now() - t_w < warm || i < calls; ++i) {
        const int timed = !(first || now() - t_w < warm);
        const double t0 = now();
        if (sym_encode_host(ctx, SYM_SCHEMA_KV_SET_REQUEST, n, NULL, bytes, offs, 0, 0, out, off) != SYM_OK)
            DIE("sym_encode_host");
        const double t1 = now();
        if (sym_decode_host(ctx, SYM_SCHEMA_KV_SET_REQUEST, n, out, off, NULL, dbytes, caps, doffs, st) != SYM_OK)
            DIE("sym_decode_host");
        const double t2 = now();
        if (first) {
            if (off[n] != total || memcmp(dk, kb, n * K) || memcmp(dv, vb, n * V) || dvo[n] != n * V) {
                fprintf(stderr, "round trip mismatch\n");
                return 1;
            }
            first = 0;
        }
        if (timed) {
            te += t1 - t0;
            td += t2 - t1;
            printf("call: encode %.2f ms, decode %.2f ms\n", 1e3 * (t1 - t0), 1e3 * (t2 - t1));
        } else {
            i = -1;  /* timed calls start after the warm-up */
        }
    }
    const double alg = (double)(n * (K + V) + 2 * 8 * (n + 1)) + (double)(total + 8 * (n + 1));
    printf("{\"encode_gbps\": %.2f, \"decode_gbps\": %.2f, \"gbps_algorithmic\": %.2f}\n", alg * calls / te / 1e9,
           (alg + n) * calls / td / 1e9, (2 * alg + n) * calls / (te + td) / 1e9);
    sym_ctx_destroy(ctx);
    return 0;
}
