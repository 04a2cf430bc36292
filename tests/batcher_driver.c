/*
 * batcher_driver.c -- many POSIX threads, each calling the per-record batcher entry points
 * (sym_batcher_encode_one / sym_batcher_decode_one) one record at a time, as aRPC's Call
 * goroutines call Serializer.Marshal (pkg/rpc/client.go:233-310, :252) and the receive paths call
 * Unmarshal (pkg/rpc/server.go:152, client.go:205).  Plain C against include/symphony_hip.h.
 *
 *   batcher_driver THREADS PER_THREAD OUT_FILE          the parity run below
 *   batcher_driver THREADS PER_THREAD - bench           timing: encode_one + decode_one per record, no
 *                                                       error cases, no output; prints elapsed_s
 *   batcher_driver 1 RECORDS - host1                     timing without the batcher: one record per
 *                                                       sym_encode_host + sym_decode_host call (n = 1)
 *
 * Thread t, record i: SetRequest{Key, Value} with the lengths and bytes of rec() below (the Python
 * test regenerates them), client IDs (1, 2) on odd i.  Each encoded record is decoded back through
 * the batcher and compared with its fields; a truncated and a bad-version copy check the error
 * statuses.  The encoded records go to OUT_FILE (thread-major, each as u32 length + bytes) for
 * tests/test_batcher.py to compare with the C oracle's MarshalSymphony.  Prints
 * "batcher_driver: R records ok in B encode / D decode batches".
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/symphony_hip.h"

static sym_batcher* g_b;
static int g_per;
static int g_bench;
static uint8_t** g_out;   /* [threads * per] encoded records */
static uint64_t* g_len;

#define DIE(...)                                                  \
    do {                                                          \
        fprintf(stderr, __VA_ARGS__);                             \
        fprintf(stderr, " [%s]\n", sym_last_error());             \
        exit(1);                                                  \
    } while (0)

static void rec(int t, int i, uint8_t* key, uint64_t* kl, uint8_t* val, uint64_t* vl) {
    *kl = (uint64_t)((t * 7 + i * 3) % 70);
    *vl = (uint64_t)((t * 13 + i * 5) % 300);
    for (uint64_t j = 0; j < *kl; ++j) key[j] = (uint8_t)(t * 31 + i * 17 + j);
    for (uint64_t j = 0; j < *vl; ++j) val[j] = (uint8_t)(t * 11 + i * 29 + 3 * j);
}

static void* worker(void* arg) {
    const int t = (int)(intptr_t)arg;
    uint8_t key[80], val[320], enc[512], dk[512], dv[512];
    for (int i = 0; i < g_per; ++i) {
        uint64_t kl, vl, n = 0;
        rec(t, i, key, &kl, val, &vl);
        const uint8_t* fields[2] = {key, val};
        const uint64_t lens[2] = {kl, vl};
        const uint32_t sid = (i & 1) ? 1 : 0, mid = (i & 1) ? 2 : 0;
        int rc = sym_batcher_encode_one(g_b, NULL, fields, lens, sid, mid, enc, sizeof(enc), &n);
        if (rc != SYM_OK || n != 30 + kl + vl) DIE("encode t=%d i=%d rc=%d n=%llu", t, i, rc, (unsigned long long)n);
        if (!g_bench) {
            const size_t at = (size_t)t * g_per + i;
            g_out[at] = malloc(n);
            memcpy(g_out[at], enc, n);
            g_len[at] = n;
        }
        /* decode it back: the fields, status OK */
        uint8_t* outs[2] = {dk, dv};
        const uint64_t caps[2] = {sizeof(dk), sizeof(dv)};
        uint64_t got[2] = {0, 0};
        uint8_t st = 99;
        rc = sym_batcher_decode_one(g_b, enc, n, NULL, outs, caps, got, &st);
        if (rc != SYM_OK || st != SYM_STATUS_OK || got[0] != kl || got[1] != vl || memcmp(dk, key, kl) ||
            memcmp(dv, val, vl))
            DIE("decode t=%d i=%d rc=%d st=%d", t, i, rc, st);
        if (!g_bench && i % 16 == 0) { /* errors Go returns: too short, wrong public version */
            rc = sym_batcher_decode_one(g_b, enc, 12, NULL, outs, caps, got, &st);
            if (rc != SYM_OK || st != SYM_STATUS_TOO_SHORT || got[0] || got[1]) DIE("short t=%d i=%d st=%d", t, i, st);
            enc[0] = 2;
            rc = sym_batcher_decode_one(g_b, enc, n, NULL, outs, caps, got, &st);
            if (rc != SYM_OK || st != SYM_STATUS_BAD_VERSION) DIE("version t=%d i=%d st=%d", t, i, st);
        }
    }
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* One record per sym_encode_host / sym_decode_host call, no batcher: the per-record latency a
 * Serializer adapter without coalescing pays. */
static int host1(int records) {
    sym_ctx* ctx = NULL;
    if (sym_ctx_create(0, &ctx) != SYM_OK) DIE("ctx");
    uint8_t key[80], val[320], enc[512], dk[512], dv[512], st;
    uint64_t ko[2], vo[2], eo[2], dko[2], dvo[2];
    double t0 = 0;
    for (int i = -100; i < records; ++i) { /* 100 untimed warm-up calls */
        if (i == 0) t0 = now_s();
        uint64_t kl, vl;
        rec(0, i < 0 ? -i : i, key, &kl, val, &vl);
        ko[0] = 0, ko[1] = kl, vo[0] = 0, vo[1] = vl;
        const uint8_t* b[2] = {key, val};
        const uint64_t* o[2] = {ko, vo};
        if (sym_encode_host(ctx, SYM_SCHEMA_KV_SET_REQUEST, 1, NULL, b, o, 0, 0, enc, eo) != SYM_OK) DIE("encode_host");
        uint8_t* db[2] = {dk, dv};
        const uint64_t caps[2] = {sizeof(dk), sizeof(dv)};
        uint64_t* dof[2] = {dko, dvo};
        if (sym_decode_host(ctx, SYM_SCHEMA_KV_SET_REQUEST, 1, enc, eo, NULL, db, caps, dof, &st) != SYM_OK ||
            st != 0 || dvo[1] != vl || memcmp(dv, val, vl))
            DIE("decode_host");
    }
    const double el = now_s() - t0;
    sym_ctx_destroy(ctx);
    printf("host1: %d records elapsed_s=%.6f\n", records, el);
    return 0;
}

int main(int argc, char** argv) {
    if (argc != 4 && argc != 5) {
        fprintf(stderr, "usage: batcher_driver THREADS PER_THREAD OUT_FILE|- [bench|host1]\n");
        return 2;
    }
    const int T = atoi(argv[1]);
    g_per = atoi(argv[2]);
    if (argc == 5 && !strcmp(argv[4], "host1")) return host1(g_per);
    g_bench = argc == 5 && !strcmp(argv[4], "bench");
    if (sym_batcher_create(0, SYM_SCHEMA_KV_SET_REQUEST, 256, 1 << 20, g_bench ? 0 : 20, &g_b) != SYM_OK) DIE("create");
    g_out = calloc((size_t)T * g_per, sizeof(uint8_t*));
    g_len = calloc((size_t)T * g_per, sizeof(uint64_t));
    pthread_t* th = malloc(sizeof(pthread_t) * T);
    const double t0 = now_s();
    for (int t = 0; t < T; ++t)
        if (pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t)) DIE("pthread_create");
    for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
    const double el = now_s() - t0;
    uint64_t eb, er, db, dr;
    if (sym_batcher_stats(g_b, &eb, &er, &db, &dr) != SYM_OK) DIE("stats");
    if (g_bench) {
        sym_batcher_destroy(g_b);
        printf("bench: %llu records in %llu encode / %llu decode batches elapsed_s=%.6f\n", (unsigned long long)er,
               (unsigned long long)eb, (unsigned long long)db, el);
        return 0;
    }
    FILE* f = fopen(argv[3], "wb");
    if (!f) DIE("open %s", argv[3]);
    for (size_t k = 0; k < (size_t)T * g_per; ++k) {
        const uint32_t l = (uint32_t)g_len[k];
        fwrite(&l, 4, 1, f);
        fwrite(g_out[k], 1, l, f);
        free(g_out[k]);
    }
    fclose(f);
    sym_batcher_destroy(g_b);
    printf("batcher_driver: %llu records ok in %llu encode / %llu decode batches\n", (unsigned long long)er,
           (unsigned long long)eb, (unsigned long long)db);
    return 0;
}
