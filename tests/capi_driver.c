/*
 * capi_driver.c -- a plain C client of libsymphony_hip.so, compiled by gcc against
 * include/symphony_hip.h (so a drift between the header's prototypes and the library shows up
 * as a compile error or a wrong answer here, which ctypes would not catch).
 *
 * It calls every typed entry point a cgo binding would (sym_encode_kv_set / _kv_get /
 * _kv_response / _echo, sym_decode_* likewise, the mixed Get/Set pair and the *_host entry
 * points) on the known-answer records hand-derived from the reference's generated code
 * (tests/golden/make_golden.py; benchmark/kv-store-symphony/symphony/kv.syn.go,
 * examples/echo_symphony/symphony/echo.syn.go), repeated across tiles, and decodes them back.
 *
 *   capi_driver            exit 0 and "capi_driver: N checks ok" when everything matches
 *
 * Built by tests/Makefile (gcc, -lamdhip64); run by tests/test_capi_typed.py on the GPU box.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/symphony_hip.h"

static int g_checks = 0;

#define CHECK(cond, ...)                                   \
    do {                                                   \
        ++g_checks;                                        \
        if (!(cond)) {                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                  \
            fprintf(stderr, " [%s]\n", sym_last_error());  \
            exit(1);                                       \
        }                                                  \
    } while (0)

#define HIPCHECK(x) CHECK((x) == hipSuccess, "%s", #x)

static size_t unhex(const char* s, uint8_t* out) {
    size_t n = 0;
    for (; s[0] && s[1]; s += 2) {
        unsigned v;
        sscanf(s, "%2x", &v);
        out[n++] = (uint8_t)v;
    }
    return n;
}

static void* dev_copy(const void* h, size_t n) {
    void* d = NULL;
    HIPCHECK(hipMalloc(&d, n + 16));
    if (n) HIPCHECK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    return d;
}

/* A column of `reps` copies of `v` (length len) with offsets. */
static void make_col(const char* v, size_t len, int reps, uint8_t** bytes, uint64_t** offs) {
    *bytes = malloc(len * reps + 1);
    *offs = malloc(8 * (reps + 1));
    for (int i = 0; i <= reps; ++i) (*offs)[i] = (uint64_t)i * len;
    for (int i = 0; i < reps; ++i) memcpy(*bytes + (size_t)i * len, v, len);
}

/* The stream must be `reps` copies of the KAT; checks every byte and offset. */
static void expect_stream(const char* what, const uint8_t* d_out, const uint64_t* d_off, int reps, const char* kat_hex) {
    uint8_t kat[256];
    const size_t k = unhex(kat_hex, kat);
    uint8_t* h = malloc(k * reps);
    uint64_t* o = malloc(8 * (reps + 1));
    HIPCHECK(hipMemcpy(h, d_out, k * reps, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(o, d_off, 8 * (reps + 1), hipMemcpyDeviceToHost));
    for (int i = 0; i < reps; ++i) {
        CHECK(o[i] == (uint64_t)i * k, "%s: offset %d is %llu", what, i, (unsigned long long)o[i]);
        CHECK(!memcmp(h + (size_t)i * k, kat, k), "%s: record %d differs from the KAT", what, i);
    }
    CHECK(o[reps] == (uint64_t)reps * k, "%s: final offset", what);
    free(h);
    free(o);
}

/* Decoded column must be `reps` copies of v. */
static void expect_col(const char* what, const uint8_t* d_b, const uint64_t* d_o, int reps, const char* v, size_t len) {
    uint64_t* o = malloc(8 * (reps + 1));
    HIPCHECK(hipMemcpy(o, d_o, 8 * (reps + 1), hipMemcpyDeviceToHost));
    uint8_t* h = malloc(len * reps + 1);
    if (len) HIPCHECK(hipMemcpy(h, d_b, len * reps, hipMemcpyDeviceToHost));
    for (int i = 0; i < reps; ++i) {
        CHECK(o[i] == (uint64_t)i * len, "%s: column offset %d", what, i);
        CHECK(!len || !memcmp(h + (size_t)i * len, v, len), "%s: value %d", what, i);
    }
    free(o);
    free(h);
}

static void expect_status_ok(const char* what, const uint8_t* d_st, int reps) {
    uint8_t* st = malloc(reps);
    HIPCHECK(hipMemcpy(st, d_st, reps, hipMemcpyDeviceToHost));
    for (int i = 0; i < reps; ++i) CHECK(st[i] == SYM_STATUS_OK, "%s: status %d = %u", what, i, st[i]);
    free(st);
}

#define HDR "010d000000" "00000000" "00000000" "01"

int main(void) {
    const int R = 1000; /* records per batch: spans 16 tiles */
    sym_ctx* ctx = NULL;
    CHECK(sym_abi_version() == SYMPHONY_HIP_ABI_VERSION, "ABI version");
    CHECK(sym_ctx_create(0, &ctx) == SYM_OK, "sym_ctx_create");
    CHECK(sym_record_overhead(SYM_SCHEMA_KV_SET_REQUEST) == 30, "SetRequest overhead");
    CHECK(sym_encoded_size_kv_mixed(4, 2, 6, 3) == 4 * 22 + 16 + 9, "mixed size");

    uint8_t *kb, *vb, *ub, *cb;
    uint64_t *ko, *vo, *uo, *co;
    make_col("ab", 2, R, &kb, &ko);
    make_col("xyz", 3, R, &vb, &vo);
    make_col("alice", 5, R, &ub, &uo);
    make_col("hello world", 11, R, &cb, &co);
    uint8_t *d_kb = dev_copy(kb, 2 * R), *d_vb = dev_copy(vb, 3 * R), *d_ub = dev_copy(ub, 5 * R),
            *d_cb = dev_copy(cb, 11 * R);
    uint64_t *d_ko = dev_copy(ko, 8 * (R + 1)), *d_vo = dev_copy(vo, 8 * (R + 1)), *d_uo = dev_copy(uo, 8 * (R + 1)),
             *d_co = dev_copy(co, 8 * (R + 1));
    int32_t id[1000], score[1000];
    for (int i = 0; i < R; ++i) {
        id[i] = 42;
        score[i] = 300;
    }
    int32_t *d_id = dev_copy(id, 4 * R), *d_score = dev_copy(score, 4 * R);

    uint8_t *d_out, *d_st, *d_k2, *d_v2;
    uint64_t *d_off, *d_ko2, *d_vo2;
    int32_t *d_id2, *d_sc2;
    HIPCHECK(hipMalloc((void**)&d_out, 64 * R));
    HIPCHECK(hipMalloc((void**)&d_off, 8 * (R + 1)));
    HIPCHECK(hipMalloc((void**)&d_st, R));
    HIPCHECK(hipMalloc((void**)&d_k2, 64 * R));
    HIPCHECK(hipMalloc((void**)&d_v2, 64 * R));
    HIPCHECK(hipMalloc((void**)&d_ko2, 8 * (R + 1)));
    HIPCHECK(hipMalloc((void**)&d_vo2, 8 * (R + 1)));
    HIPCHECK(hipMalloc((void**)&d_id2, 4 * R));
    HIPCHECK(hipMalloc((void**)&d_sc2, 4 * R));

    /* SetRequest{"ab","xyz"}, plain and with the client's IDs (service 1, Set = method 2) */
    CHECK(sym_encode_kv_set(ctx, d_kb, d_ko, d_vb, d_vo, R, 0, 0, d_out, d_off, NULL) == SYM_OK, "encode_kv_set");
    CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
    expect_stream("kv_set", d_out, d_off, R, HDR "09000000" "0f000000" "02000000" "6162" "03000000" "78797a");
    CHECK(sym_decode_kv_set(ctx, d_out, d_off, R, d_k2, 64 * R, d_ko2, d_v2, 64 * R, d_vo2, d_st, NULL) == SYM_OK,
          "decode_kv_set");
    CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
    expect_status_ok("kv_set", d_st, R);
    expect_col("kv_set key", d_k2, d_ko2, R, "ab", 2);
    expect_col("kv_set value", d_v2, d_vo2, R, "xyz", 3);
    CHECK(sym_encode_kv_set(ctx, d_kb, d_ko, d_vb, d_vo, R, 1, 2, d_out, d_off, NULL) == SYM_OK, "encode_kv_set ids");
    CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
    expect_stream("kv_set ids", d_out, d_off, R,
                  "010d000000" "01000000" "02000000" "01" "09000000" "0f000000" "02000000" "6162" "03000000" "78797a");

    /* GetRequest{"ab"} */
    CHECK(sym_encode_kv_get(ctx, d_kb, d_ko, R, 1, 1, d_out, d_off, NULL) == SYM_OK, "encode_kv_get");
    CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
    expect_stream("kv_get", d_out, d_off, R, "010d000000" "01000000" "01000000" "01" "05000000" "02000000" "6162");
    CHECK(sym_decode_kv_get(ctx, d_out, d_off, R, d_k2, 64 * R, d_ko2, d_st, NULL) == SYM_OK, "decode_kv_get");
    CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
    expect_status_ok("kv_get", d_st, R);
    expect_col("kv_get key", d_k2, d_ko2, R, "ab", 2);

    /* GetResponse{"xyz"} / SetResponse{"xyz"} */
    for (int schema = SYM_SCHEMA_KV_GET_RESPONSE; schema <= SYM_SCHEMA_KV_SET_RESPONSE; ++schema) {
        CHECK(sym_encode_kv_response(ctx, schema, d_vb, d_vo, R, 0, 0, d_out, d_off, NULL) == SYM_OK, "encode_kv_response");
        CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
        expect_stream("kv_response", d_out, d_off, R, HDR "05000000" "03000000" "78797a");
        CHECK(sym_decode_kv_response(ctx, schema, d_out, d_off, R, d_v2, 64 * R, d_vo2, d_st, NULL) == SYM_OK,
              "decode_kv_response");
        CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
        expect_status_ok("kv_response", d_st, R);
        expect_col("kv_response value", d_v2, d_vo2, R, "xyz", 3);
    }
    CHECK(sym_encode_kv_response(ctx, SYM_SCHEMA_KV_SET_REQUEST, d_vb, d_vo, R, 0, 0, d_out, d_off, NULL) ==
              SYM_ERR_INVALID, "response entry point rejects a request schema");

    /* EchoRequest{42, 300, "alice", "hello world"} (config 1's record, 54 bytes) */
    CHECK(sym_encode_echo(ctx, d_id, d_score, d_ub, d_uo, d_cb, d_co, R, 0, 0, d_out, d_off, NULL) == SYM_OK,
          "encode_echo");
    CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
    expect_stream("echo", d_out, d_off, R,
                  HDR "2a000000" "2c010000" "11000000" "1a000000" "05000000" "616c696365" "0b000000"
                      "68656c6c6f20776f726c64");
    CHECK(sym_decode_echo(ctx, d_out, d_off, R, d_id2, d_sc2, d_k2, 64 * R, d_ko2, d_v2, 64 * R, d_vo2, d_st, NULL) ==
              SYM_OK, "decode_echo");
    CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
    expect_status_ok("echo", d_st, R);
    expect_col("echo username", d_k2, d_ko2, R, "alice", 5);
    expect_col("echo content", d_v2, d_vo2, R, "hello world", 11);
    {
        int32_t a[1000], b[1000];
        HIPCHECK(hipMemcpy(a, d_id2, 4 * R, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(b, d_sc2, 4 * R, hipMemcpyDeviceToHost));
        for (int i = 0; i < R; ++i) CHECK(a[i] == 42 && b[i] == 300, "echo int32 fields, record %d", i);
    }

    /* mixed Get/Set: record i is a Get when i % 3 == 0 (its value slice "xyz" is not encoded) */
    {
        uint8_t ty[1000];
        for (int i = 0; i < R; ++i) ty[i] = i % 3 == 0 ? 0 : 1;
        uint8_t* d_ty = dev_copy(ty, R);
        CHECK(sym_encode_kv_mixed(ctx, d_ty, d_kb, d_ko, d_vb, d_vo, R, 1, 1, 2, d_out, d_off, NULL) == SYM_OK,
              "encode_kv_mixed");
        CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
        uint8_t get[64], set[64];
        const size_t lg = unhex("010d000000" "01000000" "01000000" "01" "05000000" "02000000" "6162", get);
        const size_t ls = unhex("010d000000" "01000000" "02000000" "01" "09000000" "0f000000" "02000000" "6162"
                                "03000000" "78797a", set);
        uint8_t* h = malloc(64 * R);
        uint64_t* o = malloc(8 * (R + 1));
        HIPCHECK(hipMemcpy(o, d_off, 8 * (R + 1), hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(h, d_out, o[R], hipMemcpyDeviceToHost));
        uint64_t at = 0;
        for (int i = 0; i < R; ++i) {
            const uint8_t* want = ty[i] ? set : get;
            const size_t len = ty[i] ? ls : lg;
            CHECK(o[i] == at && !memcmp(h + at, want, len), "mixed record %d", i);
            at += len;
        }
        CHECK(o[R] == at && at == sym_encoded_size_kv_mixed(R, R - (R + 2) / 3, 2 * R, 3 * (R - (R + 2) / 3)),
              "mixed total");
        CHECK(sym_decode_kv_mixed(ctx, d_out, d_off, d_ty, R, d_k2, 64 * R, d_ko2, d_v2, 64 * R, d_vo2, d_st, NULL) ==
                  SYM_OK, "decode_kv_mixed");
        CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check");
        expect_status_ok("mixed", d_st, R);
        expect_col("mixed key", d_k2, d_ko2, R, "ab", 2);
        HIPCHECK(hipMemcpy(o, d_vo2, 8 * (R + 1), hipMemcpyDeviceToHost));
        uint64_t v = 0;
        for (int i = 0; i < R; ++i) {
            CHECK(o[i] == v, "mixed value offset %d", i);
            v += ty[i] ? 3 : 0;
        }
        free(h);
        free(o);
        HIPCHECK(hipFree(d_ty));
    }

    /* every decode implementation gives the same answer through the typed entry point */
    for (int impl = SYM_DECODE_PIPELINE; impl <= SYM_DECODE_LOOKBACK; ++impl) {
        CHECK(sym_ctx_set_decode_impl(ctx, impl) == SYM_OK, "set_decode_impl %d", impl);
        CHECK(sym_encode_kv_set(ctx, d_kb, d_ko, d_vb, d_vo, R, 0, 0, d_out, d_off, NULL) == SYM_OK, "encode");
        CHECK(sym_decode_kv_set(ctx, d_out, d_off, R, d_k2, 64 * R, d_ko2, d_v2, 64 * R, d_vo2, d_st, NULL) == SYM_OK,
              "decode impl %d", impl);
        CHECK(sym_ctx_check(ctx, NULL) == SYM_OK, "check impl %d", impl);
        expect_col("impl key", d_k2, d_ko2, R, "ab", 2);
        expect_col("impl value", d_v2, d_vo2, R, "xyz", 3);
    }
    CHECK(sym_ctx_set_decode_impl(ctx, 7) == SYM_ERR_INVALID, "unknown decode impl rejected");
    CHECK(sym_ctx_set_decode_impl(ctx, SYM_DECODE_PIPELINE) == SYM_OK, "reset impl");

    /* host-memory entry points: the same KAT through sym_encode_host / sym_decode_host */
    {
        const uint8_t* hb[2] = {kb, vb};
        const uint64_t* ho[2] = {ko, vo};
        uint8_t* out = malloc(35 * R);
        uint64_t* off = malloc(8 * (R + 1));
        CHECK(sym_encode_host(ctx, SYM_SCHEMA_KV_SET_REQUEST, R, NULL, hb, ho, 1, 2, out, off) == SYM_OK, "encode_host");
        uint8_t kat[64];
        const size_t k = unhex("010d000000" "01000000" "02000000" "01" "09000000" "0f000000" "02000000" "6162"
                               "03000000" "78797a", kat);
        for (int i = 0; i < R; ++i) CHECK(off[i] == (uint64_t)i * k && !memcmp(out + (size_t)i * k, kat, k), "host record %d", i);
        uint8_t* k2 = malloc(2 * R);
        uint8_t* v2 = malloc(3 * R);
        uint64_t* ko3 = malloc(8 * (R + 1));
        uint64_t* vo3 = malloc(8 * (R + 1));
        uint8_t* st = malloc(R);
        uint8_t* cols[2] = {k2, v2};
        uint64_t* offs[2] = {ko3, vo3};
        const uint64_t caps[2] = {2 * (uint64_t)R, 3 * (uint64_t)R};
        CHECK(sym_decode_host(ctx, SYM_SCHEMA_KV_SET_REQUEST, R, out, off, NULL, cols, caps, offs, st) == SYM_OK,
              "decode_host");
        for (int i = 0; i < R; ++i)
            CHECK(st[i] == 0 && ko3[i] == 2u * i && vo3[i] == 3u * i && !memcmp(k2 + 2 * i, "ab", 2) &&
                      !memcmp(v2 + 3 * i, "xyz", 3), "host decode record %d", i);
        const uint64_t small[2] = {2 * (uint64_t)R, 3 * (uint64_t)R - 1};
        CHECK(sym_decode_host(ctx, SYM_SCHEMA_KV_SET_REQUEST, R, out, off, NULL, cols, small, offs, st) ==
                  SYM_ERR_CAPACITY, "decode_host reports a short column");
        free(out);
        free(off);
        free(k2);
        free(v2);
        free(ko3);
        free(vo3);
        free(st);
    }

    CHECK(sym_ctx_destroy(ctx) == SYM_OK, "destroy");
    printf("capi_driver: %d checks ok\n", g_checks);
    return 0;
}
