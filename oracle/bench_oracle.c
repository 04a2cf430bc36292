/*
 * bench_oracle.c -- CPU baseline timing loops over the C restatement (symphony_oracle.c).
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY: called by bench.py's cpu_baseline leg; the product library
 * never links it.  It is the reference's serialization benchmark methodology restated in C,
 * because no Go toolchain exists in this image or on the GPU box:
 *   benchmark/serialization/testcases/simple/main.go:34-37 (the record), :248-322 (Marshal loop),
 *   :324-420 (Unmarshal loop): one record per call, one goroutine, MarshalSymphony allocating its
 *   output buffer (make([]byte, size)) and UnmarshalSymphony allocating each string it decodes.
 * The loops below keep those allocation semantics (malloc per output buffer / per decoded string).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

uint64_t sym_oracle_record_size(int nfixed, int nvar, const uint64_t* lens);
uint64_t sym_oracle_marshal(int nfixed, int nvar, const int32_t* fixed, const uint8_t* const* field,
                            const uint64_t* lens, uint32_t sid, uint32_t mid, uint8_t* out);
int sym_oracle_unmarshal(int nfixed, int nvar, const uint8_t* data, uint64_t len, int32_t* fixed_out,
                         uint64_t* pos_out, uint64_t* len_out);

static double now_ns(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e9 + (double)ts.tv_nsec;
}

/* EchoRequest{Id: 42, Score: 300, Username: "alice", Content: "hello world"} (54 bytes).
 * Runs `iters` marshals, then `iters` unmarshals of the marshalled record; writes ns per
 * marshal / unmarshal.  Returns a checksum so the loops cannot be optimised away. */
uint64_t sym_oracle_bench_echo(uint64_t iters, double* marshal_ns, double* unmarshal_ns) {
    const int32_t fixed[2] = {42, 300};
    const uint8_t* fields[2] = {(const uint8_t*)"alice", (const uint8_t*)"hello world"};
    const uint64_t lens[2] = {5, 11};
    uint64_t sum = 0;
    double t0 = now_ns();
    for (uint64_t i = 0; i < iters; ++i) {
        const uint64_t size = sym_oracle_record_size(2, 2, lens);
        uint8_t* buf = malloc(size); /* make([]byte, size) */
        sym_oracle_marshal(2, 2, fixed, fields, lens, 0, 0, buf);
        sum += buf[size - 1];
        free(buf);
    }
    double t1 = now_ns();
    uint8_t rec[64];
    const uint64_t size = sym_oracle_marshal(2, 2, fixed, fields, lens, 0, 0, rec);
    for (uint64_t i = 0; i < iters; ++i) {
        int32_t fx[2];
        uint64_t pos[2], ln[2];
        sym_oracle_unmarshal(2, 2, rec, size, fx, pos, ln);
        for (int f = 0; f < 2; ++f) { /* string(data[...]) copies */
            char* s = malloc(ln[f] + 1);
            memcpy(s, rec + pos[f], ln[f]);
            sum += (uint8_t)s[0] + (uint64_t)fx[f];
            free(s);
        }
    }
    double t2 = now_ns();
    *marshal_ns = (t1 - t0) / (double)iters;
    *unmarshal_ns = (t2 - t1) / (double)iters;
    return sum;
}

uint64_t sym_oracle_encode_batch(int nfixed, int nvar, uint64_t n, const int32_t* const* fixed_cols,
                                 const uint8_t* const* bytes, const uint64_t* const* offs, uint32_t sid,
                                 uint32_t mid, uint8_t* out, uint64_t* out_off);
void sym_oracle_decode_batch(int nfixed, int nvar, uint64_t n, const uint8_t* in, const uint64_t* rec_off,
                             int32_t* const* fixed_out, uint8_t* const* bytes_out, uint64_t* const* offs_out,
                             uint8_t* status);

/* The batch restatement timed as the headline measures the GPU: `reps` rounds of encode into a
 * preallocated stream, then decode of it into preallocated columns, over the caller's whole batch
 * (bench.py passes the headline's 2^20 records: a working set of ~1 GB, far beyond the host's caches).
 * Writes each round's encode and decode seconds.  Returns the last stream's size. */
uint64_t sym_oracle_bench_batch(int nfixed, int nvar, uint64_t n, const int32_t* const* fixed, const uint8_t* const* bytes,
                                const uint64_t* const* offs, uint8_t* out, uint64_t* out_off, int32_t* const* dfixed,
                                uint8_t* const* dbytes, uint64_t* const* doffs, uint8_t* status, int reps,
                                double* enc_s, double* dec_s) {
    uint64_t size = 0;
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_ns();
        size = sym_oracle_encode_batch(nfixed, nvar, n, fixed, bytes, offs, 0, 0, out, out_off);
        const double t1 = now_ns();
        sym_oracle_decode_batch(nfixed, nvar, n, out, out_off, dfixed, dbytes, doffs, status);
        const double t2 = now_ns();
        enc_s[r] = (t1 - t0) * 1e-9;
        dec_s[r] = (t2 - t1) * 1e-9;
    }
    return size;
}
