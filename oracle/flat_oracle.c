/*
 * flat_oracle.c -- CPU restatement of the generated MarshalSymphony / UnmarshalSymphony for any flat
 * schema (fixed-width and string / bytes fields, each public or private).
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the HIP flat-schema codec
 * (arpc_amd/csrc/flat.hip).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it.
 *
 * Parity status: pinned by the reference's own access-control test values on the Fixed message
 * (cmd/symphony-gen-arpc/test/serialization_test.go:555-703), by byte equality with the kv-store
 * restatement (symphony_oracle.c, itself pinned by tests/golden/kats.json) for the all-private
 * schemas, and with the element-schema marshal of raw_oracle.c; the reference is never run (Go).
 *
 * What it restates (paths relative to the reference root; generator
 * cmd/symphony-gen-arpc/protoc-gen-symphony/main.go):
 *   fields are classified public / private in declaration order      classifyFields :1172-1239
 *   MarshalSymphony: header [0]=1, [1:5]=offsetToPrivate (= 13 + public table + public payloads),
 *     [5:13]=0; public table at 13 (fixed fields inline at their width, string fields a 4-byte
 *     ABSOLUTE payload offset), public payloads (u32 length + bytes) in field order; private
 *     version byte 1 at offsetToPrivate, private table, private payloads with offsets RELATIVE to
 *     offsetToPrivate                                                  :196-330, 334-368, 439-620
 *   UnmarshalSymphony (into a fresh struct): len < 13 -> "too short"; [0] != 1 -> "wrong public
 *     version"; offsetToPrivate >= len or data[off] != 1 -> "missing private segment"; then every
 *     public field, then every private field (table at offsetToPrivate + 1): a fixed field past
 *     the end -> "too short for field" (earlier fields keep their values); a string field whose
 *     table entry, offset or length runs past the end, or whose offset is 0, is left empty  :622-800
 *   Empty messages (no fields) are 14 bytes and unmarshal with the len < 14 check     :201-212, 628-642
 */
#include <stdint.h>
#include <string.h>

#define ST_OK 0
#define ST_TOO_SHORT 1
#define ST_BAD_VERSION 2
#define ST_NO_PRIVATE 3
#define ST_FIELD_TOO_SHORT 4

/* A field: segment (0 public, 1 private) and width (1, 4, 8; 0 = string / bytes; REP | 1/4/8 =
 * repeated fixed-width: payload [u32 count][count * w bytes], main.go:493-535, decode :795-841). */
typedef struct {
    uint8_t segment, width;
} Field;

#define REP 0x80
/* scalar fixed width (0 for payload fields) and a payload field's element width (1 for strings) */
static int scalar_w(const Field* f) { return (f->width & REP) ? 0 : f->width; }
static int elem_w(const Field* f) { return (f->width & REP) ? (f->width & 0x7f) : 1; }

static void wr32(uint8_t* p, uint32_t v) {
    for (int b = 0; b < 4; ++b) p[b] = (uint8_t)(v >> (8 * b));
}
static uint64_t rd(const uint8_t* p, int w) {
    uint64_t v = 0;
    for (int b = 0; b < w; ++b) v |= (uint64_t)p[b] << (8 * b);
    return v;
}

static uint64_t table_size(const Field* f, int nf, int seg) {
    uint64_t t = 0;
    for (int k = 0; k < nf; ++k)
        if (f[k].segment == seg) t += scalar_w(&f[k]) ? scalar_w(&f[k]) : 4;
    return t;
}

/* Marshal n records.  fixed[k] (fixed field k): n values of width bytes; var[k] / var_off[k]
 * (string field k): packed bytes + n+1 offsets; columns are indexed by field index (unused slots
 * NULL).  Returns total bytes. */
uint64_t sym_oracle_flat_encode(int nf, const Field* f, uint64_t n, const uint8_t* const* fixed,
                                const uint8_t* const* var, const uint64_t* const* var_off, uint32_t service_id,
                                uint32_t method_id, uint8_t* out, uint64_t* out_off) {
    const uint64_t pt = table_size(f, nf, 0), vt = table_size(f, nf, 1);
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t* b = out + w;
        out_off[i] = w;
        if (nf == 0) { /* :201-212 */
            memset(b, 0, 14);
            b[0] = 1;
            wr32(b + 1, 13);
            wr32(b + 5, service_id);
            wr32(b + 9, method_id);
            b[13] = 1;
            w += 14;
            continue;
        }
        uint64_t pos[2] = {13 + pt, 0}; /* payload cursor per segment (absolute) */
        uint64_t off2p = 13 + pt;
        for (int k = 0; k < nf; ++k)
            if (f[k].segment == 0 && !scalar_w(&f[k])) off2p += 4 + (var_off[k][i + 1] - var_off[k][i]);
        memset(b, 0, 13);
        b[0] = 1;
        wr32(b + 1, (uint32_t)off2p);
        wr32(b + 5, service_id); /* the client's ID patch, pkg/rpc/client.go:267-271 */
        wr32(b + 9, method_id);
        b[off2p] = 1;
        pos[1] = off2p + 1 + vt;
        uint64_t tab[2] = {13, off2p + 1};
        for (int k = 0; k < nf; ++k) {
            const int s = f[k].segment;
            const int sw = scalar_w(&f[k]);
            if (sw) {
                memcpy(b + tab[s], fixed[k] + (uint64_t)sw * i, sw);
                tab[s] += sw;
            } else {
                /* string: u32 byte length; repeated fixed: u32 element count (:506-507) */
                const uint64_t L = var_off[k][i + 1] - var_off[k][i];
                wr32(b + tab[s], (uint32_t)(s ? pos[s] - off2p : pos[s]));
                wr32(b + pos[s], (uint32_t)(L / elem_w(&f[k])));
                if (L) memcpy(b + pos[s] + 4, var[k] + var_off[k][i], L);
                pos[s] += 4 + L;
                tab[s] += 4;
            }
        }
        w += pos[1];
    }
    out_off[n] = w;
    return w;
}

/* Unmarshal n records into fresh structs: fixed[k] n values of width bytes (0 unless read);
 * var[k] packed values with var_off[k][n+1]; status[n]. */
void sym_oracle_flat_decode(int nf, const Field* f, uint64_t n, const uint8_t* in, const uint64_t* rec_off,
                            uint8_t* const* fixed, uint8_t* const* var, uint64_t* const* var_off, uint8_t* status) {
    uint64_t w[64] = {0};
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* d = in + rec_off[i];
        const uint64_t L = rec_off[i + 1] - rec_off[i];
        for (int k = 0; k < nf; ++k) {
            if (scalar_w(&f[k])) memset(fixed[k] + (uint64_t)scalar_w(&f[k]) * i, 0, scalar_w(&f[k]));
            else var_off[k][i] = w[k];
        }
        int st = ST_OK;
        if (L < (nf ? 13u : 14u)) st = ST_TOO_SHORT;
        else if (d[0] != 1) st = ST_BAD_VERSION;
        else {
            const uint64_t o = rd(d + 1, 4);
            if (o >= L || d[o] != 1) st = ST_NO_PRIVATE;
            else {
                for (int s = 0; s < 2 && st == ST_OK; ++s) {
                    const uint64_t ts = s ? o + 1 : 13;
                    uint64_t t = 0;
                    for (int k = 0; k < nf && st == ST_OK; ++k) {
                        if (f[k].segment != s) continue;
                        const int sw = scalar_w(&f[k]);
                        if (sw) {
                            if (L < ts + t + sw) {
                                st = ST_FIELD_TOO_SHORT;
                                break;
                            }
                            memcpy(fixed[k] + (uint64_t)sw * i, d + ts + t, sw);
                            t += sw;
                        } else {
                            if (L >= ts + t + 4) {
                                uint64_t po = rd(d + ts + t, 4);
                                if (s && po > 0) po += o;
                                if (po > 0 && L >= po + 4) {
                                    /* string: length (:781-782); repeated: count * width (:812-813) */
                                    const uint64_t dl = rd(d + po, 4) * (uint64_t)elem_w(&f[k]);
                                    if (L >= po + 4 + dl) {
                                        memcpy(var[k] + w[k], d + po + 4, dl);
                                        w[k] += dl;
                                    }
                                }
                            }
                            t += 4;
                        }
                    }
                }
            }
        }
        status[i] = (uint8_t)st;
    }
    for (int k = 0; k < nf; ++k)
        if (!scalar_w(&f[k])) var_off[k][n] = w[k];
}
