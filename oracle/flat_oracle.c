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
#include <stdlib.h>
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

/* ---- Batched Raw setters: XxxRaw.SetF(v) on n buffers ----
 * Restated from the generator: assertions generateRawSetters main.go:1038-1093; fixed fields
 * generateRawFixedFieldSetter :1296-1336; strings / bytes generateRawVariableFieldSetter :1567-1620;
 * repeated fixed generateRawRepeatedFixedFieldSetter :1685-1740; the remarshal path
 * generateRemarshalLogic :371-437 (e.g. GetRequestRaw.SetUsername / SetKey,
 * benchmark/kv-store-symphony-element/symphony/kv.syn.go:340-412).
 * Per buffer, in Go's order:
 *   public field: len >= 5 and data[offsetToPrivate] == 1 (a complete buffer) -> panic
 *   private field: len < 5 -> panic; offsetToPrivate >= len or data[it] != 1 -> panic
 *   table entry past the end -> error "buffer too short [for table entry]"
 *   fixed: write in place
 *   payload (string: bytes, repeated: elements): in place when the old payload offset is set and
 *     the new length / count is <= the old one (u32 length / count, then the new bytes; a string's
 *     copy() stops at the buffer end, an element or length write past it panics); otherwise
 *     remarshal: public -- unmarshal data + [0x01] + a zeroed private table (private fields come
 *     back empty), set, marshal, restore bytes [5:13], keep [0, offsetToPrivate); private --
 *     unmarshal the buffer, set, marshal (bytes [5:13] become 0, as MarshalSymphony writes them).
 *     An unmarshal error -> error "failed to unmarshal".
 * A buffer whose setter panics or errors is output unchanged with that status. */
#define SET_OK 0
#define SET_COMPLETE_BUFFER 1
#define SET_INVALID_BUFFER 2
#define SET_PUBLIC_ONLY 3
#define SET_TOO_SHORT 4
#define SET_UNMARSHAL 5
#define SET_BOUNDS 6
#define SET_BAD_LENGTH 7  /* batch convention: a repeated value that is not whole elements */

/* table offset of field k inside its segment's table (public: absolute from 13; private: from 1) */
static uint64_t field_table_off(const Field* f, int k) {
    uint64_t t = f[k].segment ? 1 : 13;
    for (int j = 0; j < k; ++j)
        if (f[j].segment == f[k].segment) t += scalar_w(&f[j]) ? scalar_w(&f[j]) : 4;
    return t;
}

/* One record: unmarshal d[0, L) into a fresh struct (the rules of sym_oracle_flat_decode), returning
 * its status; fixed fields into fx (8 bytes per field), payload fields as (pointer, bytes). */
static int unmarshal_one(int nf, const Field* f, const uint8_t* d, uint64_t L, uint8_t fx[][8], const uint8_t** vp,
                         uint64_t* vl) {
    for (int k = 0; k < nf; ++k) {
        memset(fx[k], 0, 8);
        vp[k] = d;
        vl[k] = 0;
    }
    if (L < (nf ? 13u : 14u)) return ST_TOO_SHORT;
    if (d[0] != 1) return ST_BAD_VERSION;
    const uint64_t o = rd(d + 1, 4);
    if (o >= L || d[o] != 1) return ST_NO_PRIVATE;
    for (int s = 0; s < 2; ++s) {
        const uint64_t ts = s ? o + 1 : 13;
        uint64_t t = 0;
        for (int k = 0; k < nf; ++k) {
            if (f[k].segment != s) continue;
            const int sw = scalar_w(&f[k]);
            if (sw) {
                if (L < ts + t + sw) return ST_FIELD_TOO_SHORT;
                memcpy(fx[k], d + ts + t, sw);
                t += sw;
            } else {
                if (L >= ts + t + 4) {
                    uint64_t po = rd(d + ts + t, 4);
                    if (s && po > 0) po += o;
                    if (po > 0 && L >= po + 4) {
                        const uint64_t dl = rd(d + po, 4) * (uint64_t)elem_w(&f[k]);
                        if (L >= po + 4 + dl) {
                            vp[k] = d + po + 4;
                            vl[k] = dl;
                        }
                    }
                }
                t += 4;
            }
        }
    }
    return ST_OK;
}

/* Marshal one record from fixed values fx and payloads (vp, vl); returns its size. */
static uint64_t marshal_one(int nf, const Field* f, uint8_t fx[][8], const uint8_t* const* vp, const uint64_t* vl,
                            uint32_t sid, uint32_t mid, uint8_t* b) {
    const uint8_t* cols_fixed[64];
    const uint8_t* cols_var[64];
    uint64_t offs_store[64][2];
    const uint64_t* var_off[64];
    for (int k = 0; k < nf; ++k) {
        cols_fixed[k] = fx[k];
        cols_var[k] = vp[k];
        offs_store[k][0] = 0;
        offs_store[k][1] = vl[k];
        var_off[k] = offs_store[k];
    }
    uint64_t out_off[2];
    return sym_oracle_flat_encode(nf, f, 1, cols_fixed, cols_var, var_off, sid, mid, b, out_off);
}

/* Set field k of n buffers; value i: fixed -> val + i * width; payload -> val[val_off[i], val_off[i+1]).
 * Writes the resulting buffers back to back to out / out_off[n+1]; returns the total. */
uint64_t sym_oracle_raw_set(int nf, const Field* f, int k, uint64_t n, const uint8_t* in, const uint64_t* rec_off,
                            const uint8_t* val, const uint64_t* val_off, uint8_t* out, uint64_t* out_off,
                            uint8_t* status) {
    uint64_t w = 0;
    const int pub = f[k].segment == 0, sw = scalar_w(&f[k]), ew = elem_w(&f[k]);
    uint8_t fx[64][8];
    const uint8_t* vp[64];
    uint64_t vl[64];
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* m = in + rec_off[i];
        const uint64_t L = rec_off[i + 1] - rec_off[i];
        uint8_t* o = out + w;
        out_off[i] = w;
        int st = SET_OK;
        uint64_t o2p = 0, toff = field_table_off(f, k);
        if (pub) {
            if (L >= 5) {
                o2p = rd(m + 1, 4);
                if (o2p < L && m[o2p] == 1) st = SET_COMPLETE_BUFFER;
            }
        } else {
            if (L < 5) st = SET_INVALID_BUFFER;
            else {
                o2p = rd(m + 1, 4);
                if (o2p >= L || m[o2p] != 1) st = SET_PUBLIC_ONLY;
            }
            toff += o2p;
        }
        const uint8_t* v = sw ? val + (uint64_t)sw * i : val + (val_off ? val_off[i] : 0);
        const uint64_t vn = sw ? (uint64_t)sw : val_off[i + 1] - val_off[i];
        uint64_t size = L;
        if (st == SET_OK && L < toff + (sw ? (uint64_t)sw : 4)) st = SET_TOO_SHORT;
        if (st == SET_OK && !sw && vn % (uint64_t)ew) st = SET_BAD_LENGTH;
        if (st == SET_OK && sw) {          /* fixed: in place */
            memcpy(o, m, L);
            memcpy(o + toff, v, sw);
        } else if (st == SET_OK) {         /* payload field */
            uint64_t po = rd(m + toff, 4);
            if (!pub && po > 0) po += o2p;
            uint64_t oldn = 0;
            if (po > 0 && L >= po + 4) oldn = rd(m + po, 4);  /* bytes, or count */
            const uint64_t newn = vn / (uint64_t)ew;
            if (po > 0 && newn <= oldn) {  /* in place */
                if (L < po + 4 || (ew > 1 && L < po + 4 + vn)) st = SET_BOUNDS;  /* Go panics */
                else {
                    memcpy(o, m, L);
                    wr32(o + po, (uint32_t)newn);
                    const uint64_t c = vn < L - po - 4 ? vn : L - po - 4;  /* copy() stops at the end */
                    memcpy(o + po + 4, v, c);
                }
            } else {                       /* remarshal */
                const uint64_t pts = table_size(f, nf, 1);
                uint8_t* fake = NULL;
                int ust;
                if (pub && L + 1 + pts < 5) {  /* fakeComplete[1:5] is out of range: Go panics */
                    ust = -1;
                    st = SET_BOUNDS;
                } else if (pub) {  /* data + [0x01] + zeroed private table, offsetToPrivate = len(data) */
                    fake = (uint8_t*)calloc(L + 1 + pts + 16, 1);
                    memcpy(fake, m, L);
                    wr32(fake + 1, (uint32_t)L);  /* in Go's order: [1:5] first, then the marker */
                    fake[L] = 1;
                    ust = unmarshal_one(nf, f, fake, L + 1 + pts, fx, vp, vl);
                } else {
                    ust = unmarshal_one(nf, f, m, L, fx, vp, vl);
                }
                if (ust > 0) st = SET_UNMARSHAL;
                else if (ust == 0) {
                    vp[k] = v;
                    vl[k] = vn;
                    size = marshal_one(nf, f, fx, vp, vl, 0, 0, o);
                    if (pub) {
                        const uint32_t sid = L >= 13 ? (uint32_t)rd(m + 5, 4) : 0;
                        const uint32_t mid = L >= 13 ? (uint32_t)rd(m + 9, 4) : 0;
                        wr32(o + 5, sid);
                        wr32(o + 9, mid);
                        size = rd(o + 1, 4);  /* keep the public-only part */
                    }
                }
                free(fake);
            }
        }
        if (st != SET_OK) {
            memcpy(o, m, L);
            size = L;
        }
        status[i] = (uint8_t)st;
        w += size;
    }
    out_off[n] = w;
    return w;
}
