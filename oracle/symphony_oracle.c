/*
 * symphony_oracle.c -- CPU restatement of aRPC's Symphony codec for flat schemas.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP codec in
 * arpc_amd/csrc.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product path (libsymphony_hip.so) never links or calls it.
 *
 * Parity status: pinned by known-answer vectors hand-derived from the generated Go
 * source (tests/golden/kats.json).  The reference is Go-only and no Go toolchain
 * exists in this image, so no reference-produced byte vectors exist; the
 * reference's own tests (cmd/symphony-gen-arpc/test/serialization_test.go:19-38)
 * pin round-trip invariance only.  See DESIGN.md "Oracle".
 *
 * What it restates (paths relative to the reference root):
 *   Marshal   benchmark/kv-store-symphony/symphony/kv.syn.go:611-678 (SetRequest),
 *             :74-132 (GetRequest), :333-391 (GetResponse), :963-1021 (SetResponse),
 *             examples/echo_symphony/symphony/echo.syn.go:111-184 (EchoRequest);
 *             generator cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:196-330
 *             (struct marshal), :439-469 (fixed fields), :471-491 (string fields).
 *   Unmarshal kv.syn.go:680-745, :134-185, echo.syn.go:186-263;
 *             generator main.go:622-694 (header checks), :734-793 (field decode).
 *   IDs       pkg/rpc/client.go:267-271 writes service/method IDs into [5:13].
 *
 * Schema model: `nfixed` int32 fields (declaration order, e.g. Echo Id, Score)
 * followed by `nvar` string/bytes fields.  No public fields (KV and echo have
 * none), so offset_to_private is always 13.
 *
 * Record layout (offsets absolute within the record):
 *   [0]      0x01 public version
 *   [1:5]    u32le offset_to_private = 13
 *   [5:9]    u32le service_id   (MarshalSymphony writes 0)
 *   [9:13]   u32le method_id    (MarshalSymphony writes 0)
 *   [13]     0x01 private version
 *   [14: ]   table: 4 B per fixed int32 value, then 4 B per var field holding the
 *            payload offset relative to 13
 *   payloads: per var field  u32le length, bytes
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define SYM_OK 0
#define SYM_ST_TOO_SHORT 1        /* "invalid data: too short"            */
#define SYM_ST_BAD_VERSION 2      /* "invalid data: wrong public version" */
#define SYM_ST_NO_PRIVATE 3       /* "missing private segment"            */
#define SYM_ST_FIELD_TOO_SHORT 4  /* "invalid data: too short for field"  */

static void put_u32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

static uint32_t get_u32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* Exact record size (generator main.go:1213-1239 size calculation):
 * 1 + 12 + 1 + table + sum(4 + len). */
uint64_t sym_oracle_record_size(int nfixed, int nvar, const uint64_t* lens) {
    uint64_t size = 14 + 4u * (uint64_t)(nfixed + nvar);
    for (int f = 0; f < nvar; ++f) size += 4 + lens[f];
    return size;
}

/* One record, exactly as the generated MarshalSymphony (kv.syn.go:611-678), plus
 * the client's in-place ID patch (client.go:267-271) when sid/mid are nonzero.
 * Returns the number of bytes written. */
uint64_t sym_oracle_marshal(int nfixed, int nvar, const int32_t* fixed, const uint8_t* const* field,
                            const uint64_t* lens, uint32_t sid, uint32_t mid, uint8_t* out) {
    uint64_t size = sym_oracle_record_size(nfixed, nvar, lens);
    memset(out, 0, size); /* make([]byte, size) zeroes */
    out[0] = 0x01;
    put_u32(out + 1, 13); /* publicSegmentSize = 13: no public fields */
    put_u32(out + 5, sid);
    put_u32(out + 9, mid);
    const uint64_t private_start = 13;
    out[private_start] = 0x01;
    const uint64_t table_start = private_start + 1;
    const uint64_t payload_start = table_start + 4u * (uint64_t)(nfixed + nvar);
    uint64_t payload_off = 0;
    for (int f = 0; f < nfixed; ++f) put_u32(out + table_start + 4u * f, (uint32_t)fixed[f]);
    for (int f = 0; f < nvar; ++f) {
        uint8_t* entry = out + table_start + 4u * (uint64_t)(nfixed + f);
        put_u32(entry, (uint32_t)((payload_start + payload_off) - private_start));
        put_u32(out + payload_start + payload_off, (uint32_t)lens[f]);
        if (lens[f]) memcpy(out + payload_start + payload_off + 4, field[f], lens[f]);
        payload_off += 4 + lens[f];
    }
    return size;
}

/* One record, exactly as the generated UnmarshalSymphony into a FRESH struct
 * (kv.syn.go:680-745; echo.syn.go:186-263).  Go `int` arithmetic is 64-bit, so
 * everything here is 64-bit and nothing wraps.
 *   fixed_out[f]  value of fixed field f, 0 if never assigned
 *   pos_out[f]    byte offset of var field f inside data (0 if skipped)
 *   len_out[f]    byte length of var field f (0 if skipped == Go "")
 * Returns the status code (0 = nil error). */
int sym_oracle_unmarshal(int nfixed, int nvar, const uint8_t* data, uint64_t len, int32_t* fixed_out,
                         uint64_t* pos_out, uint64_t* len_out) {
    for (int f = 0; f < nfixed; ++f) fixed_out[f] = 0;
    for (int f = 0; f < nvar; ++f) {
        pos_out[f] = 0;
        len_out[f] = 0;
    }
    if (len < 13) return SYM_ST_TOO_SHORT;                      /* main.go:647-649 */
    if (data[0] != 0x01) return SYM_ST_BAD_VERSION;             /* main.go:652-654 */
    const uint64_t off2p = get_u32(data + 1);                   /* main.go:657 */
    if (off2p >= len || data[off2p] != 0x01) return SYM_ST_NO_PRIVATE; /* main.go:662-664 */
    const uint64_t pts = off2p + 1; /* privateTableStart */
    uint64_t toff = 0;
    for (int f = 0; f < nfixed; ++f, toff += 4) {               /* main.go:734-745 */
        if (len < pts + toff + 4) return SYM_ST_FIELD_TOO_SHORT;
        fixed_out[f] = (int32_t)get_u32(data + pts + toff);
    }
    for (int f = 0; f < nvar; ++f, toff += 4) {                 /* main.go:765-793 */
        if (len >= pts + toff + 4) {
            uint64_t po = get_u32(data + pts + toff);
            if (po > 0) po += off2p;
            if (po > 0 && len >= po + 4) {
                uint64_t n = get_u32(data + po);
                if (len >= po + 4 + n) {
                    pos_out[f] = po + 4;
                    len_out[f] = n;
                }
            }
        }
    }
    return SYM_OK;
}

/* ---- batch forms: the same contract as the C-ABI in include/symphony_hip.h, on host memory ---- */

/* Encode n records.  Field f of record i is bytes[f][offs[f][i] .. offs[f][i+1]).
 * Writes the dense record stream to out and out_off[0..n] (out_off[0] = 0).
 * Returns the total number of bytes written. */
uint64_t sym_oracle_encode_batch(int nfixed, int nvar, uint64_t n, const int32_t* const* fixed_cols,
                                 const uint8_t* const* bytes, const uint64_t* const* offs, uint32_t sid,
                                 uint32_t mid, uint8_t* out, uint64_t* out_off) {
    uint64_t pos = 0;
    int32_t fx[8];
    const uint8_t* fp[8];
    uint64_t fl[8];
    for (uint64_t i = 0; i < n; ++i) {
        for (int f = 0; f < nfixed; ++f) fx[f] = fixed_cols[f][i];
        for (int f = 0; f < nvar; ++f) {
            fp[f] = bytes[f] + offs[f][i];
            fl[f] = offs[f][i + 1] - offs[f][i];
        }
        out_off[i] = pos;
        pos += sym_oracle_marshal(nfixed, nvar, fx, fp, fl, sid, mid, out + pos);
    }
    out_off[n] = pos;
    return pos;
}

/* Decode n records; record i is in[rec_off[i] .. rec_off[i+1]).  Decoded var
 * fields are packed densely: field f of record i lands at
 * bytes_out[f][offs_out[f][i] .. offs_out[f][i+1]), offs_out[f][0] = 0.
 * fixed_out may be NULL when nfixed == 0. */
void sym_oracle_decode_batch(int nfixed, int nvar, uint64_t n, const uint8_t* in, const uint64_t* rec_off,
                             int32_t* const* fixed_out, uint8_t* const* bytes_out, uint64_t* const* offs_out,
                             uint8_t* status) {
    uint64_t col[8] = {0};
    int32_t fx[8];
    uint64_t pos[8], ln[8];
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* rec = in + rec_off[i];
        const uint64_t len = rec_off[i + 1] - rec_off[i];
        status[i] = (uint8_t)sym_oracle_unmarshal(nfixed, nvar, rec, len, fx, pos, ln);
        for (int f = 0; f < nfixed; ++f) fixed_out[f][i] = fx[f];
        for (int f = 0; f < nvar; ++f) {
            offs_out[f][i] = col[f];
            if (ln[f]) memcpy(bytes_out[f] + col[f], rec + pos[f], ln[f]);
            col[f] += ln[f];
        }
    }
    for (int f = 0; f < nvar; ++f) offs_out[f][n] = col[f];
}

/* ---- mixed kv batches: GetRequest and SetRequest records in one batch ----
 * Record i is a GetRequest{Key} when type[i] == 0 (kv.syn.go:74-132 marshal, :134-185 unmarshal)
 * and a SetRequest{Key, Value} otherwise (:611-678, :680-745); the client's ID patch
 * (client.go:267-271) writes the method of the record's type (KVService: Get 1, Set 2,
 * kv_arpc.syn.go:25-28).  A GetRequest's value slice is not part of its record. */
uint64_t sym_oracle_encode_kv_mixed(uint64_t n, const uint8_t* type, const uint8_t* key, const uint64_t* key_off,
                                    const uint8_t* val, const uint64_t* val_off, uint32_t sid, uint32_t get_mid,
                                    uint32_t set_mid, uint8_t* out, uint64_t* out_off) {
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const int set = type[i] != 0;
        const uint8_t* fp[2] = {key + key_off[i], val + val_off[i]};
        const uint64_t fl[2] = {key_off[i + 1] - key_off[i], set ? val_off[i + 1] - val_off[i] : 0};
        out_off[i] = pos;
        pos += sym_oracle_marshal(0, set ? 2 : 1, NULL, fp, fl, sid, set ? set_mid : get_mid, out + pos);
    }
    out_off[n] = pos;
    return pos;
}

/* Each record unmarshalled as its type into a fresh struct; GetRequests leave the value column empty. */
void sym_oracle_decode_kv_mixed(uint64_t n, const uint8_t* in, const uint64_t* rec_off, const uint8_t* type,
                                uint8_t* key_out, uint64_t* key_off_out, uint8_t* val_out, uint64_t* val_off_out,
                                uint8_t* status) {
    uint64_t col[2] = {0, 0};
    uint8_t* outs[2] = {key_out, val_out};
    uint64_t* offs[2] = {key_off_out, val_off_out};
    int32_t fx[1];
    uint64_t pos[2], ln[2];
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* rec = in + rec_off[i];
        const uint64_t len = rec_off[i + 1] - rec_off[i];
        const int nv = type[i] != 0 ? 2 : 1;
        pos[1] = ln[1] = 0;
        status[i] = (uint8_t)sym_oracle_unmarshal(0, nv, rec, len, fx, pos, ln);
        for (int f = 0; f < 2; ++f) {
            offs[f][i] = col[f];
            if (ln[f]) memcpy(outs[f] + col[f], rec + pos[f], ln[f]);
            col[f] += ln[f];
        }
    }
    offs[0][n] = col[0];
    offs[1][n] = col[1];
}
