/*
 * raw_oracle.c -- CPU restatement of Symphony's zero-copy Raw getters and the proxy firewall element.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the HIP field extraction
 * (arpc_amd/csrc/raw_fields.hip).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg load it.
 *
 * Parity status: pinned by the known-answer values of the reference's own access-control test
 * (cmd/symphony-gen-arpc/test/serialization_test.go:555-703 on the Fixed message, whose
 * MarshalSymphony is cmd/symphony-gen-arpc/test/test.syn.go:152, restated byte by byte in
 * tests/test_raw_fields.py) and by hand-derived vectors; the reference is Go with no toolchain
 * here, so it is never run.
 *
 * What it restates (paths relative to the reference root):
 *   Raw getter of a fixed-width field (bool 1 byte, int32/uint32/float/enum 4, int64/uint64/double 8):
 *       `if len(m) < off+W { return 0 }; return LE(m[off:])`
 *                                       cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:1260-1294
 *   Raw getter of a string/bytes field: table entry = absolute (public) or private-segment-relative
 *       payload offset, 0 = unset; then a u32 length and the bytes, every step bounds-checked
 *                                       main.go:1517-1565
 *   private getters first assert a complete buffer (len >= 5, m[offsetToPrivate] == 0x01) and panic
 *       otherwise                       main.go:1003-1013
 *   table offsets: public fields from 13, private fields from 1 (relative to the private segment),
 *       advancing by the field width (fixed) or 4 (variable)   main.go:986-989, 1243-1257
 *   instance: GetRequestRaw.GetScore / GetUsername
 *                                       benchmark/kv-store-symphony-element/symphony/kv.syn.go:285-310
 *   FirewallElement.ProcessRequest: score := GetRequestRaw(payload).GetScore(); drop when
 *       score >= blockThreshold, else pass unchanged     cmd/proxy/element/firewall.go:34-52
 *   PacketVerdictPass = 1, PacketVerdictDrop = 2         cmd/proxy/util/packet.go:51-62
 *   element-schema MarshalSymphony (public Score + Username, private Key [+ Value]), used to build
 *       test inputs                     benchmark/kv-store-symphony-element/symphony/kv.syn.go:128-202,
 *                                       :1041-1124
 */
#include <stdint.h>
#include <string.h>

#define RAW_OK 0
#define RAW_INVALID_BUFFER 1 /* private getter panic: "called on invalid buffer" (len < 5) */
#define RAW_PUBLIC_ONLY 2    /* private getter panic: "called on public-only buffer" */
#define VERDICT_PASS 1
#define VERDICT_DROP 2

static uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static void wr32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

/* The private-getter assertion (main.go:1003-1013); sets *off2p when it holds. */
static int private_check(const uint8_t* m, uint64_t len, uint64_t* off2p) {
    if (len < 5) return RAW_INVALID_BUFFER;
    const uint64_t o = rd32(m + 1);
    if (o >= len || m[o] != 0x01) return RAW_PUBLIC_ONLY;
    *off2p = o;
    return RAW_OK;
}

/* One fixed-width getter; value zero-extended into *v (the caller reinterprets W bytes). */
static int get_fixed(const uint8_t* m, uint64_t len, int is_private, uint64_t table_off, unsigned width,
                     uint64_t* v) {
    *v = 0;
    uint64_t base = table_off;
    if (is_private) {
        uint64_t o = 0;
        const int st = private_check(m, len, &o);
        if (st != RAW_OK) return st;
        base = o + table_off; /* offsetToPrivate + tableOffset, main.go:1268 */
    }
    if (len < base + width) return RAW_OK; /* zero value, main.go:1272-1274 */
    uint64_t x = 0;
    for (unsigned b = 0; b < width; ++b) x |= (uint64_t)m[base + b] << (8 * b);
    *v = x;
    return RAW_OK;
}

/* One string/bytes getter: start and length of the value inside m (dlen 0 and start 0 when empty). */
static int get_bytes(const uint8_t* m, uint64_t len, int is_private, uint64_t table_off, uint64_t* start,
                     uint64_t* dlen) {
    *start = 0;
    *dlen = 0;
    uint64_t base = table_off, o = 0;
    if (is_private) {
        const int st = private_check(m, len, &o);
        if (st != RAW_OK) return st;
        base = o + table_off;
    }
    if (len < base + 4) return RAW_OK;  /* main.go:1528-1531 */
    uint64_t po = rd32(m + base);       /* :1534 */
    if (po == 0) return RAW_OK;         /* :1537-1539 unset */
    if (is_private) po += o;            /* :1542-1544 relative -> absolute */
    if (len < po + 4) return RAW_OK;    /* :1547-1549 */
    const uint64_t d = rd32(m + po);    /* :1550 */
    if (len < po + 4 + d) return RAW_OK; /* :1553-1555 */
    *start = po + 4;
    *dlen = d;
    return RAW_OK;
}

/* out: n values of `width` bytes (little-endian, width in {1, 4, 8}); status may be NULL. */
void sym_oracle_raw_fixed(uint64_t n, const uint8_t* in, const uint64_t* rec_off, int is_private, uint32_t table_off,
                          uint32_t width, void* out, uint8_t* status) {
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t v = 0;
        const int st = get_fixed(in + rec_off[i], rec_off[i + 1] - rec_off[i], is_private, table_off, width, &v);
        if (width == 1) ((uint8_t*)out)[i] = (uint8_t)v;
        else if (width == 4) ((uint32_t*)out)[i] = (uint32_t)v;
        else ((uint64_t*)out)[i] = v;
        if (status) status[i] = (uint8_t)st;
    }
}

/* out: the values back to back; out_off: n+1 offsets into out. */
void sym_oracle_raw_bytes(uint64_t n, const uint8_t* in, const uint64_t* rec_off, int is_private, uint32_t table_off,
                          uint8_t* out, uint64_t* out_off, uint8_t* status) {
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t s = 0, d = 0;
        const uint8_t* m = in + rec_off[i];
        const int st = get_bytes(m, rec_off[i + 1] - rec_off[i], is_private, table_off, &s, &d);
        out_off[i] = w;
        if (d) memcpy(out + w, m + s, d);
        w += d;
        if (status) status[i] = (uint8_t)st;
    }
    out_off[n] = w;
}

/* FirewallElement.ProcessRequest over n buffered requests: per request the score and verdict; the
 * passing requests, unchanged and in order, back to back in `kept` (kept_off: nkept+1 offsets,
 * kept_index: their positions in the input).  Returns nkept. */
uint64_t sym_oracle_firewall(uint64_t n, const uint8_t* in, const uint64_t* rec_off, uint32_t score_table_off,
                             int32_t block_threshold, int32_t* score, uint8_t* verdict, uint8_t* kept,
                             uint64_t* kept_off, uint64_t* kept_index) {
    uint64_t k = 0, w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* m = in + rec_off[i];
        const uint64_t len = rec_off[i + 1] - rec_off[i];
        uint64_t v = 0;
        (void)get_fixed(m, len, 0, score_table_off, 4, &v); /* GetScore, kv.syn.go:285-291 */
        const int32_t sc = (int32_t)(uint32_t)v;
        score[i] = sc;
        const int drop = sc >= block_threshold; /* shouldBlock, firewall.go:34-36 */
        verdict[i] = drop ? VERDICT_DROP : VERDICT_PASS;
        if (!drop) {
            kept_off[k] = w;
            kept_index[k] = i;
            if (len) memcpy(kept + w, m, len);
            w += len;
            ++k;
        }
    }
    kept_off[k] = w;
    return k;
}

/* Element-schema record size: header 13 + public table 8 + Username + private marker + table + payloads. */
uint64_t sym_oracle_element_size(int nprivate, uint64_t ulen, uint64_t klen, uint64_t vlen) {
    return 13 + 8 + 4 + ulen + 1 + 4 * (uint64_t)nprivate + 4 + klen + (nprivate == 2 ? 4 + vlen : 0);
}

/* {Get,Set}Request of the element schema: Score and Username public, Key (and Value) private
 * (kv.syn.go:1041-1124; GetRequest :128-202 is the same minus Value).  Returns the bytes written. */
uint64_t sym_oracle_marshal_element_batch(uint64_t n, int nprivate, const int32_t* score, const uint8_t* user,
                                          const uint64_t* user_off, const uint8_t* key, const uint64_t* key_off,
                                          const uint8_t* val, const uint64_t* val_off, uint8_t* out,
                                          uint64_t* out_off) {
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t ul = user_off[i + 1] - user_off[i], kl = key_off[i + 1] - key_off[i];
        const uint64_t vl = nprivate == 2 ? val_off[i + 1] - val_off[i] : 0;
        uint8_t* b = out + w;
        const uint64_t size = sym_oracle_element_size(nprivate, ul, kl, vl);
        memset(b, 0, size);
        const uint64_t pub = 13 + 4 + 4 + 4 + ul; /* publicSegmentSize, :1064-1068 */
        b[0] = 0x01;
        wr32(b + 1, (uint32_t)pub);
        wr32(b + 13, (uint32_t)score[i]);        /* Score, :1082-1083 */
        wr32(b + 17, 21);                        /* Username table entry: absolute payload offset */
        wr32(b + 21, (uint32_t)ul);
        if (ul) memcpy(b + 25, user + user_off[i], ul);
        b[pub] = 0x01;                           /* private version byte, :1094-1095 */
        const uint64_t tab = pub + 1, pay = tab + 4 * (uint64_t)nprivate;
        wr32(b + tab, (uint32_t)(pay - pub));    /* Key, relative to the private start, :1103-1108 */
        wr32(b + pay, (uint32_t)kl);
        if (kl) memcpy(b + pay + 4, key + key_off[i], kl);
        if (nprivate == 2) {                     /* Value, :1110-1115 */
            const uint64_t p2 = pay + 4 + kl;
            wr32(b + tab + 4, (uint32_t)(p2 - pub));
            wr32(b + p2, (uint32_t)vl);
            if (vl) memcpy(b + p2 + 4, val + val_off[i], vl);
        }
        out_off[i] = w;
        w += size;
    }
    out_off[n] = w;
    return w;
}
