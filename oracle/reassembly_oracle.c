/*
 * reassembly_oracle.c -- CPU restatement of aRPC's receive-side reassembly of DataPacket fragments.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the HIP reassembler (arpc_amd/csrc/reassemble.hip).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * Parity status: the reference has no test of DataReassembler and is Go with no
 * toolchain here; this restatement is pinned by hand-derived known-answer cases in
 * tests/test_reassembly.py and by round trips through the packetizer oracle (fragment_oracle.c).
 *
 * What it restates (paths relative to the reference root), for datagrams in arrival order:
 *   UDPTransport.Receive: len < 1 -> error; type byte with no codec -> error; Error packets are
 *     not reassembled; DataPacketCodec.Deserialize errors drop the datagram
 *                                        pkg/transport/transport.go:253-317
 *   DataPacketCodec.Deserialize: >= 31 bytes, payload = data[31 : 31+PayloadLen] (trailing bytes
 *     ignored), "too short for declared payload length" otherwise
 *                                        pkg/packet/builtin_packets.go:118-161
 *   DataReassembler.ProcessFragment: one state per RPCID (request and response alike); a fragment
 *     overwrites any earlier one with the same (SeqNumber, FragmentIndex); MoreFragments = false
 *     marks the sequence's last fragment (lastFragmentIndex = max such index, from 0); the message
 *     completes when the number of distinct sequence numbers equals the ARRIVING packet's
 *     TotalPackets and every sequence 0..Total-1 has its last fragment and all indices
 *     0..lastFragmentIndex; it is then the payloads in (seq, index) order, the state is deleted and
 *     the message is returned with the completing packet
 *                                        pkg/transport/fragmentation.go:49-183
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define RX_CONSUMED 0   /* part of a completed message */
#define RX_PENDING 1    /* still held by the reassembler at the end of the batch */
#define RX_NOT_DATA 2   /* Error packet or a type with no codec: not reassembled */
#define RX_TOO_SHORT 3  /* len < 1, or < 31 for a DataPacket header */
#define RX_BAD_LENGTH 4 /* "data too short for declared payload length" */
#define HDR 31

typedef struct {
    uint64_t rpc;
    uint16_t total, seq;
    uint8_t more, fidx;
    uint64_t pay, plen; /* payload offset in the wire stream and length */
} Frag;

static uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* Parse datagram j; returns its status (RX_PENDING for a DataPacket). */
static int parse(const uint8_t* wire, const uint64_t* dg_off, uint64_t j, Frag* f) {
    const uint8_t* d = wire + dg_off[j];
    const uint64_t n = dg_off[j + 1] - dg_off[j];
    if (n < 1) return RX_TOO_SHORT;
    if (d[0] != 1 && d[0] != 2) return RX_NOT_DATA; /* Request / Response only (builtin_packets.go:13-18) */
    if (n < HDR) return RX_TOO_SHORT;
    uint64_t rpc = 0;
    for (int b = 0; b < 8; ++b) rpc |= (uint64_t)d[1 + b] << (8 * b);
    f->rpc = rpc;
    f->total = rd16(d + 9);
    f->seq = rd16(d + 11);
    f->more = d[13] != 0;
    f->fidx = d[14];
    f->plen = rd32(d + 27);
    if (n < HDR + f->plen) return RX_BAD_LENGTH;
    f->pay = dg_off[j] + HDR;
    return RX_PENDING;
}

typedef struct {
    uint64_t rpc;
    int used;
    int64_t* win; /* arrival indices in the current window, in arrival order */
    uint64_t nwin, capwin;
} Group;

typedef struct {
    Group* g;
    uint64_t size;
} Table;

static Group* lookup(Table* t, uint64_t rpc) {
    uint64_t h = (rpc * 0x9E3779B97F4A7C15ull) & (t->size - 1);
    while (t->g[h].used && t->g[h].rpc != rpc) h = (h + 1) & (t->size - 1);
    if (!t->g[h].used) {
        t->g[h].used = 1;
        t->g[h].rpc = rpc;
    }
    return &t->g[h];
}

/* The latest window entry with (seq, idx), or -1. */
static int64_t find(const Group* g, const Frag* fr, uint16_t seq, unsigned idx) {
    for (uint64_t a = g->nwin; a-- > 0;) {
        const Frag* f = &fr[g->win[a]];
        if (f->seq == seq && f->fidx == idx) return g->win[a];
    }
    return -1;
}

/* Completion check of fragmentation.go:96-133 on the window; fills last[s] for s < total. */
static int complete(const Group* g, const Frag* fr, uint16_t total, unsigned* last) {
    uint64_t distinct = 0;
    for (uint64_t a = 0; a < g->nwin; ++a) {
        uint64_t b = 0;
        while (b < a && fr[g->win[b]].seq != fr[g->win[a]].seq) ++b;
        distinct += b == a;
    }
    if (distinct != total) return 0;
    for (unsigned s = 0; s < total; ++s) {
        int seen = 0, has_last = 0;
        unsigned li = 0;
        for (uint64_t a = 0; a < g->nwin; ++a) {
            const Frag* f = &fr[g->win[a]];
            if (f->seq != s) continue;
            seen = 1;
            if (!f->more) {
                has_last = 1;
                if (f->fidx >= li) li = f->fidx;
            }
        }
        if (!seen || !has_last) return 0;
        for (unsigned i = 0; i <= li; ++i)
            if (find(g, fr, (uint16_t)s, i) < 0) return 0;
        last[s] = li;
    }
    return 1;
}

/* Reassembles n datagrams (wire + dg_off[n+1], arrival order).  Completed messages, in completion
 * order: bytes in msg (capacity: the payload bytes of the batch suffice), msg_off[nmsg+1], their
 * RPCID and the arrival index of the completing datagram.  status[n]: RX_*.  Returns nmsg. */
uint64_t sym_oracle_reassemble(uint64_t n, const uint8_t* wire, const uint64_t* dg_off, uint8_t* msg,
                               uint64_t* msg_off, uint64_t* msg_rpc, uint64_t* msg_dg, uint8_t* status) {
    Frag* fr = (Frag*)calloc(n ? n : 1, sizeof(Frag));
    Table t;
    t.size = 16;
    while (t.size < 2 * n) t.size <<= 1;
    t.g = (Group*)calloc(t.size, sizeof(Group));
    unsigned* last = (unsigned*)malloc(65536 * sizeof(unsigned));
    uint64_t nmsg = 0, w = 0;
    for (uint64_t j = 0; j < n; ++j) {
        status[j] = (uint8_t)parse(wire, dg_off, j, &fr[j]);
        if (status[j] != RX_PENDING) continue;
        Group* g = lookup(&t, fr[j].rpc);
        if (g->nwin == g->capwin) {
            g->capwin = g->capwin ? 2 * g->capwin : 4;
            g->win = (int64_t*)realloc(g->win, g->capwin * sizeof(int64_t));
        }
        g->win[g->nwin++] = (int64_t)j;
        if (!complete(g, fr, fr[j].total, last)) continue;
        msg_off[nmsg] = w;
        for (unsigned s = 0; s < fr[j].total; ++s)
            for (unsigned i = 0; i <= last[s]; ++i) {
                const Frag* f = &fr[find(g, fr, (uint16_t)s, i)];
                memcpy(msg + w, wire + f->pay, f->plen);
                w += f->plen;
            }
        msg_rpc[nmsg] = fr[j].rpc;
        msg_dg[nmsg] = j;
        ++nmsg;
        for (uint64_t a = 0; a < g->nwin; ++a) status[g->win[a]] = RX_CONSUMED;
        g->nwin = 0; /* delete(r.incoming, RPCID) */
    }
    msg_off[nmsg] = w;
    for (uint64_t h = 0; h < t.size; ++h) free(t.g[h].win);
    free(t.g);
    free(fr);
    free(last);
    return nmsg;
}
