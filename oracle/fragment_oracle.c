/*
 * fragment_oracle.c -- CPU restatement of aRPC's send-side packetization of Symphony data.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the HIP packetizer (arpc_amd/csrc/packetize.hip).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * Parity status: the production fragmenter has no test in the reference (its test file tests a
 * local copy that differs, cmd/symphony-gen-arpc/test/fragment_test.go:47-125 -- SURVEY.md 4),
 * and the reference is Go-only with no toolchain here, so this restatement is pinned only by the
 * hand-derived known-answer vectors in tests/test_fragment.py.
 *
 * What it restates (paths relative to the reference root):
 *   FragmentPackets(data, mtu)          pkg/transport/symphony_fragmentation.go:23-125
 *   the Send loop: effectiveMTU = MaxUDPPayloadSize - 31, one DataPacket per fragment with
 *     TotalPackets = uint16(#fragments), SeqNumber = uint16(index), MoreFragments = false,
 *     FragmentIndex = 0                 pkg/transport/transport.go:146-201
 *   DataPacketCodec.Serialize (31-byte header, little-endian)
 *                                       pkg/packet/builtin_packets.go:59-114
 */
#include <stdint.h>
#include <string.h>

#define FRAG_OK 0
#define FRAG_TOO_SHORT 1  /* "data too short for offset header" (symphony_fragmentation.go:33-35) */
#define FRAG_BAD_OFFSET 2 /* "invalid offset"                    (symphony_fragmentation.go:37-39) */
#define DATA_PACKET_HEADER 31

/* Fragment sizes of one record, in order; returns the count (or -status when Go returns an error).
 * sizes may be NULL (count only). */
static int64_t fragment_sizes(const uint8_t* data, uint64_t len, uint64_t mtu, uint64_t* sizes) {
    int64_t k = 0;
    if (len <= mtu) { /* :28-30 */
        if (sizes) sizes[0] = len;
        return 1;
    }
    if (len < 5) return -FRAG_TOO_SHORT; /* :33-35 */
    const uint64_t off2p = (uint64_t)data[1] | ((uint64_t)data[2] << 8) | ((uint64_t)data[3] << 16) |
                           ((uint64_t)data[4] << 24); /* :36 */
    if (off2p > len) return -FRAG_BAD_OFFSET;          /* :37-39 */
    const uint64_t pub = off2p, priv = len - off2p;
    uint64_t poff = 0;
    while (pub - poff > mtu) { /* :48-54 public packets */
        if (sizes) sizes[k] = mtu;
        ++k;
        poff += mtu;
    }
    const uint64_t meet = pub - poff;
    if (priv > 0) { /* :61-101 meeting packet(s) */
        const uint64_t head = priv % mtu;
        const uint64_t total = meet + head;
        if (total <= mtu) {
            if (sizes) sizes[k] = total;
            ++k;
        } else {
            if (sizes) {
                sizes[k] = mtu;
                sizes[k + 1] = total - mtu;
            }
            k += 2;
        }
        for (uint64_t rest = priv - head; rest > 0; rest -= mtu) { /* :111-122 private packets */
            if (sizes) sizes[k] = mtu;
            ++k;
        }
    } else if (meet > 0) { /* :102-107 */
        if (sizes) sizes[k] = meet;
        ++k;
    }
    return k;
}

static void put16(uint8_t* p, uint16_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
}
static void put32(uint8_t* p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
static void put64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

/* Plan: per record i, first[i] = datagrams before it, out_off[i] = wire bytes before it (payload
 * + 31 per datagram); [n] holds the totals.  status[i] = FRAG_*; failed records emit nothing
 * (Send returns the error before sending anything, transport.go:151-154). */
void sym_oracle_fragment_plan(uint64_t n, const uint8_t* in, const uint64_t* rec_off, uint32_t max_udp_payload,
                              uint64_t* first, uint64_t* out_off, uint8_t* status) {
    const uint64_t mtu = (uint64_t)max_udp_payload - DATA_PACKET_HEADER; /* transport.go:147-148 */
    uint64_t dg = 0, bytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t len = rec_off[i + 1] - rec_off[i];
        first[i] = dg;
        out_off[i] = bytes;
        const int64_t k = fragment_sizes(in + rec_off[i], len, mtu, NULL);
        status[i] = (uint8_t)(k < 0 ? -k : FRAG_OK);
        if (k > 0) {
            dg += (uint64_t)k;
            bytes += len + DATA_PACKET_HEADER * (uint64_t)k;
        }
    }
    first[n] = dg;
    out_off[n] = bytes;
}

/* Write every datagram (serialized DataPacket) back to back; dg_off[j] = start of datagram j,
 * dg_off[total] = total bytes.  addr = {dst_ip[4], dst_port (u16 LE), src_ip[4], src_port}. */
void sym_oracle_fragment_write(uint64_t n, const uint8_t* in, const uint64_t* rec_off, uint32_t max_udp_payload,
                               uint8_t packet_type, const uint64_t* rpc_id, const uint8_t* dst_ip, uint16_t dst_port,
                               const uint8_t* src_ip, uint16_t src_port, uint8_t* out, uint64_t* dg_off,
                               uint64_t* sizes_scratch) {
    const uint64_t mtu = (uint64_t)max_udp_payload - DATA_PACKET_HEADER;
    uint64_t pos = 0, dg = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* data = in + rec_off[i];
        const uint64_t len = rec_off[i + 1] - rec_off[i];
        const int64_t k = fragment_sizes(data, len, mtu, sizes_scratch);
        uint64_t src = 0;
        for (int64_t s = 0; s < k; ++s) {
            uint8_t* h = out + pos;
            const uint64_t fl = sizes_scratch[s];
            h[0] = packet_type;                   /* builtin_packets.go:78 */
            put64(h + 1, rpc_id[i]);              /* :79 */
            put16(h + 9, (uint16_t)k);            /* :80 TotalPackets = uint16(len(fragments)) */
            put16(h + 11, (uint16_t)s);           /* :81 SeqNumber = uint16(seqNum) */
            h[13] = 0;                            /* :84-88 MoreFragments = false */
            h[14] = 0;                            /* :91 FragmentIndex = 0 */
            memcpy(h + 15, dst_ip, 4);            /* :94 */
            put16(h + 19, dst_port);              /* :97 */
            memcpy(h + 21, src_ip, 4);            /* :100 */
            put16(h + 25, src_port);              /* :103 */
            put32(h + 27, (uint32_t)fl);          /* :106 */
            if (fl) memcpy(h + 31, data + src, fl); /* :109 */
            dg_off[dg++] = pos;
            pos += DATA_PACKET_HEADER + fl;
            src += fl;
        }
    }
    dg_off[dg] = pos;
}
