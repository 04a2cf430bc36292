// packetize.hip -- batched send-side packetization of Symphony records on gfx950.
//
// Restates, for n records at once, what aRPC's UDPTransport.Send does to one marshalled message
// (pkg/transport/transport.go:146-201): FragmentPackets(data, MaxUDPPayloadSize - 31)
// (pkg/transport/symphony_fragmentation.go:23-125) and one serialized DataPacket per fragment
// (pkg/packet/builtin_packets.go:59-114: 31-byte little-endian header, then the fragment), with
// TotalPackets = uint16(#fragments), SeqNumber = uint16(index), MoreFragments = 0,
// FragmentIndex = 0.  The output is every datagram back to back plus a datagram offset table:
// exactly the byte strings Send hands to WriteToUDP, in order.
//
// Fragments are consecutive slices of their record, so the wire stream is the record stream with
// a 31-byte header inserted before every fragment.  Two steps:
//  * plan: per record, its datagram count and wire bytes (a closed form of FragmentPackets from its
//    length and offset_to_private), then two device-wide exclusive scans (rocPRIM) -> each record's
//    first datagram index and wire offset;
//  * write: output-stationary like encode_kernel -- a wave owns 64 records, lane = aligned 16-byte
//    output chunk; a chunk is at most one datagram's tail plus the next one's header (datagrams are
//    >= 31 bytes), assembled from a per-record header template in LDS (SeqNumber and PayloadLen
//    patched in registers) and the payload's aligned source blocks, then one 16-byte store.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses memset

#include <rocprim/device/device_scan.hpp>

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

namespace frag {

constexpr int kHdr = 31;       // DataPacket header bytes (builtin_packets.go:68)
constexpr int kWaveRecs = 64;  // records per wave tile
constexpr int kWaves = 4;
constexpr int kSlot = 48;      // header template slot: 16 zero bytes, 31 header bytes, one zero byte

// Fragment layout of one record (FragmentPackets): kpub full public packets, nmeet (0-2) meeting
// packets of meet0 / meet1 bytes, then full private packets; M = payload bytes per datagram.
struct Layout {
    u64 kpub, nmeet, meet0, meet1, npk;
};

__host__ __device__ inline bool layout_of(u64 L, u64 off2p, u64 M, Layout& o) {
    o = Layout{0, 1, L, 0, 1};
    if (L <= M) return true;  // symphony_fragmentation.go:28-30: the whole record, one packet
    if (off2p > L) return false;  // :37-39 "invalid offset"
    const u64 pub = off2p, priv = L - off2p;
    o.kpub = pub > M ? (pub - 1) / M : 0;  // :48-54: full packets while more than M remain
    const u64 meet = pub - o.kpub * M;
    if (priv > 0) {  // :61-101
        const u64 head = priv % M, tot = meet + head;
        if (tot <= M) {
            o.nmeet = 1;
            o.meet0 = tot;
        } else {
            o.nmeet = 2;
            o.meet0 = M;
            o.meet1 = tot - M;
        }
        o.npk = o.kpub + o.nmeet + (priv - head) / M;  // :111-122
    } else {  // :102-107
        o.nmeet = meet > 0 ? 1 : 0;
        o.meet0 = meet;
        o.npk = o.kpub + o.nmeet;
    }
    return true;
}

// Fragment d's payload start (within the record) and length.
__device__ inline void frag_of(const Layout& l, u64 M, u64 d, u64& start, u64& len) {
    if (d < l.kpub) {
        start = d * M;
        len = M;
    } else if (d < l.kpub + l.nmeet) {
        const bool second = d > l.kpub;
        start = l.kpub * M + (second ? l.meet0 : 0);
        len = second ? l.meet1 : l.meet0;
    } else {
        start = l.kpub * M + l.meet0 + l.meet1 + (d - l.kpub - l.nmeet) * M;
        len = M;
    }
}

// q / D for q < 2^31 (tile positions are 32-bit) and D < 2^32: a 32-bit division, not a 64-bit one.
__device__ inline u64 div_small(u64 q, u64 D) { return (u64)((u32)q / (u32)D); }

// The datagram holding wire byte q (>= 0, < 2^31) of the record's datagram sequence.
__device__ inline u64 dgram_at(const Layout& l, u64 M, u64 q) {
    const u64 D = M + kHdr, A = l.kpub * D;
    if (q < A) return div_small(q, D);
    q -= A;
    if (l.nmeet >= 1) {
        if (q < l.meet0 + kHdr) return l.kpub;
        q -= l.meet0 + kHdr;
    }
    if (l.nmeet == 2) {
        if (q < l.meet1 + kHdr) return l.kpub + 1;
        q -= l.meet1 + kHdr;
    }
    const u64 d = l.kpub + l.nmeet + div_small(q, D);
    return d < l.npk ? d : l.npk - 1;
}

__device__ inline u64 record_off2p(const uint8_t* rec, u64 L, u64 M) {
    if (L <= M || L < 5) return 0;  // not needed / "too short" decided by the caller
    return (u64)rec[1] | ((u64)rec[2] << 8) | ((u64)rec[3] << 16) | ((u64)rec[4] << 24);
}

// ---- plan: per-record datagram count and wire bytes (inputs of the two scans)
__global__ __launch_bounds__(256) void frag_count_kernel(const uint8_t* in, const u64* rec_off, u64 n, u64 M,
                                                         u64* cnt, u64* bytes, uint8_t* status) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i > n) return;
    if (i == n) {  // scan inputs have n+1 entries: the last exclusive prefix is the total
        cnt[n] = 0;
        bytes[n] = 0;
        return;
    }
    const u64 s = rec_off[i], L = rec_off[i + 1] - s;
    uint8_t st = SYM_FRAG_OK;
    Layout l;
    if (L > M && L < 5) {
        st = SYM_FRAG_TOO_SHORT;  // :33-35 "data too short for offset header"
    } else if (!layout_of(L, record_off2p(in + s, L, M), M, l)) {
        st = SYM_FRAG_BAD_OFFSET;
    }
    status[i] = st;
    cnt[i] = st == SYM_FRAG_OK ? l.npk : 0;
    bytes[i] = st == SYM_FRAG_OK ? L + kHdr * l.npk : 0;
}

// ---- write
// 5.1 KiB per wave (7 workgroups per CU; 7.5 KiB with 64-byte slots and u64 layouts gave 5).  A
// header window reads up to 15 bytes past its slot: the next slot's leading zeros, or `pad`.
struct WaveLds {
    char tmpl[kWaveRecs * kSlot + 16];  // per record: 16 zero bytes, the 31-byte header (seq = len = 0), a zero
    int o[kWaveRecs + 1];               // record's wire start relative to the tile; [cnt] = span
    u32 kpub[kWaveRecs], nmeet[kWaveRecs], meet0[kWaveRecs], meet1[kWaveRecs], npk[kWaveRecs];  // < 2^31: tile check
    u64 addr[kWaveRecs];                // record's first byte (address)
};

struct WriteParams {
    const uint8_t* in;
    const u64* rec_off;
    u64 n;
    u64 M;
    uint8_t type;
    const u64* rpc_id;
    uint8_t dst_ip[4], src_ip[4];
    uint16_t dst_port, src_port;
    const u64* first;
    const u64* out_off;
    const uint8_t* status;
    uint8_t* out;
    u64* dg_off;
    unsigned* err;
};

__global__ __launch_bounds__(kWaves * 64) void frag_write_kernel(WriteParams p) {
    __shared__ WaveLds lds_all[kWaves];
    __shared__ MaskTable masks;
    mask_table_init(masks, threadIdx.x);
    __syncthreads();  // the only workgroup barrier
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    WaveLds& S = lds_all[wave];
    const u64 r0 = ((u64)blockIdx.x * kWaves + wave) * kWaveRecs;
    if (r0 >= p.n) return;  // wave-uniform
    const int cnt = (int)min((u64)kWaveRecs, p.n - r0);
    const u64 T0 = p.out_off[r0], T1 = p.out_off[r0 + cnt];  // uniform
    if (T1 - T0 >= ((u64)1 << 31)) {  // tile positions are 32-bit
        if (lane == 0) atomicOr(p.err, kErrTooLarge);
        return;
    }
    const u64 M = p.M;

    // ---- phase 1 (lane = record): layout, header template, datagram offsets
    if (lane < cnt) {
        const u64 r = r0 + lane;
        const u64 s = p.rec_off[r], L = p.rec_off[r + 1] - s;
        Layout l{0, 0, 0, 0, 0};
        if (p.status[r] == SYM_FRAG_OK) layout_of(L, record_off2p(p.in + s, L, M), M, l);
        const u64 O = p.out_off[r];
        S.o[lane] = (int)(O - T0);
        if (lane == cnt - 1) S.o[cnt] = (int)(T1 - T0);
        S.kpub[lane] = l.kpub;
        S.nmeet[lane] = l.nmeet;
        S.meet0[lane] = l.meet0;
        S.meet1[lane] = l.meet1;
        S.npk[lane] = l.npk;
        S.addr[lane] = (u64)(uintptr_t)(p.in + s);
        // header template (builtin_packets.go:78-106), SeqNumber and PayloadLen left 0
        u32 h[kSlot / 4];
#pragma unroll
        for (int k = 0; k < kSlot / 4; ++k) h[k] = 0;
        const u64 id = p.rpc_id[r];
        img_put_u8<16 + 0>(h, p.type);
        img_put_u32<16 + 1>(h, (u32)id);
        img_put_u32<16 + 5>(h, (u32)(id >> 32));
        img_put_u32<16 + 9>(h, (u32)(uint16_t)l.npk);  // TotalPackets = uint16(len(fragments))
        img_put_u32<16 + 15>(h, (u32)p.dst_ip[0] | ((u32)p.dst_ip[1] << 8) | ((u32)p.dst_ip[2] << 16) |
                                    ((u32)p.dst_ip[3] << 24));
        img_put_u32<16 + 19>(h, (u32)p.dst_port);
        img_put_u32<16 + 21>(h, (u32)p.src_ip[0] | ((u32)p.src_ip[1] << 8) | ((u32)p.src_ip[2] << 16) |
                                    ((u32)p.src_ip[3] << 24));
        img_put_u32<16 + 25>(h, (u32)p.src_port);
        uint2* slot = (uint2*)&S.tmpl[lane * kSlot];
#pragma unroll
        for (int k = 0; k < kSlot / 8; ++k) slot[k] = make_uint2(h[2 * k], h[2 * k + 1]);
        // datagram offset table: datagram j of the batch starts at dg_off[j]
        const u64 f0 = p.first[r];
        for (u64 d = 0; d < l.npk; ++d) {
            u64 fs, fl;
            frag_of(l, M, d, fs, fl);
            p.dg_off[f0 + d] = O + fs + kHdr * d;
        }
        if (r == p.n - 1) p.dg_off[p.first[p.n]] = p.out_off[p.n];
    } else {  // a slot past the tile's last record: its leading zeros end the last record's windows
        uint2* slot = (uint2*)&S.tmpl[lane * kSlot];
        slot[0] = slot[1] = make_uint2(0, 0);
    }
    if (lane == 0) ((uint2*)&S.tmpl[kWaveRecs * kSlot])[0] = ((uint2*)&S.tmpl[kWaveRecs * kSlot])[1] = make_uint2(0, 0);
    wave_sync();

    // ---- phase 2 (lane = aligned 16-byte wire chunk)
    const int span = (int)(T1 - T0);
    const i64 mis = (i64)((uintptr_t)p.out & 15);
    const int firstc = (int)((((i64)T0 + mis) & ~(i64)15) - mis - (i64)T0);  // in (-16, 0]
    uint8_t* const out_t = p.out + T0;
    // A 16-byte payload window reads up to 31 bytes before its fragment and 15 after: inside the
    // stream unless the tile sits within 32 bytes of the stream's ends (batch edges).
    const u64 s_lo = p.rec_off[0], s_hi = p.rec_off[p.n];
    const bool tile_safe = p.rec_off[r0] >= s_lo + 32 && p.rec_off[r0 + cnt] + 16 <= s_hi;
    const uintptr_t dummy = (uintptr_t)p.in & ~(uintptr_t)15;  // any readable block; its bytes are masked off
    // header window at datagram byte b in [-16, 31) of record k's template, with seq / len patched
    auto header_window = [&](int k, int b, u64 seq, u64 flen) -> u32x4 {
        u32x4 v = lds16u(S.tmpl, k * kSlot + 16 + b);
        u32 t[4] = {v.x, v.y, v.z, v.w};
        if (11 - b > -4 && 11 - b < 16) or_u32_at((u32)(uint16_t)seq, 11 - b, t);  // SeqNumber
        if (27 - b > -4 && 27 - b < 16) or_u32_at((u32)flen, 27 - b, t);           // PayloadLen
        return u32x4{t[0], t[1], t[2], t[3]};
    };
    // the wire chunk at tile position P (aligned 16 bytes): header bytes from the templates, payload
    // bytes from one byte-unaligned load
    auto chunk = [&](int P) -> u32x4 {
        const int k = lds_search_64(S.o, cnt, max(P, 0));
        const Layout l{S.kpub[k], S.nmeet[k], S.meet0[k], S.meet1[k], S.npk[k]};
        const i64 q = (i64)P - S.o[k];  // >= -15
        const u64 d = q < 0 ? 0 : dgram_at(l, M, (u64)q);
        u64 fs, fl;
        frag_of(l, M, d, fs, fl);
        const i64 h0 = (i64)(fs + kHdr * d);  // datagram start within the record's wire bytes
        const int b = (int)(q - h0);          // chunk start within the datagram, >= -15
        u32x4 r = {0, 0, 0, 0};
        if (b < kHdr) r = header_window(k, b, d, fl);
        {  // payload bytes of this datagram inside the chunk: chunk offsets [kHdr - b, kHdr + fl - b)
            const int lo = max(kHdr - b, 0);
            const int hi = (int)min((i64)kHdr + (i64)fl - b, (i64)16);
            const uintptr_t X0 = (uintptr_t)(S.addr[k] + fs) + (uintptr_t)(i64)(b - kHdr);  // chunk byte t <- X0 + t
            if (tile_safe) {  // one byte-unaligned load, unconditional (no wait until the store)
                const u32x4 w = ld16u(lo < hi ? X0 : dummy);
                r |= w & range_mask(masks, lo, hi);
            } else if (lo < hi) {  // batch-edge tiles: only the aligned blocks holding payload bytes
                u32 t[4] = {r.x, r.y, r.z, r.w};
                or_window_global(X0, lo, hi, t);
                r = u32x4{t[0], t[1], t[2], t[3]};
            }
        }
        const i64 end = h0 + kHdr + (i64)fl;  // this datagram's end within the record
        if (q + 16 > end) {  // the next datagram's header starts inside this chunk
            int k2 = k;
            u64 d2 = d + 1;
            if (d2 >= l.npk) {  // first datagram of the next record that has any
                k2 = k + 1;
                while (k2 < cnt && S.npk[k2] == 0) ++k2;
                d2 = 0;
            }
            if (k2 < cnt) {
                const Layout l2{S.kpub[k2], S.nmeet[k2], S.meet0[k2], S.meet1[k2], S.npk[k2]};
                u64 fs2, fl2;
                frag_of(l2, M, d2, fs2, fl2);
                r |= header_window(k2, (int)(end - q) * -1, d2, fl2);
            }
        }
        return r;
    };
    // kU chunks per lane per step: every load of the step is issued before its stores
    constexpr int kU = 4;
    for (int B = firstc; B < span; B += 16 * 64 * kU) {  // wave-uniform loop
        u32x4 r[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int P = B + 16 * 64 * u + 16 * lane;
            r[u] = P < span ? chunk(P) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int P = B + 16 * 64 * u + 16 * lane;
            if (P >= span) continue;
            const u32 rr[4] = {r[u].x, r[u].y, r[u].z, r[u].w};
            store_chunk(out_t, P, 0, span, rr, true);  // (nontemporal: measured on, DESIGN.md section 4 Stores)
        }
    }
}

}  // namespace frag

size_t frag_scan_temp_bytes(uint64_t n) {
    size_t bytes = 0;
    (void)rocprim::exclusive_scan(nullptr, bytes, (const u64*)nullptr, (u64*)nullptr, (u64)0, (size_t)n + 1,
                                  rocprim::plus<u64>());
    return (bytes + 255) & ~(size_t)255;
}

hipError_t launch_frag_plan(const uint8_t* in, const u64* rec_off, u64 n, u64 M, u64* cnt, u64* bytes,
                            u64* first, u64* out_off, uint8_t* status, void* temp, size_t temp_bytes,
                            hipStream_t stream) {
    hipLaunchKernelGGL(frag::frag_count_kernel, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, stream, in,
                       rec_off, n, M, cnt, bytes, status);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = temp_bytes;
    e = rocprim::exclusive_scan(temp, tb, (const u64*)cnt, first, (u64)0, (size_t)n + 1, rocprim::plus<u64>(), stream);
    if (e != hipSuccess) return e;
    tb = temp_bytes;
    return rocprim::exclusive_scan(temp, tb, (const u64*)bytes, out_off, (u64)0, (size_t)n + 1, rocprim::plus<u64>(),
                                   stream);
}

hipError_t launch_frag_write(const FragWriteArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    frag::WriteParams p{};
    p.in = a.in;
    p.rec_off = a.rec_off;
    p.n = a.n;
    p.M = a.M;
    p.type = a.type;
    p.rpc_id = a.rpc_id;
    for (int i = 0; i < 4; ++i) {
        p.dst_ip[i] = a.dst_ip[i];
        p.src_ip[i] = a.src_ip[i];
    }
    p.dst_port = a.dst_port;
    p.src_port = a.src_port;
    p.first = a.first;
    p.out_off = a.out_off;
    p.status = a.status;
    p.out = a.out;
    p.dg_off = a.dg_off;
    p.err = a.err;
    const u64 tiles = (a.n + frag::kWaveRecs - 1) / frag::kWaveRecs;
    hipLaunchKernelGGL(frag::frag_write_kernel, dim3((unsigned)((tiles + frag::kWaves - 1) / frag::kWaves)),
                       dim3(frag::kWaves * 64), 0, stream, p);
    return hipGetLastError();
}

}  // namespace symhip
