// reassemble.hip -- batched receive-side reassembly of aRPC DataPackets on gfx950.
//
// Restates, for n datagrams received in a given order, what UDPTransport.Receive
// (pkg/transport/transport.go:253-317) + DataPacketCodec.Deserialize (pkg/packet/builtin_packets.go:
// 118-161) + DataReassembler.ProcessFragment (pkg/transport/fragmentation.go:49-183) return one call
// at a time: every completed message, in completion order, with its RPCID and completing datagram,
// plus each datagram's fate (consumed by a message, still pending, or dropped by the parser).
//
// The reassembler keeps one state per RPCID and its decisions for one RPCID depend only on that
// RPCID's datagrams in arrival order, so the batch is regrouped rather than replayed:
//  1. parse (thread per datagram): header checks; then the RPCID inserted into an open-addressing
//     hash table (agent-scope CAS), whose claiming arrival's index is the group key -- or, when the
//     RPCIDs never decrease, the run head -- so groups sort roughly in order of appearance and an
//     in-order stream keeps its arrival order through every later pass (coalesced);
//  2. a stable LSD radix sort of (group key, arrival index) on ~log2(n)+1 key bits, 8 bits a pass
//     (sort_*_kernel below): each group becomes a contiguous run in arrival order;
//  3. group pass (thread per group): the ProcessFragment state machine over the group's run, with
//     per-sequence state (fragment-index bitmap, last index, latest index-0 fragment) in a scratch
//     slice owned by the group, O(1) work per datagram; it records, at each completing datagram,
//     the message's (bytes, segments, 1);
//  4. an exclusive scan of those triples in ARRIVAL order gives every message its index, byte
//     offset and first segment -- completion order across RPCIDs is arrival order of the
//     completing datagrams, as in the one-at-a-time loop;
//  5. the group pass again, now writing message offsets / RPCIDs / completing datagrams and the
//     message's payload segments (wire offset, length) in (seq, fragment index) order;
//  6. the segment gather of raw_fields.hip copies the payloads into the message stream.
// Most batches are "simple" (every DataPacket one whole message) or packetizer "runs" (parse_kernel)
// and finish after step 1 with an emit and the gather.  The call never waits on the host: steps 1a-6
// are queued for every batch and each of their kernels reads the parse's device flags first and
// exits at once for those (the stream stays asynchronous and capturable).

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"
#include "gather_tile.hpp"

#include <algorithm>

namespace symhip {

namespace rx {

using raw::Pair;

constexpr int kHdr = 31;        // DataPacket header (builtin_packets.go:68)
constexpr u64 kEmpty = ~0ull;   // free hash slot; an RPCID equal to it gets the table slot `special`
constexpr u32 kNoSlot = ~0u;    // slot of a datagram that is not a DataPacket

struct SeqState {    // one sequence number of the group's current message
    u32 bits[8];     // fragment indices received (0..255)
    u32 latest0;     // arrival index of the latest fragment with index 0
    u32 flags;       // 1 seen, 2 has its last fragment, 4 complete; lastFragmentIndex << 8
};

__device__ inline u64 mix64(u64 x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// meta: seq | total << 16 | more << 32 | fragment index << 40
__device__ inline u32 m_seq(u64 m) { return (u32)(m & 0xffff); }
__device__ inline u32 m_total(u64 m) { return (u32)((m >> 16) & 0xffff); }
__device__ inline bool m_more(u64 m) { return (m >> 32) & 1; }
__device__ inline u32 m_fidx(u64 m) { return (u32)((m >> 40) & 0xff); }

struct Args {
    const uint8_t* wire;
    const u64* dg_off;
    u64 n;
    u64* table;
    u64 tmask;
    u32 special, nodata;   // table slot of the RPCID == kEmpty; group key of non-DataPackets (= n)
    u32* first;            // per table slot (+1 for `special`): the group key, the claiming arrival's index
    u32* slot;             // per datagram: its RPCID's table slot
    u64* rpc;
    u64* meta;
    u32* plen;
    u32* gid;
    u32* idx;
    const u32* gs;         // sorted group keys / arrival indices (gid / idx themselves when the
    const u32* is;         // keys came out non-decreasing: *unsorted == 0 and the sort did nothing)
    unsigned* unsorted;       // (sharded flag words, flag_set)
    const unsigned* nonmono;  // not every datagram a DataPacket with RPCIDs non-decreasing: hash them
    unsigned* gen;            // single words written by emit_kernel: the general path runs; nonmono
    unsigned* nm;
    SeqState* state;
    uint8_t* status;
    Pair* cnt;             // per arrival (n+1): (message bytes, segments << 32 | messages)
    Pair* agg;             // its tile totals (simple batches: written by parse_kernel)
    Pair* super_p;         // their two-level group totals (gather_tile.hpp publish_tile_total): the parse's
    Pair* agg_c;           // the general path's tile totals of the triples (added up by group pass 0)
    Pair* super_c;         // and their group totals
    const Pair* pre;       // its exclusive scan
    u64* msg_off;
    u64* msg_rpc;
    u64* msg_dg;
    u64* seg_src;
    u64* seg_len;
    Pair* seg_pre;         // the segment gather's tile prefixes (the general path's): written where the
                           // segments are, see emit_kernel
};

__device__ inline void block_scan_pair(Pair v, Pair& excl, Pair& tile_total);
__host__ __device__ inline u64 tiles(u64 m) { return (m + 255) / 256; }

// The batch's flag words, each in kShards copies on lines of their own (flag w of shard s at flags[32 s
// + w], all zeroed per call): [0] not simple, [1] keys out of order (key_kernel), [2] not every
// datagram a DataPacket with RPCIDs non-decreasing, [3] a run that is not the packetizer's.  A
// workgroup raises a flag in its own shard (blockIdx % kShards), and a reader ORs the shards.  (Round
// 6: with one word per flag the ~2000 workgroups resident at once all found it clear and all
// atomically set it, serialised at the memory side: ~17 us in key_kernel and ~20 in the parse of a
// batch that sets a flag everywhere.)  The general path's kernels run only for a batch that is
// neither simple nor runs (emit_kernel), i.e. [0] && ([2] || [3]) (uniform).
constexpr int kShards = 16;
constexpr size_t kFlagBytes = kShards * 128;
__device__ __forceinline__ bool flag_set(const unsigned* w) {  // w: flag word of shard 0
    unsigned v = 0;
#pragma unroll
    for (int s = 0; s < kShards; ++s) v |= w[32 * s];
    return v != 0;
}
__device__ __forceinline__ void flag_raise(unsigned* w, bool any) {  // whole workgroup; the atomic only while clear
    if (__syncthreads_or(any) && threadIdx.x == 0) {
        unsigned* p = w + 32 * (blockIdx.x % kShards);
        if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) atomicOr(p, 1u);
    }
}
// The general path's later kernels read one word instead, `gen` (and `nm`, flag [2]), which its first
// launch (init_kernel) writes from the shards: an empty launch of a single-datagram or runs batch
// then costs one load per workgroup, not 16-48 (those launches run beside the payload copy and take
// CU slots from it while they last).
__device__ __forceinline__ bool gated_off(const unsigned* gate) { return *gate == 0; }

// ---- 1a'. the hash table set to "empty" (general path, RPCIDs out of order)
// (The general path's first launch: it also writes the gate words from the parse's flag shards.)
__global__ __launch_bounds__(256) void init_kernel(u64* table, u32* first, u64 ts, const unsigned* flags,
                                                   unsigned* gen, unsigned* nm) {
    const bool nonmono = flag_set(flags + 2), general = flag_set(flags) && (nonmono || flag_set(flags + 3));
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // read by the general path's later launches
        *gen = general;
        *nm = nonmono;
    }
    if (!general || !nonmono) return;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < ts; i += (u64)gridDim.x * 256) table[i] = kEmpty;
    if (blockIdx.x == 0 && threadIdx.x == 0) first[ts] = ~0u;  // (the special slot's key; the others are
                                                               // written by the CAS that claims the slot)
}

// When every datagram is a DataPacket and the RPCIDs never decrease, each RPCID's datagrams form one
// contiguous run, so its group is that run and its first arrival the run's head: the hash table (and
// the sort, the keys being in order) is not needed.  The parse finds out (round 6: before, a launch of
// its own); the hash and key kernels branch on its word (the packetizer's send order and one client's
// increasing RPCIDs are this case).

// ---- 2. stable LSD radix sort of (key, value) u32 pairs, 8 key bits per pass, 2048 pairs a tile.
// A pass: per-tile digit counts (digit-major, so a row scan per digit gives every tile its offset
// inside the digit), the row scans, then the scatter: a tile's pairs in order -- wave w takes its
// 512, eight steps of 64 -- ranked among equal digits by a ballot match inside the wave and a
// running per-wave count in LDS, then offset by the earlier waves' counts, the tile's offset and
// the digit's start.  Every kernel is gated (general path only).
constexpr int kSortTile = 2048;
constexpr int kSortWaveItems = kSortTile / 4;
constexpr int kDigits = 256;

// lanes of the wave whose digit equals this lane's (among lanes with `valid`)
__device__ __forceinline__ u64 match_digit(u32 d, bool valid) {
    u64 m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const u64 bal = __ballot(valid && ((d >> b) & 1u));
        m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    return m;
}

__device__ __forceinline__ u32 rank_below(u64 m) {
    return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
}

__device__ __forceinline__ void sort_hist_tile(const u32* keys, u64 n, int shift, u32* hist, u64 ntiles, u64 tile) {
    __shared__ u32 h[kDigits];
    h[threadIdx.x] = 0;
    __syncthreads();
    const u64 base = tile * kSortTile;
    for (int k = 0; k < kSortTile / 256; ++k) {
        const u64 j = base + (u64)k * 256 + threadIdx.x;
        const bool valid = j < n;
        const u32 d = valid ? (keys[j] >> shift) & (kDigits - 1) : 0u;
        const u64 m = match_digit(d, valid);
        if (valid && rank_below(m) == 0) atomicAdd(&h[d], (u32)__popcll(m));  // one add per digit and wave
    }
    __syncthreads();
    hist[(u64)threadIdx.x * ntiles + tile] = h[threadIdx.x];
}

__global__ __launch_bounds__(256) void sort_hist_kernel(const u32* keys, u64 n, int shift, u32* hist, u64 ntiles,
                                                        const unsigned* gen, const unsigned* unsorted) {
    if (gated_off(gen) || !flag_set(unsorted)) return;
    sort_hist_tile(keys, n, shift, hist, ntiles, blockIdx.x);
}

// block-wide exclusive scan of one u32 per thread (256 threads)
__device__ __forceinline__ u32 block_excl_u32(u32 v, u32& total) {
    __shared__ u32 ws[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u32 inc = wave_incl_scan_u32(v, lane);
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    u32 pre = 0;
    for (int q = 0; q < wave; ++q) pre += ws[q];
    total = ws[0] + ws[1] + ws[2] + ws[3];
    __syncthreads();
    return pre + inc - v;
}

__device__ __forceinline__ void sort_rowscan_row(u32* hist, u64 ntiles, u32* rowtot, int digit) {
    u32* row = hist + (u64)digit * ntiles;
    u32 carry = 0;
    for (u64 b = 0; b < ntiles; b += 256) {  // uniform loop
        const u64 i = b + threadIdx.x;
        const u32 v = i < ntiles ? row[i] : 0u;
        u32 tot;
        const u32 ex = block_excl_u32(v, tot);
        if (i < ntiles) row[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) rowtot[digit] = carry;
}

__global__ __launch_bounds__(256) void sort_rowscan_kernel(u32* hist, u64 ntiles, u32* rowtot, const unsigned* gen,
                                                           const unsigned* unsorted) {
    if (gated_off(gen) || !flag_set(unsorted)) return;
    sort_rowscan_row(hist, ntiles, rowtot, blockIdx.x);
}

__device__ __forceinline__ void sort_scatter_tile(const u32* kin, const u32* vin, u32* kout, u32* vout, u64 n, int shift,
                                                  const u32* hist, u64 ntiles, const u32* rowtot, u64 tile) {
    __shared__ u32 cnt[4][kDigits];  // per wave: running count of each digit, then its output base
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32 tot;
    const u32 dstart = block_excl_u32(rowtot[threadIdx.x], tot);  // the digit's first output position
    const u32 tbase = dstart + hist[(u64)threadIdx.x * ntiles + tile];
#pragma unroll
    for (int w = 0; w < 4; ++w) cnt[w][threadIdx.x] = 0;
    __syncthreads();
    constexpr int kSteps = kSortWaveItems / 64;
    u32 key[kSteps], val[kSteps], pos[kSteps];
    const u64 base = tile * kSortTile + (u64)wave * kSortWaveItems;
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
        const u64 j = base + (u64)k * 64 + lane;
        const bool valid = j < n;
        key[k] = valid ? kin[j] : 0u;
        val[k] = valid ? vin[j] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {  // in order: the rank is stable
        const bool valid = base + (u64)k * 64 + lane < n;
        const u32 d = (key[k] >> shift) & (kDigits - 1);
        const u64 m = match_digit(d, valid);
        const u32 r = rank_below(m);
        pos[k] = valid ? cnt[wave][d] + r : 0u;
        wave_sync();  // every lane has read its digit's count before the leaders advance it
        if (valid && r == 0) cnt[wave][d] += (u32)__popcll(m);
        wave_sync();
    }
    __syncthreads();
    {  // per digit: the waves' counts -> their output bases
        const int d = threadIdx.x;
        u32 b = tbase;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const u32 c = cnt[w][d];
            cnt[w][d] = b;
            b += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
        if (base + (u64)k * 64 + lane >= n) continue;
        const u32 at = cnt[wave][(key[k] >> shift) & (kDigits - 1)] + pos[k];
        kout[at] = key[k];
        vout[at] = val[k];
    }
}

__global__ __launch_bounds__(256) void sort_scatter_kernel(const u32* kin, const u32* vin, u32* kout, u32* vout, u64 n,
                                                           int shift, const u32* hist, u64 ntiles, const u32* rowtot,
                                                           const unsigned* gen, const unsigned* unsorted) {
    if (gated_off(gen) || !flag_set(unsorted)) return;
    sort_scatter_tile(kin, vin, kout, vout, n, shift, hist, ntiles, rowtot, blockIdx.x);
}

// The whole sort in ONE launch (round 6, tuning builds only, SYMHIP_RX_VARIANT=2): the passes'
// phases (tile counts, row scans, scatter) separated by a software grid barrier instead of launch
// boundaries, so a batch whose keys are in order already pays one gated launch, not nine (~5 us
// each) -- but a batch that needs the sort pays far more (launch_reassemble).  The grid is at most one workgroup per CU, so all of it becomes resident; a barrier that
// still has not filled after kBarrierTicks (another stream's kernels holding the CUs that long) gives
// up with kErrTimeout (SYM_ERR_DEVICE from sym_ctx_check), so the launch always ends.
constexpr u64 kBarrierTicks = 50000000;  // 500 ms of s_memrealtime (100 MHz)
struct SortArgs {
    u32* kb[2];
    u32* vb[2];
    u64 n;
    u32* hist;
    u64 ntiles;
    u32* rowtot;
    const unsigned* gen;
    const unsigned* unsorted;
    unsigned* bar;  // arrivals, zeroed per call
    unsigned* err;
    unsigned bits;
};
__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned target, unsigned* err) {
    __threadfence();  // every wave's stores of the phase, released at agent scope
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const u64 t0 = __builtin_amdgcn_s_memrealtime();
        int good = 1;
        while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > kBarrierTicks) {
                atomicOr(err, kErrTimeout);
                good = 0;
                break;
            }
        }
        ok = good;
    }
    __syncthreads();
    __threadfence();  // acquire: the other workgroups' stores
    return ok != 0;
}
__global__ __launch_bounds__(256) void sort_all_kernel(SortArgs s) {
    if (gated_off(s.gen) || !flag_set(s.unsorted)) return;  // uniform: every workgroup leaves at once
    const u64 G = gridDim.x;
    unsigned arrivals = 0;
    int cur = 0;
    for (unsigned shift = 0; shift < s.bits; shift += 8, cur ^= 1) {
        for (u64 t = blockIdx.x; t < s.ntiles; t += G) {
            sort_hist_tile(s.kb[cur], s.n, (int)shift, s.hist, s.ntiles, t);
            __syncthreads();  // the tile's LDS counts are reset by the next tile
        }
        if (!grid_barrier(s.bar, arrivals += (unsigned)G, s.err)) return;
        for (u64 d = blockIdx.x; d < kDigits; d += G) sort_rowscan_row(s.hist, s.ntiles, s.rowtot, (int)d);
        if (!grid_barrier(s.bar, arrivals += (unsigned)G, s.err)) return;
        for (u64 t = blockIdx.x; t < s.ntiles; t += G) {
            sort_scatter_tile(s.kb[cur], s.vb[cur], s.kb[cur ^ 1], s.vb[cur ^ 1], s.n, (int)shift, s.hist, s.ntiles,
                              s.rowtot, t);
            __syncthreads();
        }
        if (shift + 8 < s.bits && !grid_barrier(s.bar, arrivals += (unsigned)G, s.err)) return;
    }
}

// ---- 1. parse (transport.go:266-283, builtin_packets.go:118-161): status, RPCID, meta, payload
// length, and which of two batch kinds that need no regrouping the batch is:
//  * "simple": every DataPacket a whole message in one datagram (TotalPackets 1, sequence 0,
//    fragment 0, last).  Then each DataPacket completes its own message on arrival whatever else
//    the batch holds (no RPCID ever keeps state): the messages are the DataPackets in arrival order.
//  * "runs" (round 6): every datagram a DataPacket, RPCIDs non-decreasing, and each run of equal
//    RPCIDs what the packetizer sends for one message -- sequence numbers 0..k-1 in order, TotalPackets
//    k, one fragment each.  An RPCID then appears in one run only, and ProcessFragment completes the
//    run's message at its last datagram, with the run's payloads in arrival order as its bytes (group
//    pass 0's fast case, made a batch-wide property): the messages are the runs in arrival order.
// A datagram checks its run against its neighbours (the workgroup's edges parse theirs again).
// cnt[i] = (payload bytes, 1 segment << 32 | 1 if the datagram ends its run) for a pending DataPacket.
// One datagram's header (the parse below): status, RPCID, meta and payload length (the last three
// only for a pending DataPacket).
struct Parsed {
    uint8_t st;
    u32 pl;
    u64 r, m;
};
__device__ __forceinline__ Parsed parse_one(const Args& a, u64 i) {
    Parsed q{SYM_RX_PENDING, 0, 0, 0};
    {
        const u64 s = a.dg_off[i], L = a.dg_off[i + 1] - s;
        const uintptr_t p = (uintptr_t)(a.wire + s);
        uint8_t& st = q.st;
        u32& pl = q.pl;
        if (L >= kHdr && s + 32 <= a.dg_off[a.n]) {
            // the whole header in two byte-unaligned 16-byte loads, issued together (the common case)
            const u32x4 w0 = ld16u(p), w1 = ld16u(p + 16);
            const u32 w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
            auto u32_at = [&](int q) {  // q is a constant: the shifts fold
                return q % 4 == 0 ? w[q / 4] : (w[q / 4] >> (8 * (q % 4))) | (w[q / 4 + 1] << (32 - 8 * (q % 4)));
            };
            const u32 t = w[0] & 0xff;
            pl = u32_at(27);
            if (t != 1 && t != 2) {
                st = SYM_RX_NOT_DATA;                    // Error packet, or no codec for the type
            } else if (L < (u64)kHdr + pl) {
                st = SYM_RX_BAD_LENGTH;                  // "too short for declared payload length"
            } else {
                q.r = (u64)u32_at(1) | ((u64)u32_at(5) << 32);
                q.m = (u64)(u32_at(11) & 0xffff) | ((u64)(u32_at(9) & 0xffff) << 16) |
                      ((u64)(((w[3] >> 8) & 0xff) != 0) << 32) | ((u64)((w[3] >> 16) & 0xff) << 40);
            }
        } else if (L < 1) {
            st = SYM_RX_TOO_SHORT;                       // "data too short to read packet type"
        } else if (const u32 t = ld_u8(p); t != 1 && t != 2) {
            st = SYM_RX_NOT_DATA;
        } else if (L < kHdr) {
            st = SYM_RX_TOO_SHORT;                       // "data too short for DataPacket header"
        } else {  // a header within 32 bytes of the batch end: byte loads
            pl = ld_u32(p + 27);
            if (L < (u64)kHdr + pl) {
                st = SYM_RX_BAD_LENGTH;
            } else {
                q.r = (u64)ld_u32(p + 1) | ((u64)ld_u32(p + 5) << 32);
                q.m = (u64)(ld_u32(p + 11) & 0xffff) | ((u64)(ld_u32(p + 9) & 0xffff) << 16) |
                      ((u64)(ld_u8(p + 13) != 0) << 32) | ((u64)ld_u8(p + 14) << 40);
            }
        }
    }
    return q;
}

__global__ __launch_bounds__(256) void parse_kernel(Args a, unsigned* flags) {
    __shared__ u64 s_rpc[256], s_meta[256];
    __shared__ uint8_t s_ok[256];
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    Pair c = {0, 0};  // entries past the datagrams (entry n included) are zero
    bool simple = true, pend = false;
    u64 r = 0, m = 0;
    u32 pl = 0;
    if (i < a.n) {
        const Parsed q = parse_one(a, i);
        pend = q.st == SYM_RX_PENDING;
        if (pend) {
            r = q.r;
            m = q.m;
            pl = q.pl;
            a.rpc[i] = q.r;
            a.meta[i] = q.m;
            a.plen[i] = q.pl;
            simple = m_total(q.m) == 1 && m_seq(q.m) == 0 && m_fidx(q.m) == 0 && !m_more(q.m);
        }
        a.status[i] = q.st;
    }
    s_rpc[threadIdx.x] = r;
    s_meta[threadIdx.x] = m;
    s_ok[threadIdx.x] = pend;
    __syncthreads();
    bool bad = false, odd = false;  // RPCIDs out of order (or not a DataPacket); not a packetizer run
    if (i < a.n) {
        bool pp = false, np = false;  // the neighbours: pending, RPCID, meta
        u64 pr = 0, pm = 0, nr = 0;
        if (threadIdx.x > 0) {
            pp = s_ok[threadIdx.x - 1] != 0;
            pr = s_rpc[threadIdx.x - 1];
            pm = s_meta[threadIdx.x - 1];
        } else if (i > 0) {
            const Parsed q = parse_one(a, i - 1);
            pp = q.st == SYM_RX_PENDING;
            pr = q.r;
            pm = q.m;
        }
        if (i + 1 < a.n) {
            if (threadIdx.x < 255) {
                np = s_ok[threadIdx.x + 1] != 0;
                nr = s_rpc[threadIdx.x + 1];
            } else {
                const Parsed q = parse_one(a, i + 1);
                np = q.st == SYM_RX_PENDING;
                nr = q.r;
            }
        }
        bad = !pend || (i > 0 && (!pp || r < pr));
        if (pend) {
            const bool same_prev = i > 0 && pp && pr == r, same_next = np && nr == r;
            const u32 sq = m_seq(m), T = m_total(m);
            odd = m_fidx(m) != 0 || m_more(m) || sq != (same_prev ? m_seq(pm) + 1 : 0u) ||
                  (same_prev && T != m_total(pm)) || (!same_next && sq + 1 != T);
            c = Pair{pl, ((u64)1 << 32) | (u64)!same_next};
        }
    }
    if (i <= a.n) a.cnt[i] = c;
    // one raise per workgroup and flag (flag_raise; a wave-level atomicOr on one word serialised ~20k
    // atomics per batch of multi-datagram messages, ~200 us)
    flag_raise(flags, !simple);
    flag_raise(flags + 2, bad);
    flag_raise(flags + 3, odd);
    Pair e, t;  // this tile's totals, for the scan of the triples (simple batches and runs)
    block_scan_pair(c, e, t);
    if (threadIdx.x == 0) raw::publish_tile_total(a.agg, a.super_p, blockIdx.x, t);
}

// ---- 1a. general path: the RPCID into an open-addressing hash table (agent-scope CAS); the
// thread whose CAS claims the slot writes its arrival index into first[slot], and that index is the
// group key (any one arrival of the RPCID serves: every output is placed by the arrival-order scan,
// so the order of the groups only matters for locality -- and the claiming arrival is usually an
// early one, so the groups still sort roughly in order of appearance).  The datagrams of one
// workgroup first meet in an LDS table, and only one of them per RPCID goes to the global table
// (round 6: the batch's ~2.7M random atomics, one CAS and one atomicMin per datagram, ran at the
// chip's atomic rate, ~120 us for config 3 shuffled within windows of 64).  The per-arrival triples
// are recomputed by group pass 0.
constexpr int kLocalSlots = 512;
constexpr u32 kKeyLater = ~0u;  // gid of a datagram whose RPCID another workgroup claimed (keys are <= n)
__global__ __launch_bounds__(256) void hash_kernel(Args a, const unsigned* gate) {
    if (gated_off(gate)) return;
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < a.n) {
        a.cnt[i] = Pair{0, 0};
        a.idx[i] = (u32)i;
    }
    if (!*a.nm) return;  // (uniform) runs of equal RPCIDs: key_kernel takes the run heads
    __shared__ u64 s_key[kLocalSlots];
    __shared__ u32 s_slot[kLocalSlots], s_gkey[kLocalSlots];
    for (int k = threadIdx.x; k < kLocalSlots; k += 256) s_key[k] = kEmpty;
    __syncthreads();
    const bool pend = i < a.n && a.status[i] == SYM_RX_PENDING;
    const u64 r = pend ? a.rpc[i] : kEmpty;
    int e = 0;
    bool lead = false;  // the workgroup's first thread to hold this RPCID
    if (r != kEmpty) {
        u32 h = (u32)(mix64(r) >> 40) & (kLocalSlots - 1);
        for (;;) {
            const u64 prev = atomicCAS((unsigned long long*)&s_key[h], (unsigned long long)kEmpty, (unsigned long long)r);
            if (prev == kEmpty) {
                lead = true;
                break;
            }
            if (prev == r) break;
            h = (h + 1) & (kLocalSlots - 1);
        }
        e = (int)h;
    }
    u32 g = kNoSlot;  // table slot
    if (lead) {       // open addressing; the table has >= 2n slots, so a free slot is always found
        u64 h = mix64(r) & a.tmask;
        bool claimed = false;
        for (;;) {
            const u64 prev = atomicCAS((unsigned long long*)&a.table[h], (unsigned long long)kEmpty, (unsigned long long)r);
            if (prev == kEmpty) {
                a.first[h] = (u32)i;  // the group key, for other workgroups' datagrams (key_kernel)
                claimed = true;
                break;
            }
            if (prev == r) break;
            h = (h + 1) & a.tmask;
        }
        g = (u32)h;
        s_slot[e] = g;
        s_gkey[e] = claimed ? (u32)i : kKeyLater;
    }
    __syncthreads();
    u32 key = a.nodata;
    if (pend) {
        if (r == kEmpty) {  // the RPCID equal to the empty marker: its own slot, claimed the same way
            g = a.special;
            atomicCAS(&a.first[g], ~0u, (u32)i);
            key = kKeyLater;
        } else {
            if (!lead) g = s_slot[e];
            key = s_gkey[e];
        }
    }
    if (i < a.n) {
        a.slot[i] = g;
        a.gid[i] = key;  // kKeyLater: claimed by another workgroup, key_kernel reads first[slot]
    }
}

// ---- simple batches and runs (parse_kernel): the messages in arrival order, from the scan of the
// parse's triples -- a simple batch's message m is its m-th DataPacket (the segment count), a run's
// message is the run (the count of run ends).  The kernel is queued before the host knows the batch
// kind and does nothing for other batches (except zeroing the segment count, so the gather after
// it is empty too).
//   The segment gather's tile prefixes come from here too (round 6): segment s's output offset is
// known, so the first segment of every 256-segment tile writes its tile's prefix and entry n the
// total at tile ceil(nseg / 256) -- no tile-total and scan launches before the gather.
__global__ __launch_bounds__(256) void emit_kernel(Args a, const unsigned* flags, u64* nmsg, u64* nseg,
                                                   Pair* seg_pre) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    const bool simple = !flag_set(flags), nonmono = flag_set(a.nonmono);
    const bool general = !simple && (nonmono || flag_set(flags + 3));
    if (general) {  // the general path's batch
        if (i == 0) *nseg = 0;
        return;
    }
    const bool data = i < a.n && a.status[i] == SYM_RX_PENDING;
    const Pair v = i <= a.n ? a.cnt[i] : Pair{0, 0};  // the parse's triple
    Pair e, t;
    block_scan_pair(v, e, t);
    const Pair b = raw::tile_prefix_2l(a.agg, a.super_p, blockIdx.x, (a.n + 256) / 256);  // the parse's totals
    const u64 bytes = b.bytes + e.bytes, seg = (b.count + e.count) >> 32, ends = (b.count + e.count) & 0xffffffffull;
    if (data) {
        const u64 r = a.rpc[i];
        a.seg_src[seg] = a.dg_off[i] + kHdr;
        a.seg_len[seg] = v.bytes;
        a.status[i] = SYM_RX_CONSUMED;
        if ((seg & 255) == 0) seg_pre[seg >> 8] = Pair{bytes, 0};
        if (simple) {
            a.msg_off[seg] = bytes;
            a.msg_rpc[seg] = r;
            a.msg_dg[seg] = i;
        } else {  // runs: every datagram pending, so the neighbours in arrival order are the run's
            if (i == 0 || a.rpc[i - 1] != r) a.msg_off[ends] = bytes;  // the run's first datagram
            if (v.count & 1) {                                          // its last
                a.msg_rpc[ends] = r;
                a.msg_dg[ends] = i;
            }
        }
    }
    if (i == a.n) {  // entry n: the totals
        const u64 nm = simple ? seg : ends;
        *nmsg = nm;
        a.msg_off[nm] = bytes;
        *nseg = seg;
        seg_pre[tiles(seg)] = Pair{bytes, 0};
    }
}

// ---- 1b. group key: the run head when the RPCIDs never decrease, so an in-order stream keeps its
// arrival order and every later pass reads and writes it coalesced; else the hash table's key
__global__ __launch_bounds__(256) void key_kernel(Args a, const unsigned* gate) {
    if (gated_off(gate)) return;
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    bool down = false;  // a key below its predecessor's: the batch needs the sort
    const bool nonmono = *a.nm != 0;
    if (i < a.n && !nonmono) {  // the run head: every datagram is a pending DataPacket here
        // The RPCIDs never decrease on this path, so the head is the first index holding r: one load
        // when i starts its run (the common case), else a gallop back (steps 1, 2, 4, ...) to an index
        // below the run, then a binary search -- O(log run) loads, so one RPCID repeated over a whole
        // batch costs 2^20 * ~40 loads, not a walk of the run per datagram.
        const u64 r = a.rpc[i];
        u64 h = i;
        if (i > 0 && a.rpc[i - 1] == r) {
            i64 lo = -1, hi = (i64)i - 1;  // rpc[lo] < r (lo = -1: none), rpc[hi] == r
            for (i64 step = 1;; step <<= 1) {
                const i64 c = hi - step;
                if (c < 0) break;
                if (a.rpc[c] != r) {
                    lo = c;
                    break;
                }
                hi = c;
            }
            while (hi - lo > 1) {
                const i64 mid = lo + (hi - lo) / 2;
                if (a.rpc[mid] == r) hi = mid;
                else lo = mid;
            }
            h = (u64)hi;
        }
        a.gid[i] = (u32)h;  // non-decreasing
    } else if (nonmono) {  // (uniform) the key the hash kernel left -- or its slot's, claimed by
                              // another workgroup -- and the previous one from LDS
        __shared__ u32 s_gid[256];
        auto key_of = [&](u64 j) {
            const u32 k = a.gid[j];
            return k == kKeyLater ? a.first[a.slot[j]] : k;
        };
        const u32 g = i < a.n ? key_of(i) : 0u;
        s_gid[threadIdx.x] = g;
        __syncthreads();
        if (i < a.n) {
            if (a.gid[i] != g) a.gid[i] = g;
            if (i > 0) down = g < (threadIdx.x > 0 ? s_gid[threadIdx.x - 1] : key_of(i - 1));
        }
    }
    flag_raise(a.unsorted, down);  // (one atomic per workgroup on one word had cost ~55 us per batch)
}

__device__ inline bool seq_complete(const SeqState& x) {
    if (!(x.flags & 2)) return false;
    const u32 li = x.flags >> 8;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const int hi = (int)li - 32 * w;  // highest wanted bit in this word
        if (hi < 0) break;
        const u32 need = hi >= 31 ? ~0u : (2u << hi) - 1u;
        if ((x.bits[w] & need) != need) return false;
    }
    return true;
}

// Group pass 0's triple for arrival j, and its share of j's tile total: the workgroup's own tile and
// the next one (where a run that starts here usually completes) in LDS, flushed once at the end;
// farther tiles (long runs, or sorted groups) by global atomics.  (Round 6: this replaced a
// tile-total launch over the triples between the group pass and the scan.)
__device__ __forceinline__ void put_cnt(const Args& a, u64 j, Pair v, u64* sb, u64* sc) {
    a.cnt[j] = v;
    const u64 t = j >> 8, d = t - blockIdx.x;
    if (d < 2) {
        atomicAdd((unsigned long long*)&sb[d], (unsigned long long)v.bytes);
        atomicAdd((unsigned long long*)&sc[d], (unsigned long long)v.count);
    } else {
        raw::add_tile_total(a.agg_c, a.super_c, t, v);
    }
}

// ---- 3 / 5. the ProcessFragment state machine over one group's run (fragmentation.go:62-181)
template <int PASS>
__device__ __forceinline__ void group_one(const Args& a, u64 q0, u64* lb, u64* lc) {
    if (q0 >= a.n) return;
    const u32 g = a.gs[q0];
    if (g == a.nodata) return;                   // not a DataPacket (sorted last)
    if (q0 > 0 && a.gs[q0 - 1] == g) return;     // not the first of its group
    u64 e = q0 + 1;
    while (e < a.n && a.gs[e] == g) ++e;
    const u64 k = e - q0;                        // sequence numbers >= k can never complete
    {  // one message of k packets, TotalPackets k, one fragment each, SeqNumbers 0..k-1 -- in order
       // (the packetizer's run), or in any order for k <= 64 (a reordered one, round 6).  The machine
       // below completes it at its last arrival (only then are all k sequence numbers in) with the
       // packets in sequence order as the segments; say so without the per-sequence state.
        bool fast = true, inorder = true;
        u64 bytes = 0, seen = 0;
        for (u64 t = 0; t < k && fast; ++t) {
            const u32 j = a.is[q0 + t];
            const u64 m = a.meta[j];
            const u32 sq = m_seq(m);
            inorder = inorder && sq == t;
            fast = m_total(m) == k && m_fidx(m) == 0 && !m_more(m) &&
                   (inorder || (k <= 64 && sq < k && !((seen >> sq) & 1)));
            if (k <= 64) seen |= (u64)1 << (sq & 63);
            bytes += a.plen[j];
        }
        if (fast) {
            const u32 jl = a.is[e - 1];
            if constexpr (PASS == 0) {
                put_cnt(a, jl, Pair{bytes, (k << 32) | 1u}, lb, lc);
                for (u64 t = 0; t < k; ++t) a.status[a.is[q0 + t]] = SYM_RX_CONSUMED;
            } else {
                const Pair pp = a.pre[jl];
                const u64 mi = pp.count & 0xffffffffull, sb = pp.count >> 32;
                a.msg_off[mi] = pp.bytes;
                a.msg_rpc[mi] = a.rpc[jl];
                a.msg_dg[mi] = jl;
                u64 at = pp.bytes;  // the segment's output offset (in order: a running sum)
                for (u64 t = 0; t < k; ++t) {
                    const u32 j = a.is[q0 + t];
                    const u32 pl = a.plen[j];
                    u64 sg = sb + t;
                    if (!inorder) {  // its place in sequence order, behind the packets of lower numbers
                        const u32 sq = m_seq(a.meta[j]);
                        sg = sb + sq;
                        at = pp.bytes;
                        for (u64 t2 = 0; t2 < k; ++t2) {
                            const u32 j2 = a.is[q0 + t2];
                            if (m_seq(a.meta[j2]) < sq) at += a.plen[j2];
                        }
                    }
                    a.seg_src[sg] = a.dg_off[j] + kHdr;
                    a.seg_len[sg] = pl;
                    if ((sg & 255) == 0) a.seg_pre[sg >> 8] = Pair{at, 0};
                    at += pl;
                }
            }
            return;
        }
    }
    SeqState* S = a.state + q0;
    for (u64 t = 0; t < k; ++t) S[t] = SeqState{};
    u64 r = q0;  // first datagram of the current message
    u32 distinct = 0, ncomplete = 0, maxseq = 0;
    bool big = false;
    for (u64 q = q0; q < e; ++q) {
        const u32 j = a.is[q];
        const u64 m = a.meta[j];
        const u32 s = m_seq(m), T = m_total(m), fi = m_fidx(m);
        if (s >= k) {
            big = true;
        } else {
            SeqState x = S[s];
            const bool was = seq_complete(x);
            if (!(x.flags & 1)) {
                x.flags |= 1;
                ++distinct;
            }
            x.bits[fi >> 5] |= 1u << (fi & 31);
            if (fi == 0) x.latest0 = j;            // a later fragment overwrites (map store, :79-83)
            if (!m_more(m)) {                       // :87-93
                const u32 li = max(x.flags >> 8, fi);
                x.flags = (x.flags & 0xffu) | 2u | (li << 8);
            }
            const bool now = seq_complete(x);
            ncomplete += (u32)now - (u32)was;
            S[s] = x;
        }
        maxseq = max(maxseq, s);
        // :99-133 -- distinct sequence numbers == TotalPackets of THIS packet and all complete
        if (big || T == 0 || maxseq >= T || distinct != T || ncomplete != T) continue;
        u64 bytes = 0, segs = 0, ob = 0, sb = 0;
        if constexpr (PASS == 1) {
            const Pair pp = a.pre[j];
            const u64 mi = pp.count & 0xffffffffull;
            sb = pp.count >> 32;
            ob = pp.bytes;
            a.msg_off[mi] = ob;
            a.msg_rpc[mi] = a.rpc[j];
            a.msg_dg[mi] = j;
        }
        for (u32 s2 = 0; s2 < T; ++s2) {           // :153-161, (seq, fragment index) order
            const SeqState x = S[s2];
            const u32 li = x.flags >> 8;
            for (u32 f = 0; f <= li; ++f) {
                u32 src = x.latest0;
                if (f > 0)                          // rare: the latest arrival with (s2, f)
                    for (u64 b = q + 1; b-- > r;) {
                        const u64 mb = a.meta[a.is[b]];
                        if (m_seq(mb) == s2 && m_fidx(mb) == f) {
                            src = a.is[b];
                            break;
                        }
                    }
                if constexpr (PASS == 1) {
                    a.seg_src[sb + segs] = a.dg_off[src] + kHdr;
                    a.seg_len[sb + segs] = a.plen[src];
                    if (((sb + segs) & 255) == 0) a.seg_pre[(sb + segs) >> 8] = Pair{ob + bytes, 0};
                }
                bytes += a.plen[src];
                ++segs;
            }
        }
        if constexpr (PASS == 0) put_cnt(a, j, Pair{bytes, (segs << 32) | 1u}, lb, lc);
        for (u64 b = r; b <= q; ++b) {              // :175-178: the RPCID's state is deleted
            const u32 jb = a.is[b];
            if constexpr (PASS == 0) a.status[jb] = SYM_RX_CONSUMED;
            const u32 sb2 = m_seq(a.meta[jb]);
            if (sb2 < k) S[sb2] = SeqState{};
        }
        r = q + 1;
        distinct = ncomplete = maxseq = 0;
        big = false;
    }
}
template <int PASS>
__global__ __launch_bounds__(256) void group_kernel(Args a, const unsigned* gate) {
    if (gated_off(gate)) return;
    if (!flag_set(a.unsorted)) {  // the keys were in order already: the sort left them in gid / idx
        a.gs = a.gid;
        a.is = a.idx;
    }
    __shared__ u64 sb[2], sc[2];  // pass 0: the totals of this workgroup's tile and the next
    if constexpr (PASS == 0) {
        if (threadIdx.x < 2) sb[threadIdx.x] = sc[threadIdx.x] = 0;
        __syncthreads();
    }
    group_one<PASS>(a, (u64)blockIdx.x * 256 + threadIdx.x, sb, sc);
    if constexpr (PASS == 0) {
        __syncthreads();
        if (threadIdx.x < 2 && (sb[threadIdx.x] | sc[threadIdx.x]))
            raw::add_tile_total(a.agg_c, a.super_c, blockIdx.x + threadIdx.x, Pair{sb[threadIdx.x], sc[threadIdx.x]});
    }
}

// ---- 4. exclusive scan of the per-arrival triples (256 per tile)
__device__ inline void block_scan_pair(Pair v, Pair& excl, Pair& tile_total) {
    __shared__ u64 wb[4], wc[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 ib = wave_incl_scan_u64(v.bytes, lane), ic = wave_incl_scan_u64(v.count, lane);
    if (lane == 63) {
        wb[wave] = ib;
        wc[wave] = ic;
    }
    __syncthreads();
    u64 pb = 0, pc = 0;
    for (int q = 0; q < wave; ++q) {
        pb += wb[q];
        pc += wc[q];
    }
    excl = Pair{pb + ib - v.bytes, pc + ic - v.count};
    tile_total = Pair{wb[0] + wb[1] + wb[2] + wb[3], wc[0] + wc[1] + wc[2] + wc[3]};
}

// The exclusive scan applied (tile prefixes from the two-level totals), and at the last entry (m - 1:
// a zero triple, so its prefix is the grand total) the message count, closing offset and segment count.
__global__ __launch_bounds__(256) void pair_scan_apply_kernel(const Pair* v, u64 m, const Pair* agg, const Pair* super,
                                                              Pair* out, u64* msg_off, u64* nmsg, u64* nseg,
                                                              Pair* seg_pre, const unsigned* gate) {
    if (gated_off(gate)) return;
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    Pair e, t;
    block_scan_pair(i < m ? v[i] : Pair{0, 0}, e, t);
    const Pair b = raw::tile_prefix_2l(agg, super, blockIdx.x, (m + 255) / 256);
    if (i < m) out[i] = Pair{b.bytes + e.bytes, b.count + e.count};
    if (i == m - 1) {
        const u64 tb = b.bytes + e.bytes, tc = b.count + e.count;
        const u64 nm = tc & 0xffffffffull;
        *nmsg = nm;
        msg_off[nm] = tb;
        *nseg = tc >> 32;
        seg_pre[tiles(tc >> 32)] = Pair{tb, 0};  // the segments' total (group pass 1 writes the tile prefixes)
    }
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
inline u64 table_size(u64 n) {
    u64 t = 1024;
    while (t < 2 * n) t <<= 1;
    return t;
}
inline unsigned log2u(u64 t) {
    unsigned b = 0;
    while (((u64)1 << b) < t) ++b;
    return b;
}
inline unsigned key_bits(u64 n) { return log2u(n + 1) + 1; }  // keys in [0, n]

struct Layout {
    size_t table, first, slot, rpc, meta, plen, gid, idx, gs, is, state, cnt, pre, agg, seg_src, seg_len, pre2, pre3, nseg, nseg2, flag, unsorted, nonmono, gen, nm, bar, sup_p, sup_c, agg_c, zero_bytes, hist, rowtot, total;
};

inline u64 sort_tiles(u64 n) { return (n + kSortTile - 1) / kSortTile; }

inline Layout layout(u64 n) {
    Layout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += al256(bytes);
        return at;
    };
    const u64 TS = table_size(n);
    L.table = take(TS * 8);
    L.first = take((TS + 1) * 4);
    L.slot = take(n * 4);
    L.rpc = take(n * 8);
    L.meta = take(n * 8);
    L.plen = take(n * 4);
    L.gid = take(n * 4);
    L.idx = take(n * 4);
    L.gs = take(n * 4);
    L.is = take(n * 4);
    L.state = take(n * sizeof(SeqState));
    L.cnt = take((n + 1) * sizeof(Pair));
    L.pre = take((n + 1) * sizeof(Pair));
    L.agg = take((tiles(n + 1) + 1) * sizeof(Pair));
    L.seg_src = take(n * 8);
    L.seg_len = take(n * 8);
    L.pre2 = take((tiles(n) + 1) * sizeof(Pair));
    L.pre3 = take((tiles(n) + 1) * sizeof(Pair));  // the single-datagram path's own (it runs beside the general path)
    L.nseg = take(8);
    // the general path's segment count, the parse's flag, the key order and RPCID order flags, the
    // sort's barrier, then the group totals of the parse's tile totals, the group totals and tile
    // totals of the general path's triples: zeroed together, one memset per call
    const size_t sup = raw::super_bytes(tiles(n + 1));
    L.zero_bytes = 128 + kFlagBytes + 2 * sup + (tiles(n + 1) + 1) * sizeof(Pair);
    L.nseg2 = take(L.zero_bytes);
    L.flag = L.nseg2 + 128;  // kShards lines of four flag words (flag_set)
    L.sup_p = L.flag + kFlagBytes;  // (lines of their own: the atomics on the totals stay off the flags')
    L.sup_c = L.sup_p + sup;
    L.agg_c = L.sup_c + sup;
    L.unsorted = L.flag + 4;
    L.nonmono = L.flag + 8;
    L.gen = L.nseg2 + 8;
    L.nm = L.nseg2 + 12;
    L.bar = L.nseg2 + 24;
    L.hist = take((size_t)kDigits * sort_tiles(n) * 4);
    L.rowtot = take(kDigits * 4);
    L.total = o;
    return L;
}

}  // namespace rx

size_t reassemble_ws_bytes(u64 n) { return rx::layout(n).total; }

hipError_t launch_reassemble(const uint8_t* wire, const u64* dg_off, u64 n, uint8_t* msg, u64 msg_cap, u64* msg_off,
                             u64* msg_rpc, u64* msg_dg, u64* nmsg, uint8_t* status, void* ws, unsigned* err,
                             hipStream_t stream, hipStream_t aux, hipEvent_t fork, hipEvent_t join) {
    using rx::Pair;
    const rx::Layout L = rx::layout(n);
    char* w = (char*)ws;
    const u64 TS = rx::table_size(n);
    rx::Args a{};
    a.wire = wire;
    a.dg_off = dg_off;
    a.n = n;
    a.table = (u64*)(w + L.table);
    a.tmask = TS - 1;
    a.special = (u32)TS;
    a.nodata = (u32)n;
    a.first = (u32*)(w + L.first);
    a.slot = (u32*)(w + L.slot);
    a.rpc = (u64*)(w + L.rpc);
    a.meta = (u64*)(w + L.meta);
    a.plen = (u32*)(w + L.plen);
    a.gid = (u32*)(w + L.gid);
    a.idx = (u32*)(w + L.idx);
    a.state = (rx::SeqState*)(w + L.state);
    a.status = status;
    a.cnt = (Pair*)(w + L.cnt);
    a.pre = (const Pair*)(w + L.pre);
    a.msg_off = msg_off;
    a.msg_rpc = msg_rpc;
    a.msg_dg = msg_dg;
    a.seg_src = (u64*)(w + L.seg_src);
    a.seg_len = (u64*)(w + L.seg_len);
    a.seg_pre = (Pair*)(w + L.pre2);
    a.unsorted = (unsigned*)(w + L.unsorted);
    a.nonmono = (const unsigned*)(w + L.nonmono);
    a.gen = (unsigned*)(w + L.gen);
    a.nm = (unsigned*)(w + L.nm);
    const unsigned* gen = a.gen;
    const dim3 b256(256);
    const unsigned* flag = (const unsigned*)(w + L.flag);
    const dim3 gq((unsigned)rx::tiles(n));
    const u64 nt = rx::tiles(n + 1);
    Pair* agg = (Pair*)(w + L.agg);
    a.agg = agg;
    a.super_p = (Pair*)(w + L.sup_p);
    a.super_c = (Pair*)(w + L.sup_c);
    a.agg_c = (Pair*)(w + L.agg_c);
    // the payload segments' tile prefixes, then the gather (segment count on the device); gate:
    // the general path's copy, which does nothing for a simple batch
    // the payload gather (segment count and tile prefixes on the device); general: the general path's
    // copy, which does nothing for a simple batch (its segment count stays 0)
    auto seg_tail = [&](u64* nseg, bool general, hipStream_t st) -> hipError_t {
        Pair* pre2 = (Pair*)(w + (general ? L.pre2 : L.pre3));
        raw::GatherArgs ga{};
        ga.in = wire;
        ga.n = n;
        ga.n_ptr = nseg;
        ga.lo_ptr = dg_off;
        ga.hi_ptr = dg_off + n;
        ga.pre = pre2;
        ga.seg_src = a.seg_src;
        ga.seg_len = a.seg_len;
        ga.out = msg;
        ga.cap = msg_cap;
        ga.err = err;
        ga.seg_bytes_hint = msg_cap / n;  // (the capacity is usually the wire size)
        ga.nt = 2;  // nontemporal at any span (see DESIGN)
        return launch_segment_gather(ga, st);
    };
    // Simple batches (every DataPacket one whole message) complete here: parse (with the tile
    // totals of the per-arrival triples), their scan, the messages, the gather.  For other batches
    // the emit writes no message and zero segments, so this gather is empty.
    u64* nseg = (u64*)(w + L.nseg);
    u64* nseg2 = (u64*)(w + L.nseg2);
    hipError_t e = hipMemsetAsync(w + L.nseg2, 0, L.zero_bytes, stream);  // nseg2, the flags, the group totals
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rx::parse_kernel, dim3((unsigned)nt), b256, 0, stream, a, (unsigned*)flag);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // The general path is queued for every batch; each of its kernels exits at once unless the
    // parse's flags say so (no host read: the call stays asynchronous).  It runs on `aux`, forked
    // here and joined at the end, so for a single-datagram or runs batch its empty launches overlap
    // the emit and the copy below.  The two branches share no buffer that both write for the same
    // batch: every write of the main branch past this point is for a batch the general path skips
    // (its zero segment count for the others excepted, in a word of its own), every write of the
    // general branch for one it takes.
    hipStream_t gs = stream;
    if (aux && fork && join) {
        if ((e = hipEventRecord(fork, stream)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(aux, fork, 0)) != hipSuccess) return e;
        gs = aux;
    }
    hipLaunchKernelGGL(rx::emit_kernel, dim3((unsigned)nt), b256, 0, stream, a, flag, nmsg, nseg, (Pair*)(w + L.pre3));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = seg_tail(nseg, false, stream)) != hipSuccess) return e;
    hipLaunchKernelGGL(rx::init_kernel, dim3((unsigned)std::min<u64>(rx::tiles(TS + 1), 4096)), b256, 0, gs, a.table,
                       a.first, TS, flag, a.gen, a.nm);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(rx::hash_kernel, gq, b256, 0, gs, a, gen);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(rx::key_kernel, gq, b256, 0, gs, a, gen);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    {  // 2. the stable radix sort, ping-ponging between (gid, idx) and (gs, is); only when the keys
       // are out of order (set by key_kernel, so only for a batch on the general path)
        u32* kb[2] = {a.gid, (u32*)(w + L.gs)};
        u32* vb[2] = {a.idx, (u32*)(w + L.is)};
        const u64 st = rx::sort_tiles(n);
        u32* hist = (u32*)(w + L.hist);
        u32* rowtot = (u32*)(w + L.rowtot);
        const unsigned bits = rx::key_bits(n);
        int cur = 0;
        // three launches a pass: the one-launch form (sort_all_kernel) costs one empty launch instead of
        // nine for a batch with its keys in order, but with its grid of one workgroup per CU each
        // phase works through its tiles in rounds: config 3 shuffled within windows of 64, 1.05 ->
        // 1.62 ms (profiles/r06_rx_sort_ab.txt), for 3-11 us on the batches that skip the sort
        bool one_launch = false;
#ifdef SYMHIP_TUNING
        one_launch = tuning_variant("SYMHIP_RX_VARIANT") == 2;
#endif
        if (one_launch) {
            static int cus[16] = {0};
            int dev = 0;
            if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
            int& ncu = cus[dev & 15];
            if (ncu == 0 && (e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
                return e;
            rx::SortArgs sa{{kb[0], kb[1]}, {vb[0], vb[1]}, n, hist, st, rowtot, gen, a.unsorted,
                            (unsigned*)(w + L.bar), err, bits};
            hipLaunchKernelGGL(rx::sort_all_kernel, dim3((unsigned)std::min<u64>(st, (u64)ncu)), b256, 0, gs, sa);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            cur = (int)(((bits + 7) / 8) & 1);
        } else {
            for (unsigned shift = 0; shift < bits; shift += 8, cur ^= 1) {
                hipLaunchKernelGGL(rx::sort_hist_kernel, dim3((unsigned)st), b256, 0, gs, (const u32*)kb[cur], n,
                                   (int)shift, hist, st, gen, a.unsorted);
                hipLaunchKernelGGL(rx::sort_rowscan_kernel, dim3(rx::kDigits), b256, 0, gs, hist, st, rowtot, gen,
                                   a.unsorted);
                hipLaunchKernelGGL(rx::sort_scatter_kernel, dim3((unsigned)st), b256, 0, gs, (const u32*)kb[cur],
                                   (const u32*)vb[cur], kb[cur ^ 1], vb[cur ^ 1], n, (int)shift, (const u32*)hist, st,
                                   (const u32*)rowtot, gen, a.unsorted);
                if ((e = hipGetLastError()) != hipSuccess) return e;
            }
        }
        a.gs = kb[cur];
        a.is = vb[cur];
    }
    hipLaunchKernelGGL(rx::group_kernel<0>, gq, b256, 0, gs, a, gen);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(rx::pair_scan_apply_kernel, dim3((unsigned)nt), b256, 0, gs, (const Pair*)a.cnt, n + 1,
                       (const Pair*)a.agg_c, (const Pair*)a.super_c, (Pair*)(w + L.pre), msg_off, nmsg, nseg2,
                       (Pair*)(w + L.pre2), gen);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(rx::group_kernel<1>, gq, b256, 0, gs, a, gen);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = seg_tail(nseg2, true, gs)) != hipSuccess) return e;
    if (gs != stream) {
        if ((e = hipEventRecord(join, gs)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(stream, join, 0)) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace symhip
