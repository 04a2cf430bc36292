// gather_tile.hpp -- one 256-segment tile of the output-stationary segment gather (raw_fields.hip's
// gather_kernel; flat.hip's fused decode emit kernel takes the same tiles of several fields).
#pragma once
#include <type_traits>

#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {
namespace raw {

constexpr int kSegs = 64;  // segments per wave tile
constexpr int kWaves = 4;

// ---- gather: each workgroup owns a 256-record tile; out gets the segments back to back
struct WaveLds {
    u64 addr[kSegs];   // segment's source address
    int o[kSegs + 1];  // segment's output start relative to the wave's; [cnt] = span
};

__device__ __forceinline__ u64 readlane_u64(u64 v, int l) {
    return (u64)(u32)__builtin_amdgcn_readlane((u32)v, l) | ((u64)(u32)__builtin_amdgcn_readlane((u32)(v >> 32), l) << 32);
}

// ---- two-level tile prefixes without a scan launch (round 6): the kernel that produces the tiles'
// totals also adds each one into the total of its group of kSuperTiles tiles (agent-scope atomics into
// Pairs zeroed before the call, one 128-byte line per group: with 256-tile groups packed into a few
// lines the atomics of thousands of workgroups serialised on them, +55 us per launch); a consumer of
// tile b then sums, in one workgroup reduction, the totals of the groups before b's and of the tiles
// before b inside its group.  Saves the single-workgroup scan launch (~9 us of launch boundaries)
// between producer and consumer.  (Not used by the gather itself: inside gather_tile the prefix code
// cost 10-18 VGPRs, a wave per SIMD, more than the launch it saves.)
constexpr u64 kSuperTiles = 64;
constexpr u64 kSuperStride = 8;  // Pairs per group total: one 128-byte line each
__host__ __device__ inline u64 super_bytes(u64 ntiles) { return ((ntiles + kSuperTiles - 1) / kSuperTiles + 1) * kSuperStride * 16; }
__device__ __forceinline__ void publish_tile_total(Pair* agg, Pair* super, u64 tile, Pair t) {
    agg[tile] = t;
    Pair* g = super + (tile / kSuperTiles) * kSuperStride;
    if (t.bytes) atomicAdd((unsigned long long*)&g->bytes, (unsigned long long)t.bytes);
    if (t.count) atomicAdd((unsigned long long*)&g->count, (unsigned long long)t.count);
}
// The same totals built by adding contributions (agg and super zeroed before the producer runs).
__device__ __forceinline__ void add_tile_total(Pair* agg, Pair* super, u64 tile, Pair t) {
    Pair* g = super + (tile / kSuperTiles) * kSuperStride;
    if (t.bytes) {
        atomicAdd((unsigned long long*)&agg[tile].bytes, (unsigned long long)t.bytes);
        atomicAdd((unsigned long long*)&g->bytes, (unsigned long long)t.bytes);
    }
    if (t.count) {
        atomicAdd((unsigned long long*)&agg[tile].count, (unsigned long long)t.count);
        atomicAdd((unsigned long long*)&g->count, (unsigned long long)t.count);
    }
}
// Whole workgroup of 256 threads (every thread calls it): tile's exclusive prefix; the grand total of the
// ntiles tiles into *total when given.
__device__ inline Pair tile_prefix_2l(const Pair* agg, const Pair* super, u64 tile, u64 ntiles, Pair* total = nullptr) {
    __shared__ u64 rb[4], rc[4], sb[4], sc[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 g = tile / kSuperTiles, r = tile % kSuperTiles, nsup = (ntiles + kSuperTiles - 1) / kSuperTiles;
    u64 b = 0, c = 0, tb = 0, tc = 0;
    if ((u64)threadIdx.x < r) {
        const Pair v = agg[g * kSuperTiles + threadIdx.x];
        b = v.bytes;
        c = v.count;
    }
    for (u64 j = threadIdx.x; j < nsup; j += 256) {
        const Pair v = super[j * kSuperStride];
        if (j < g) {
            b += v.bytes;
            c += v.count;
        }
        tb += v.bytes;
        tc += v.count;
    }
    b = wave_sum_u64(b);
    c = wave_sum_u64(c);
    if (total) {
        tb = wave_sum_u64(tb);
        tc = wave_sum_u64(tc);
    }
    if (lane == 0) {
        rb[wave] = b;
        rc[wave] = c;
        sb[wave] = tb;
        sc[wave] = tc;
    }
    __syncthreads();
    // (wave-uniform, and made provably so: the callers' arithmetic on them stays scalar, as it is on a
    // prefix loaded from a scan's output)
    const Pair out{(u64)uniform_i64((i64)(rb[0] + rb[1] + rb[2] + rb[3])), (u64)uniform_i64((i64)(rc[0] + rc[1] + rc[2] + rc[3]))};
    if (total)
        *total = Pair{(u64)uniform_i64((i64)(sb[0] + sb[1] + sb[2] + sb[3])), (u64)uniform_i64((i64)(sc[0] + sc[1] + sc[2] + sc[3]))};
    __syncthreads();  // rb.. are rewritten by the next call
    return out;
}

// One 256-segment tile (a workgroup loop body of gather_kernel, or of flat.hip's dec_emit_kernel).
// pre[ntiles] is the total: a scan over the capacity's tiles has it there too, at the exclusive
// prefix of the first empty tile.
template <bool FW, int KU = 4, bool NT = false>
__device__ __forceinline__ void gather_tile(const GatherArgs& a, u64 tile, u64 n, u64 ntiles, WaveLds* lds_all,
                                            const MaskTable& masks, u64* wsum_b, u64* wsum_c) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 i = tile * 256 + threadIdx.x;

    // ---- phase 1 (thread = record): length, keep flag, in-tile exclusive scan
    u64 src = 0, len = 0, keep = 0;
    if (i < n) {
        if constexpr (FW) {
            src = a.rec_off[i];
            keep = a.verdict[i] == SYM_VERDICT_PASS;
            len = keep ? a.rec_off[i + 1] - src : 0;
        } else {
            src = a.seg_src[i];
            len = a.seg_len[i];
        }
    }
    const u64 ib = wave_incl_scan_u64(len, lane);
    const u32 ic = FW ? wave_incl_scan_u32_dpp((u32)keep) : 0u;
    if (lane == 63) {
        wsum_b[wave] = ib;
        wsum_c[wave] = ic;
    }
    __syncthreads();  // the only workgroup barrier
    const Pair total = a.pre[ntiles];
    const Pair tp = a.pre[tile];
    if (total.bytes > a.cap) {  // output does not fit: nothing is written (uniform)
        if (i == 0) atomicOr(a.err, kErrCapacity);
        return;
    }
    u64 wb = tp.bytes, wc = tp.count;
    for (int q = 0; q < wave; ++q) {
        wb += wsum_b[q];
        wc += wsum_c[q];
    }
    const u64 d = wb + ib - len;  // this segment's output start
    if constexpr (FW) {
        const u64 rank = wc + ic - keep;
        if (keep) {
            a.out_off[rank] = d;
            if (a.kept_index) a.kept_index[rank] = i;
        }
        if (i == n - 1) {
            a.out_off[rank + keep] = d + len;
            *a.nkept = rank + keep;
        }
    } else {
        if (a.out_off && i < n) a.out_off[i] = d;
        if (a.out_off && i == n - 1) a.out_off[n] = d + len;
    }

    // ---- phase 2 (wave = 64 segments, lane = aligned 16-byte output chunk)
    const u64 r0 = tile * 256 + (u64)wave * kSegs;
    if (r0 >= n) return;  // wave-uniform
    const int cnt = (int)min((u64)kSegs, n - r0);
    WaveLds& S = lds_all[wave];
    const u64 D0 = readlane_u64(d, 0), D1 = readlane_u64(d + len, cnt - 1);
    if (D1 - D0 >= ((u64)1 << 31)) {  // positions are 32-bit
        if (lane == 0) atomicOr(a.err, kErrTooLarge);
        return;
    }
    const u64 in_lo = *a.lo_ptr, in_hi = *a.hi_ptr;
    // Only non-empty segments go to LDS (dropped records, unset values): a chunk then usually
    // covers one or two of them, which the unrolled path below loads without a loop.
    const bool live = lane < cnt && len > 0;
    const u64 lm = __ballot(live);
    const int slot = __builtin_amdgcn_mbcnt_hi((u32)(lm >> 32), __builtin_amdgcn_mbcnt_lo((u32)lm, 0u));
    const int nl = __popcll(lm);
    const int span = (int)(D1 - D0);
    const bool nt = NT && (span <= kNtSpan || a.nt == 2);  // (st16; nt 2: at any span)
    if (live) {
        S.addr[slot] = (u64)(uintptr_t)(a.in + src);
        S.o[slot] = (int)(d - D0);
    }
    if (lane == 0) S.o[nl] = span;
    // a 16-byte window reads up to 15 bytes either side of its segment
    const bool safe = __all(!live || (src >= in_lo + 16 && src + len + 16 <= in_hi));
    wave_sync();
    if (nl == 0) return;
    // the copy, instantiated per store kind (NT kernels only: with the nontemporal copy present in
    // the kernel the general reassembly path's gather ran 406 -> 440 us with plain stores selected)
    auto copy = [&](auto ntc) {
        constexpr bool NTS = decltype(ntc)::value;
        const i64 mis = (i64)((uintptr_t)a.out & 15);
        const int firstc = (int)((((i64)D0 + mis) & ~(i64)15) - mis - (i64)D0);  // in (-16, 0]
        uint8_t* const out_t = a.out + D0;
        if (safe) {
            // kU chunks per lane per step: every load of the step is issued before its stores
            constexpr int kU = KU;
            for (int B = firstc; B < span; B += 16 * 64 * kU) {  // wave-uniform loop
                u32x4 r[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int P = B + 16 * 64 * u + 16 * lane;
                    r[u] = u32x4{0, 0, 0, 0};
                    if (P >= span) continue;
                    const int k0 = lds_search_64(S.o, nl, max(P, 0));
                    const int o0 = S.o[k0], o1 = S.o[k0 + 1];
                    const bool two = k0 + 1 < nl && o1 < P + 16;  // the next segment starts in this chunk
                    const int o2 = two ? S.o[k0 + 2] : o1;
                    const uintptr_t X0 = (uintptr_t)(S.addr[k0] + (u64)(i64)(P - o0));
                    r[u] = ld16u(X0) & range_mask(masks, o0 - P, o1 - P);
                    if (two)  // (a chunk inside one segment, the usual case, issues one load)
                        r[u] |= ld16u((uintptr_t)(S.addr[k0 + 1] + (u64)(i64)(P - o1))) & range_mask(masks, o1 - P, o2 - P);
                    for (int k = k0 + 2; two && k < nl && S.o[k] < P + 16; ++k)  // segments < 16 bytes
                        r[u] |= ld16u((uintptr_t)(S.addr[k] + (u64)(i64)(P - S.o[k]))) &
                                range_mask(masks, S.o[k] - P, S.o[k + 1] - P);
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int P = B + 16 * 64 * u + 16 * lane;
                    if (P >= span) continue;
                    const u32 rr[4] = {r[u].x, r[u].y, r[u].z, r[u].w};
                    store_chunk(out_t, P, 0, span, rr, NTS);
                }
            }
            return;
        }
        for (int B = firstc; B < span; B += 16 * 64) {  // batch-edge waves: aligned blocks only
            const int P = B + 16 * lane;
            if (P >= span) continue;
            u32 t[4] = {0, 0, 0, 0};
            for (int k = lds_search_64(S.o, nl, max(P, 0)); k < nl; ++k) {
                const int lo = S.o[k] - P;
                if (lo >= 16) break;
                const int hi = min(S.o[k + 1] - P, 16);
                or_window_global((uintptr_t)(S.addr[k] + (u64)(i64)(P - S.o[k])), max(lo, 0), hi, t);
            }
            store_chunk(out_t, P, 0, span, t, NTS);
        }
    };
    if constexpr (NT) {
        if (nt) copy(std::true_type{});
        else copy(std::false_type{});
    } else {
        copy(std::false_type{});
    }
}

}  // namespace raw
}  // namespace symhip
