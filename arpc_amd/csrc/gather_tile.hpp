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
    if (total.bytes > a.cap) {  // output does not fit: nothing is written (uniform)
        if (i == 0) atomicOr(a.err, kErrCapacity);
        return;
    }
    const Pair tp = a.pre[tile];
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
    const bool nt = NT && span <= kNtSpan;  // (st16)
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
