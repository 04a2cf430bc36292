// pipe_words.hpp -- epoch-tagged aggregate / prefix words shared by the pipelined launches
// (decode_pipe.hip: parsers -> scanner -> copiers; encode.hip mixed batches: sizers -> scanner ->
// encode tiles).  A word is its own flag: 8 bytes {epoch, status, value} written and polled with
// agent-scope relaxed atomics (MI355X_MICROARCH.md visibility, form "R2"); the epoch tag means the
// words never need clearing between calls (sym_ctx owns them; capi.cpp next_epoch()).
#pragma once
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {
namespace pipe {

// Word: [63:44] epoch, [43:42] status (1 = aggregate, 2 = exclusive prefix), [41:0] value.
constexpr int kEpochShift = 44;
constexpr u64 kStAgg = 1ull << 42;
constexpr u64 kStPre = 2ull << 42;
constexpr u64 kValMask = (1ull << 42) - 1;
// Bounded waits, in wall time (s_memrealtime runs at 100 MHz).  No wait is needed for progress: a
// scanner idle for kWaitTicks exits (its consumers look back instead), and a consumer whose word has
// not come after kFallbackTicks resolves it itself, so the grid always drains with correct results
// (kErrTimeout is therefore never set).
constexpr u64 kWaitTicks = 25000000;  // 250 ms: the scanner gives up (copiers fall back) after this idle time
constexpr u64 kFallbackTicks = 100000; // 1 ms: a copier waits this long for its prefix before looking back
__device__ __forceinline__ u64 now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ u64 lane_u64_pub(u64 v, int l) {
    return (u64)(u32)__builtin_amdgcn_readlane((u32)v, l) | ((u64)(u32)__builtin_amdgcn_readlane((u32)(v >> 32), l) << 32);
}
__device__ __forceinline__ bool tagged(u64 w, u32 epoch) { return (u32)(w >> kEpochShift) == epoch; }
__device__ __forceinline__ u64 make_word(u32 epoch, u64 st, u64 v) {
    return ((u64)epoch << kEpochShift) | st | (v & kValMask);
}
__device__ __forceinline__ void store_word(u64* w, u64 v) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 load_word(u64* w) { return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Workgroup barrier that orders LDS only: outstanding global stores keep flying (__syncthreads()
// would wait for them).  Global loads whose data is used were waited on at their use.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------- the streaming scanner
struct ScanLds {  // the scanner's scratch (a 256-thread scanner)
    u64 red[4];
    int first[4];
};

// One workgroup of NT threads.  Each step takes the aggregate words of the next NT*SK tiles, finds
// the first tile whose word is not yet published (the frontier), and publishes the exclusive prefix
// of every tile before it.  A tile's prefix so depends only on earlier tiles, whoever published
// their aggregates.  S needs u64 red[NT/64] and int first[NT/64].
//
// The next step's window (from the new frontier on) is loaded BEFORE this step's prefix stores are
// issued: gfx950's vmcnt counts loads and stores in one in-order counter, so loads issued after the
// stores would wait for the stores' write acknowledgements too -- two memory round trips per step
// instead of one.  For the same reason every lane issues all of its SK stores (lanes past the
// frontier write into `sink`, the >= 256 bytes after the prefix words: decode_pipe_flag_bytes()),
// so no path through the step has fewer stores after the loads than another.
template <int NV, int SK, int NT = 256, typename LdsT>
__device__ void scanner(u64* aw, u64* pw, u64 ntiles, u32 epoch, LdsT& S, u64* dbg = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kPer = SK;  // tiles per thread per step
    constexpr int kW = NT / 64;  // waves
    constexpr u64 kStep = (u64)NT * kPer;
    u64* const sink = pw + (size_t)NV * ntiles + (lane & 31);
    const auto load_window = [&](u64 (&w)[NV][kPer], u64 b) {  // unconditional loads (clamped index)
        const u64 t0 = b + (u64)tid * kPer;
#pragma unroll
        for (int f = 0; f < NV; ++f)
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const u64 x = load_word(&aw[(size_t)f * ntiles + min(t0 + k, ntiles - 1)]);
                w[f][k] = t0 + k < ntiles ? x : make_word(epoch, kStAgg, 0);
            }
    };
    u64 carry[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) carry[f] = 0;
    u64 idle_since = 0;  // 0: the frontier moved on the last step
    u64 v[NV][kPer];
    load_window(v, 0);
    for (u64 base = 0; base < ntiles;) {
        const u64 t0 = base + (u64)tid * kPer;
        u32 miss = (u32)kStep;  // this thread's first unpublished tile (relative to base)
#pragma unroll
        for (int k = kPer - 1; k >= 0; --k) {
            bool ok = true;
#pragma unroll
            for (int f = 0; f < NV; ++f) ok = ok && tagged(v[f][k], epoch);
            if (!ok) miss = (u32)(tid * kPer + k);
        }
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) miss = min(miss, (u32)__shfl_xor((int)miss, d, 64));
        if (lane == 0) S.first[wave] = (int)miss;
        lds_barrier();
        u32 m = (u32)S.first[0];
#pragma unroll
        for (int q = 1; q < kW; ++q) m = min(m, (u32)S.first[q]);
        lds_barrier();  // S.first is rewritten by the next step
        m = (u32)min((u64)m, ntiles - base);
        if (m == 0) {  // the frontier has not moved: wait a little (bounded), then look again
            const u64 t = uniform_i64((i64)now_ticks());
            if (idle_since == 0) idle_since = t;
            if (t - idle_since > kWaitTicks) return;  // the consumers resolve the rest by look-back
            __builtin_amdgcn_s_sleep(2);
            load_window(v, base);
            continue;
        }
        idle_since = 0;
        u64 nv[NV][kPer];
        load_window(nv, base + m);  // in flight while this step's prefixes are computed and stored
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            u64 x[kPer], sum = 0;
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                x[k] = (u32)(tid * kPer + k) < m ? v[f][k] & kValMask : 0;
                sum += x[k];
            }
            // word values are 42-bit, so up to two of them sum below 2^43: DPP scan (no shuffles)
            u64 inc;
            if constexpr (kPer <= 2) inc = wave_incl_scan_u43_dpp(sum);
            else inc = wave_incl_scan_u64(sum, lane);
            if (lane == 63) S.red[wave] = inc;
            lds_barrier();
            u64 wpre = 0, tot = 0;
#pragma unroll
            for (int q = 0; q < kW; ++q) {
                const u64 t = S.red[q];
                if (q < wave) wpre += t;
                tot += t;
            }
            lds_barrier();  // S.red is rewritten for the next column / step
            u64 run = carry[f] + wpre + inc - sum;
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const bool mine = (u32)(tid * kPer + k) < m;
                store_word(mine ? &pw[(size_t)f * ntiles + t0 + k] : sink, make_word(epoch, kStPre, run));
                run += x[k];
            }
            carry[f] += tot;
        }
        if (dbg) {  // tuning timelines only
#pragma unroll
            for (int k = 0; k < kPer; ++k)
                if ((u32)(tid * kPer + k) < m) dbg[(t0 + k) * 8 + 5] = now_ticks();
        }
        base += m;
#pragma unroll
        for (int f = 0; f < NV; ++f)
#pragma unroll
            for (int k = 0; k < kPer; ++k) v[f][k] = nv[f][k];
    }
}

// ---------------------------------------------------------------- look-back (the fallback)
// Exclusive prefix of `tile` per column (wave 0 of its copier; lane k looks at tile hi - k).  The
// nearest earlier tile with a published prefix word ends the walk: prefix = its prefix + its
// aggregate + the aggregates of the tiles in between.  Never waits: a missing aggregate is computed
// here by tile_agg(t, a) (the whole wave; a[] wave-uniform) and published.
template <int NV, typename AggFn>
__device__ void lookback_with(u64* aw, u64* pw, u64 ntiles, u64 tile, u32 epoch, i64 (&pre)[NV], AggFn&& tile_agg) {
    const int lane = threadIdx.x & 63;
    u64 sum[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) sum[f] = 0;
    for (i64 hi = (i64)tile - 1; hi >= 0; hi -= 64) {  // wave-uniform loop
        const i64 t = hi - lane;
        const bool valid = t >= 0;
        u64 pv[NV], av[NV];
        bool hp = valid, ha = valid;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            pv[f] = valid ? load_word(&pw[(size_t)f * ntiles + t]) : 0;
            av[f] = valid ? load_word(&aw[(size_t)f * ntiles + t]) : 0;
            hp = hp && tagged(pv[f], epoch);
            ha = ha && tagged(av[f], epoch);
        }
        const u64 pm = __ballot(hp);
        const int stop = pm ? (int)__builtin_ctzll(pm) : 64;  // lanes [0, stop] contribute
        u64 need = __ballot(valid && lane <= stop && !ha);
        while (need) {  // wave-uniform
            const int k = (int)__builtin_ctzll(need);
            need &= need - 1;
            u64 a[NV];
            tile_agg((u64)(hi - k), a);  // whole wave; wave-uniform a[]
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                if (lane == k) av[f] = make_word(epoch, kStAgg, a[f]);
                if (lane == 0) store_word(&aw[(size_t)f * ntiles + (u64)(hi - k)], make_word(epoch, kStAgg, a[f]));
            }
        }
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 c = valid && lane <= stop ? (av[f] & kValMask) + (lane == stop ? pv[f] & kValMask : 0) : 0;
            sum[f] += (u64)uniform_i64((i64)wave_sum_u64(c));
        }
        if (pm) break;
    }
#pragma unroll
    for (int f = 0; f < NV; ++f) pre[f] = (i64)sum[f];
}

}  // namespace pipe
}  // namespace symhip
