// decode.hip -- batched Symphony UnmarshalSymphony for flat schemas on gfx950.
//
// Restates, for n records at once, the generated per-record unmarshaller into a fresh
// struct: benchmark/kv-store-symphony/symphony/kv.syn.go:680-745 (SetRequest; Get/Resp
// analogous), examples/echo_symphony/symphony/echo.syn.go:186-263 (int32 fields), from the
// generator's rules cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:622-694, :734-793.
//
// Design (single pass, one tile of kWaveRecs=64 records per wave, decoupled look-back):
//  * Workgroups (16 waves, 1024 records) take look-back tiles in ticket order (one atomic
//    per workgroup: a single counter word sustains only ~88 increments/us), so every tile a
//    workgroup waits on is already held by a running workgroup.  Tiles of 1024 records keep
//    the look-back shallow even when hundreds of workgroups start together.
//  * Parse (lane = record): the record's first 48 bytes land in LDS with three byte-unaligned
//    16-byte loads; Go's header checks and, per field, the table-entry / length-prefix bounds
//    checks (64-bit arithmetic, as Go's int) read from there, or from global memory for
//    offsets past the window.  Emits the status byte, int32 fields, and each string
//    field's (source position, length).
//  * Scan: 64-lane DPP scan of the field lengths per wave, wave aggregates through LDS; wave 0
//    publishes the tile aggregate, looks back over predecessors' 8-byte {flag, value} words
//    (agent-scope relaxed atomics; the word IS the flag) and publishes the inclusive prefix.
//  * Copy (lane = aligned 16-byte chunk of an output column, natural order): a chunk inside
//    one field is one byte-unaligned 16-byte load from the record stream; chunks spanning
//    field ends merge masked windows.  One global_store_dwordx4 per chunk; byte stores only
//    at the tile's two column edges.
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

constexpr int kWaveRecs = 64;                    // records per wave (parse / copy unit)
constexpr int kWaves = 16;                       // waves per 1024-thread workgroup
constexpr int kTileRecs = kWaveRecs * kWaves;    // records per look-back tile (one per workgroup)
constexpr int kWin = 48;  // header bytes staged per record
constexpr u64 kFlagAgg = 1ull << 62;
constexpr u64 kFlagInc = 2ull << 62;
constexpr u64 kValMask = (1ull << 62) - 1;
constexpr unsigned kSpinLimit = 1u << 22;

size_t decode_workspace_bytes(int nvar, uint64_t n) {
    const uint64_t tiles = (n + kTileRecs - 1) / kTileRecs;
    const size_t bytes = sizeof(DecodeWsHeader) + (size_t)nvar * tiles * sizeof(uint64_t);
    return (bytes + 15) & ~(size_t)15;
}

// Decoupled look-back for one column, run by one full wave.  Returns the tile's exclusive prefix.
__device__ u64 lookback(u64* words, u64 tile, u64 agg, unsigned* err, int lane) {
    if (tile == 0) {
        if (lane == 0) __hip_atomic_store(&words[0], kFlagInc | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&words[tile], kFlagAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u64 excl = 0;
    i64 base = (i64)tile - 1;
    for (;;) {
        const i64 idx = base - lane;
        u64 w = kFlagInc;  // virtual predecessor of tile 0
        if (idx >= 0) {
            unsigned spins = 0;
            for (;;) {
                w = __hip_atomic_load(&words[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((w >> 62) != 0 || ++spins >= kSpinLimit) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if ((w >> 62) == 0) {  // timed out: report, and stop here so the kernel drains
                atomicOr(err, kErrTimeout);
                w = kFlagInc;
            }
        }
        const u64 inc = __ballot((w >> 62) == 2);
        const u64 v = w & kValMask;
        if (inc) {
            const int pl = __ffsll((long long)inc) - 1;
            excl += wave_sum_u64(lane <= pl ? v : 0);
            break;
        }
        excl += wave_sum_u64(v);
        base -= 64;
    }
    if (lane == 0) __hip_atomic_store(&words[tile], kFlagInc | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

template <int NV>
struct alignas(16) DecWaveLds {
    uint8_t win[kWaveRecs * kWin];  // first kWin bytes of each record (parse)
    int dst[NV][kWaveRecs + 1];     // field start in the tile's column range; [cnt] = tile aggregate
    u64 src[NV][kWaveRecs];         // payload position in the input stream
    u32 counts[64];                 // record starts per chunk of one copy step
};

// DIAG (timing diagnostics only, tools/kbench.py): 1 = skip the copy, 2 = skip the look-back.
template <int NF, int NV, int DIAG>
__global__ __launch_bounds__(1024) void decode_kernel(DecodeParams p) {
    __shared__ DecWaveLds<NV> lds_all[kWaves];
    __shared__ MaskTable masks;
    __shared__ u64 s_wagg[NV][kWaves];  // wave aggregates
    __shared__ u64 s_tile_prefix[NV];
    __shared__ u32 s_ticket;

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    DecWaveLds<NV>& S = lds_all[wave];
    const u64 ntiles = (p.n + kTileRecs - 1) / kTileRecs;
    DecodeWsHeader* hdr = (DecodeWsHeader*)p.ws;
    u64* look = (u64*)((char*)p.ws + sizeof(DecodeWsHeader));

    if (threadIdx.x == 0) s_ticket = atomicAdd(&hdr->ticket, 1u);
    mask_table_init(masks, threadIdx.x);
    __syncthreads();
    const u64 tile = (u64)__builtin_amdgcn_readfirstlane(s_ticket);  // grid size == ntiles
    const u64 r0 = tile * kTileRecs + (u64)wave * kWaveRecs;
    const int cnt = r0 < p.n ? (int)min((u64)kWaveRecs, p.n - r0) : 0;  // 0: wave past the end

    // ---------------- parse: Go's UnmarshalSymphony checks, one record per lane ----------------
    u64 flen[NV], fsrc[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) flen[f] = fsrc[f] = 0;
    u64 start = 0, len = 0;
    if (lane < cnt) {
        start = p.rec_off[r0 + lane];
        len = p.rec_off[r0 + lane + 1] - start;
    }
    const uintptr_t d = (uintptr_t)(p.in + start);
    const bool win = lane < cnt && len >= (u64)kWin;  // window loads stay inside the record
    if (win) {
#pragma unroll
        for (int k = 0; k < kWin / 16; ++k) *(u32x4*)&S.win[lane * kWin + 16 * k] = ld16u(d + 16 * k);
    }
    wave_sync();
    const uint8_t* wb = &S.win[lane * kWin];
    auto rd8 = [&](u64 q) -> u32 { return (win && q < (u64)kWin) ? (u32)wb[q] : ld_u8(d + q); };
    auto rd32 = [&](u64 q) -> u32 {
        return (win && q + 4 <= (u64)kWin) ? *(const u32*)(wb + q) : *(gc_u32*)(d + q);  // unaligned OK
    };
    if (lane < cnt) {
        const u64 r = r0 + lane;
        u32 st = 0;
        int32_t fx[NF > 0 ? NF : 1];
#pragma unroll
        for (int f = 0; f < (NF > 0 ? NF : 1); ++f) fx[f] = 0;
        if (len < 13) {
            st = 1;  // "invalid data: too short"
        } else if (rd8(0) != 0x01) {
            st = 2;  // "invalid data: wrong public version"
        } else {
            const u64 off2p = rd32(1);
            if (off2p >= len || rd8(off2p) != 0x01) {
                st = 3;  // "missing private segment"
            } else {
                const u64 pts = off2p + 1;
                u64 toff = 0;
#pragma unroll
                for (int f = 0; f < NF; ++f, toff += 4) {
                    if (st == 0) {
                        if (len < pts + toff + 4) st = 4;  // "invalid data: too short for field"
                        else fx[f] = (int32_t)rd32(pts + toff);
                    }
                }
                if (st == 0) {
#pragma unroll
                    for (int f = 0; f < NV; ++f, toff += 4) {
                        if (len >= pts + toff + 4) {
                            u64 po = rd32(pts + toff);
                            if (po > 0) po += off2p;
                            if (po > 0 && len >= po + 4) {
                                const u64 nb = rd32(po);
                                if (len >= po + 4 + nb) {
                                    fsrc[f] = start + po + 4;
                                    flen[f] = nb;
                                }
                            }
                        }
                    }
                }
            }
        }
        p.status[r] = (uint8_t)st;
#pragma unroll
        for (int f = 0; f < NF; ++f) p.fixed[f][r] = fx[f];
    }

    // ---------------- scan + look-back ----------------
    u64 prefix[NV], agg[NV], excl[NV];
    // 32-bit DPP scan unless some field in the tile is >= 2^26 bytes (then 64-bit shuffles)
    bool small = true;
#pragma unroll
    for (int f = 0; f < NV; ++f) small = small && flen[f] < (1u << 26);
    const bool all_small = __ballot(!small) == 0;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u64 inc = all_small ? (u64)wave_incl_scan_u32_dpp((u32)flen[f]) : wave_incl_scan_u64(flen[f], lane);
        agg[f] = (u64)uniform_i64((i64)__shfl((long long)inc, 63, 64));
        excl[f] = inc - flen[f];
    }
    // tile scan: wave aggregates -> wave 0 looks back once for the whole workgroup
    if (lane == 0) {
#pragma unroll
        for (int f = 0; f < NV; ++f) s_wagg[f][wave] = agg[f];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 tile_agg = lane < kWaves ? s_wagg[f][lane] : 0;
            const u64 tsum = (u64)uniform_i64((i64)wave_sum_u64(tile_agg));
            u64 pre;
            if constexpr (DIAG == 2) {
                pre = tile * tsum;  // timing only: no look-back (offsets wrong unless tiles are equal)
            } else {
                pre = lookback(look + (u64)f * ntiles, tile, tsum, p.err, lane);
            }
            if (lane == 0) s_tile_prefix[f] = pre;
        }
    }
    __syncthreads();
    bool too_large = false;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        u64 pre = s_tile_prefix[f];
        for (int w = 0; w < wave; ++w) pre += s_wagg[f][w];
        prefix[f] = (u64)uniform_i64((i64)pre);
        too_large |= agg[f] >= ((u64)1 << 31);
    }
    if (lane < cnt) {
        const u64 r = r0 + lane;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            p.offs[f][r] = prefix[f] + excl[f];
            if (r == p.n - 1) p.offs[f][p.n] = prefix[f] + agg[f];
        }
    }
    if (too_large) {  // column positions are 32-bit inside a tile
        if (lane == 0) atomicOr(p.err, kErrTooLarge);
        return;
    }
    if constexpr (DIAG == 1) return;  // timing only: no copy
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        S.dst[f][lane] = (int)excl[f];  // lanes >= cnt hold the aggregate
        S.src[f][lane] = fsrc[f];
    }
    if (lane == 0) {
#pragma unroll
        for (int f = 0; f < NV; ++f) S.dst[f][kWaveRecs] = (int)agg[f];
    }
    S.counts[lane] = 0;
    wave_sync();

    // ---------------- copy: natural-order chunks of each output column ----------------
    const uintptr_t in_lo = ((uintptr_t)(p.in + p.rec_off[0])) & ~(uintptr_t)15;
    const uintptr_t in_hi = ((uintptr_t)(p.in + p.rec_off[p.n]) + 15) & ~(uintptr_t)15;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const int span = (int)agg[f];
        if (span == 0) continue;
        const i64 C0 = (i64)prefix[f];
        const i64 cap = (i64)p.cap[f];
        if (lane == 0 && C0 + span > cap) atomicOr(p.err, kErrCapacity);
        const int lim = (int)max((i64)0, min((i64)span, cap - C0));
        const i64 mis = (i64)((uintptr_t)p.bytes[f] & 15);
        const int first = (int)(((C0 + mis) & ~(i64)15) - mis - C0);  // in (-16, 0]
        uint8_t* const out_t = p.bytes[f] + C0;
        const int* dst = S.dst[f];
        // record-role registers: lane k = record k's column start (tile-relative)
        const i64 my_d = lane < cnt ? (i64)excl[f] : ((i64)1 << 40);
        for (int B = first; B < lim; B += 16 * 64) {  // wave-uniform loop
            // Chunk l's record = (#records with start <= P_l) - 1.  Record k is first counted at
            // chunk ceil((d_k - B)/16); short fields can put several starts in one chunk, so
            // the marks are counts (LDS atomics) and a DPP scan turns them into prefix counts.
            const i64 ck = (my_d - B + 15) >> 4;
            const u64 before = __ballot(ck <= 0);
            if (ck >= 1 && ck <= 63) atomicAdd(&S.counts[ck], 1u);
            wave_sync();
            const u32 c = S.counts[lane];
            S.counts[lane] = 0;
            const u32 inc = __ballot(c > 1) == 0
                ? (u32)__builtin_amdgcn_mbcnt_hi((u32)(__ballot(c != 0) >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((u32)__ballot(c != 0), 0u)) + c
                : wave_incl_scan_u32_dpp(c);
            const int counted = (int)__popcll(before) + (int)inc;
            const int j = counted > 0 ? counted - 1 : 0;  // 0 only for the chunk straddling the tile start
            const int P = B + 16 * lane;
            if (P >= lim) continue;
            const int dj = dst[j], Lj = dst[j + 1] - dj;
            u32x4 r;
            if (P >= dj && P + 16 <= dj + Lj) {
                // the whole chunk comes from one field: [X, X+16) lies inside the record
                r = ld16u((uintptr_t)(p.in + S.src[f][j]) + (uintptr_t)(i64)(P - dj));
            } else {
                r = u32x4{0, 0, 0, 0};
                for (int k = j; k < cnt; ++k) {
                    const int dk = dst[k];
                    if (dk >= P + 16) break;
                    const int Lk = dst[k + 1] - dk;
                    if (Lk == 0) continue;
                    const uintptr_t X = (uintptr_t)(p.in + S.src[f][k]) + (uintptr_t)(i64)(P - dk);
                    u32x4 v;
                    if (X >= in_lo && X + 16 <= in_hi) {
                        v = ld16u(X);
                    } else {  // stream edges only: aligned blocks holding valid bytes
                        u32 tmp[4] = {0, 0, 0, 0};
                        or_window_global(X, max(dk - P, 0), min(dk + Lk - P, 16), tmp);
                        v = u32x4{tmp[0], tmp[1], tmp[2], tmp[3]};
                    }
                    r |= v & range_mask(masks, dk - P, dk + Lk - P);
                }
            }
            const u32 rr[4] = {r.x, r.y, r.z, r.w};
            store_chunk(out_t, P, 0, lim, rr);
        }
    }
}

template <int NF, int NV>
static void launch_layout(const DecodeParams& p, dim3 grid, dim3 block, hipStream_t stream) {
    if (p.variant == 101)
        hipLaunchKernelGGL((decode_kernel<NF, NV, 1>), grid, block, 0, stream, p);
    else if (p.variant == 102)
        hipLaunchKernelGGL((decode_kernel<NF, NV, 2>), grid, block, 0, stream, p);
    else
        hipLaunchKernelGGL((decode_kernel<NF, NV, 0>), grid, block, 0, stream, p);
}

hipError_t launch_decode(const DecodeParams& p, hipStream_t stream) {
    hipError_t e;
    if (p.n == 0) {
        for (int f = 0; f < p.lay.nvar; ++f)
            if ((e = hipMemsetAsync(p.offs[f], 0, sizeof(uint64_t), stream)) != hipSuccess) return e;
        return hipSuccess;
    }
    if ((e = hipMemsetAsync(p.ws, 0, decode_workspace_bytes(p.lay.nvar, p.n), stream)) != hipSuccess) return e;
    const dim3 grid((unsigned)((p.n + kTileRecs - 1) / kTileRecs));  // one look-back tile per workgroup
    const dim3 block(64 * kWaves);
    if (p.lay.nfixed == 0 && p.lay.nvar == 1)
        launch_layout<0, 1>(p, grid, block, stream);
    else if (p.lay.nfixed == 0 && p.lay.nvar == 2)
        launch_layout<0, 2>(p, grid, block, stream);
    else if (p.lay.nfixed == 2 && p.lay.nvar == 2)
        launch_layout<2, 2>(p, grid, block, stream);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace symhip
