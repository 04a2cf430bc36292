// decode.hip -- batched Symphony UnmarshalSymphony for flat schemas on gfx950.
//
// Restates, for n records at once, the generated per-record unmarshaller into a fresh
// struct: benchmark/kv-store-symphony/symphony/kv.syn.go:680-745 (SetRequest; Get/Resp
// analogous), examples/echo_symphony/symphony/echo.syn.go:186-263 (int32 fields), from the
// generator's rules cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:622-694, :734-793.
//
// Design (single pass, one tile of kWaveRecs=64 records per wave, decoupled look-back):
//  * Waves take tiles in ticket order (atomic counter), so every tile a wave waits on is
//    already held by a running wave; the 4 waves of a workgroup never synchronize.
//  * Parse (lane = record): the record's first 48 bytes land in LDS with three byte-unaligned
//    16-byte loads; Go's header checks and, per field, the table-entry / length-prefix bounds
//    checks (64-bit arithmetic, as Go's int) read from there, or from global memory for
//    offsets past the window.  Emits the status byte, int32 fields, and each string
//    field's (source position, length).
//  * Scan: 64-lane shuffle scan of the field lengths; the wave publishes its tile aggregate,
//    looks back over predecessors' 8-byte {flag, value} words (agent-scope relaxed atomics;
//    the word IS the flag) and publishes its inclusive prefix.
//  * Copy (lane = aligned 16-byte chunk of an output column, natural order): a chunk inside
//    one field is one byte-unaligned 16-byte load from the record stream; chunks spanning
//    field ends merge masked windows.  One global_store_dwordx4 per chunk; byte stores only
//    at the tile's two column edges.
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

constexpr int kWaveRecs = 64;
constexpr int kWaves = 4;
constexpr int kWin = 48;  // header bytes staged per record
constexpr u64 kFlagAgg = 1ull << 62;
constexpr u64 kFlagInc = 2ull << 62;
constexpr u64 kValMask = (1ull << 62) - 1;
constexpr unsigned kSpinLimit = 1u << 22;

size_t decode_workspace_bytes(int nvar, uint64_t n) {
    const uint64_t tiles = (n + kWaveRecs - 1) / kWaveRecs;
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
};

template <int NF, int NV>
__global__ __launch_bounds__(256) void decode_kernel(DecodeParams p) {
    __shared__ DecWaveLds<NV> lds_all[kWaves];
    __shared__ MaskTable masks;
    mask_table_init(masks, threadIdx.x);
    __syncthreads();  // the only workgroup barrier

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    DecWaveLds<NV>& S = lds_all[wave];
    const u64 ntiles = (p.n + kWaveRecs - 1) / kWaveRecs;
    DecodeWsHeader* hdr = (DecodeWsHeader*)p.ws;
    u64* look = (u64*)((char*)p.ws + sizeof(DecodeWsHeader));

    u32 ticket = 0;
    if (lane == 0) ticket = atomicAdd(&hdr->ticket, 1u);
    const u64 tile = (u64)__shfl((int)ticket, 0, 64);
    if (tile >= ntiles) return;  // surplus wave of the last workgroup
    const u64 r0 = tile * kWaveRecs;
    const int cnt = (int)min((u64)kWaveRecs, p.n - r0);

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
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u64 inc = wave_incl_scan_u64(flen[f], lane);
        agg[f] = (u64)__shfl((long long)inc, 63, 64);
        excl[f] = inc - flen[f];
    }
    bool too_large = false;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        prefix[f] = lookback(look + (u64)f * ntiles, tile, agg[f], p.err, lane);
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
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        S.dst[f][lane] = (int)excl[f];  // lanes >= cnt hold the aggregate
        S.src[f][lane] = fsrc[f];
    }
    if (lane == 0) {
#pragma unroll
        for (int f = 0; f < NV; ++f) S.dst[f][kWaveRecs] = (int)agg[f];
    }
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
        for (int P = first + 16 * lane; P < lim; P += 16 * 64) {
            const int j = lds_search_64(dst, cnt, max(P, 0));
            const int dj = dst[j], Lj = dst[j + 1] - dj;
            const uintptr_t Xj = (uintptr_t)(p.in + S.src[f][j]) + (uintptr_t)(i64)(P - dj);
            u32x4 r;
            if (P >= dj && P + 16 <= dj + Lj) {
                r = ld16u(Xj);  // the whole chunk comes from one field: [Xj, Xj+16) is in the record
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

hipError_t launch_decode(const DecodeParams& p, hipStream_t stream) {
    hipError_t e;
    if (p.n == 0) {
        for (int f = 0; f < p.lay.nvar; ++f)
            if ((e = hipMemsetAsync(p.offs[f], 0, sizeof(uint64_t), stream)) != hipSuccess) return e;
        return hipSuccess;
    }
    if ((e = hipMemsetAsync(p.ws, 0, decode_workspace_bytes(p.lay.nvar, p.n), stream)) != hipSuccess) return e;
    const u64 tiles = (p.n + kWaveRecs - 1) / kWaveRecs;
    const dim3 grid((unsigned)((tiles + kWaves - 1) / kWaves));
    const dim3 block(64 * kWaves);
    if (p.lay.nfixed == 0 && p.lay.nvar == 1)
        hipLaunchKernelGGL((decode_kernel<0, 1>), grid, block, 0, stream, p);
    else if (p.lay.nfixed == 0 && p.lay.nvar == 2)
        hipLaunchKernelGGL((decode_kernel<0, 2>), grid, block, 0, stream, p);
    else if (p.lay.nfixed == 2 && p.lay.nvar == 2)
        hipLaunchKernelGGL((decode_kernel<2, 2>), grid, block, 0, stream, p);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace symhip
