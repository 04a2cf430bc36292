// decode.hip -- batched Symphony UnmarshalSymphony for flat schemas on gfx950.
//
// Restates, for n records at once, the generated per-record unmarshaller into a fresh
// struct: benchmark/kv-store-symphony/symphony/kv.syn.go:680-745 (SetRequest; Get/Resp
// analogous), examples/echo_symphony/symphony/echo.syn.go:186-263 (int32 fields), from the
// generator's rules cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:622-694, :734-793.
//
// Design (single pass, decoupled look-back):
//  * Workgroups take tiles of kTile=256 records in ticket order (atomic counter), so every
//    tile a workgroup waits on is already held by a running workgroup.
//  * Parse (one thread per record): Go's three header checks and, per field, the table
//    entry / length-prefix bounds checks in 64-bit arithmetic; emits the status byte,
//    int32 fields, and each string field's (source position, length).
//  * Scan: 64-lane shuffle scan + LDS across the 4 waves gives tile-local column offsets;
//    wave 0 publishes the tile aggregate, looks back over predecessors' 8-byte
//    {flag, value} words (agent-scope relaxed atomics, the word IS the flag) and publishes
//    the inclusive prefix.
//  * Copy (one thread per aligned 16-byte chunk of each output column): binary search of
//    the chunk's first field, funnel-shifted aligned loads from the record stream, one
//    global_store_dwordx4 per chunk; byte stores only at the tile's two column edges.
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

constexpr u64 kFlagAgg = 1ull << 62;
constexpr u64 kFlagInc = 2ull << 62;
constexpr u64 kValMask = (1ull << 62) - 1;
constexpr unsigned kSpinLimit = 1u << 22;

size_t decode_workspace_bytes(int nvar, uint64_t n) {
    const uint64_t tiles = (n + kTile - 1) / kTile;
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
        u64 v = w & kValMask;
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

template <int NF, int NV>
__global__ __launch_bounds__(256) void decode_kernel(DecodeParams p) {
    __shared__ u64 s_dst[NV][kTile + 1];  // tile-local exclusive column offsets; [cnt..] = aggregate
    __shared__ u64 s_src[NV][kTile];      // payload position in the input stream (relative to p.in)
    __shared__ u64 s_wsum[NV][4];
    __shared__ u64 s_prefix[NV];
    __shared__ unsigned s_tile;

    DecodeWsHeader* hdr = (DecodeWsHeader*)p.ws;
    const u64 ntiles = (p.n + kTile - 1) / kTile;
    u64* look = (u64*)((char*)p.ws + sizeof(DecodeWsHeader));

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(&hdr->ticket, 1u);
    __syncthreads();
    const u64 tile = s_tile;
    const u64 r0 = tile * kTile;
    const int cnt = (int)min((u64)kTile, p.n - r0);

    // ---------------- parse: Go's UnmarshalSymphony checks, one record per thread ----------------
    u64 flen[NV], fsrc[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) flen[f] = fsrc[f] = 0;
    if (tid < cnt) {
        const u64 r = r0 + tid;
        const u64 start = p.rec_off[r];
        const u64 len = p.rec_off[r + 1] - start;
        const uintptr_t d = (uintptr_t)(p.in + start);
        u32 st = 0;
        int32_t fx[NF > 0 ? NF : 1];
#pragma unroll
        for (int f = 0; f < (NF > 0 ? NF : 1); ++f) fx[f] = 0;
        if (len < 13) {
            st = 1;  // "invalid data: too short"
        } else if (ld_u8(d) != 0x01) {
            st = 2;  // "invalid data: wrong public version"
        } else {
            const u64 off2p = ld_u32(d + 1);
            if (off2p >= len || ld_u8(d + off2p) != 0x01) {
                st = 3;  // "missing private segment"
            } else {
                const u64 pts = off2p + 1;
                u64 toff = 0;
#pragma unroll
                for (int f = 0; f < NF; ++f, toff += 4) {
                    if (st == 0) {
                        if (len < pts + toff + 4) st = 4;  // "invalid data: too short for field"
                        else fx[f] = (int32_t)ld_u32(d + pts + toff);
                    }
                }
                if (st == 0) {
#pragma unroll
                    for (int f = 0; f < NV; ++f, toff += 4) {
                        if (len >= pts + toff + 4) {
                            u64 po = ld_u32(d + pts + toff);
                            if (po > 0) po += off2p;
                            if (po > 0 && len >= po + 4) {
                                const u64 nb = ld_u32(d + po);
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

    // ---------------- tile scan of field lengths ----------------
    u64 incl[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        incl[f] = wave_incl_scan_u64(flen[f], lane);
        if (lane == 63) s_wsum[f][wave] = incl[f];
    }
    __syncthreads();
    u64 agg[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        u64 wbase = 0;
        agg[f] = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            if (w < wave) wbase += s_wsum[f][w];
            agg[f] += s_wsum[f][w];
        }
        s_dst[f][tid] = wbase + incl[f] - flen[f];
        s_src[f][tid] = fsrc[f];
        if (tid == 0) s_dst[f][kTile] = agg[f];
    }
    if (wave == 0) {
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 pre = lookback(look + (u64)f * ntiles, tile, agg[f], p.err, lane);
            if (lane == 0) s_prefix[f] = pre;
        }
    }
    __syncthreads();

    if (tid < cnt) {
        const u64 r = r0 + tid;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            p.offs[f][r] = s_prefix[f] + s_dst[f][tid];
            if (r == p.n - 1) p.offs[f][p.n] = s_prefix[f] + agg[f];
        }
    }

    // ---------------- copy: one aligned 16-byte chunk of each output column per thread ----------------
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const i64 col_lo = (i64)s_prefix[f];
        const i64 col_hi = col_lo + (i64)agg[f];
        const i64 cap = (i64)p.cap[f];
        if (tid == 0 && col_hi > cap) atomicOr(p.err, kErrCapacity);
        const i64 lim = col_hi < cap ? col_hi : cap;
        const i64 mis = (i64)((uintptr_t)p.bytes[f] & 15);
        const i64 first = ((col_lo + mis) & ~(i64)15) - mis;
        const u64* dst = s_dst[f];
        for (i64 P = first + 16 * tid; P < lim; P += 16 * kTile) {
            const i64 Pc = P > col_lo ? P : col_lo;
            const int j = lds_search_256(dst, cnt, (u64)(Pc - col_lo));
            u32 r[4] = {0, 0, 0, 0};
            for (int k = j; k < cnt; ++k) {
                const i64 dk = col_lo + (i64)dst[k];
                if (dk >= P + 16) break;
                const i64 L = (i64)(dst[k + 1] - dst[k]);
                if (L == 0) continue;
                const i64 tlo = dk - P > 0 ? dk - P : 0;
                const i64 thi = dk + L - P < 16 ? dk + L - P : 16;
                const uintptr_t X = (uintptr_t)(p.in + s_src[f][k]) + (uintptr_t)(P - dk);
                or_window_global(X, (int)tlo, (int)thi, r);
            }
            store_chunk(p.bytes[f], P, col_lo, lim, r);
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
    const dim3 grid((unsigned)((p.n + kTile - 1) / kTile));
    const dim3 block(256);
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
