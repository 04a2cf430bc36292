// decode.hip -- batched Symphony UnmarshalSymphony for flat schemas on gfx950.
//
// Restates, for n records at once, the generated per-record unmarshaller into a fresh
// struct: benchmark/kv-store-symphony/symphony/kv.syn.go:680-745 (SetRequest; Get/Resp
// analogous), examples/echo_symphony/symphony/echo.syn.go:186-263 (int32 fields), from the
// generator's rules cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:622-694, :734-793.
//
// Design (single pass, one tile of kWaveRecs=64 records per wave, decoupled look-back):
//  * Workgroups (8 record waves, 512 records, + 1 look-back wave) take look-back tiles in ticket
//    order (one atomic per workgroup: a single counter word sustains only ~88 increments/us),
//    so every tile a workgroup waits on is already held by a running workgroup.
//  * Parse (lane = record): the record's first 48 bytes land in LDS with three byte-unaligned
//    16-byte loads; Go's header checks and, per field, the table-entry / length-prefix bounds
//    checks (64-bit arithmetic, as Go's int) read from there, or from global memory for
//    offsets past the window.  Emits the status byte, int32 fields, and each string
//    field's (source position, length).
//  * Scan: 64-lane DPP scan of the field lengths per wave, wave aggregates through LDS.  A ninth
//    wave per workgroup publishes the tile aggregate, looks back over predecessors' 8-byte
//    {flag, value} words (agent-scope relaxed atomics; the word IS the flag) and publishes the
//    inclusive prefix; two columns run at once, one per half-wave, each lane checking 16 words
//    (a 512-tile window per step).  It runs while the record waves' copy loads are in flight.
//  * Copy: every field is a run of 16-byte chunks (the last one moved back to end at the field
//    end), so each chunk is one byte-unaligned 16-byte load and one 16-byte store.  A wave
//    issues the loads for its first kRB steps (64 chunks each) right after parsing -- the
//    header lines are still in L2, and the loads fly while the look-back wave works -- and
//    stores them once the tile prefix is known, refilling each register slot with the load
//    kRB steps ahead (a rolling pipeline) until its columns are done.
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

constexpr int kWaveRecs = 64;                    // records per wave (parse / copy unit)
constexpr int kWaves = 8;                        // record waves per workgroup
constexpr int kThreads = 64 * (kWaves + 1);      // + one look-back wave
constexpr int kTileRecs = kWaveRecs * kWaves;    // records per look-back tile (one per workgroup)
constexpr int kRB = 8;                            // 16-byte chunks per lane held across the look-back
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
// Lane l checks the kLookWords predecessors base-l*kLookWords-k (k = 0..kLookWords-1), so one step
// covers a window of 64*kLookWords tiles: enough to reach the last inclusive prefix in one step
// even when every resident workgroup publishes its aggregate at about the same time.
constexpr int kLookWords = 8;
__device__ u64 lookback(u64* words, u64 tile, u64 agg, unsigned* err, int lane) {
    if (tile == 0) {
        if (lane == 0) __hip_atomic_store(&words[0], kFlagInc | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&words[tile], kFlagAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u64 excl = 0;
    i64 base = (i64)tile - 1 - (i64)lane * kLookWords;
    for (;;) {
        u64 w[kLookWords];
#pragma unroll
        for (int k = 0; k < kLookWords; ++k)
            w[k] = base - k >= 0 ? __hip_atomic_load(&words[base - k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : kFlagInc;  // virtual predecessor of tile 0
        unsigned spins = 0;
        for (;;) {
            bool pending = false;
#pragma unroll
            for (int k = 0; k < kLookWords; ++k) pending |= (w[k] >> 62) == 0;
            if (!pending) break;
            if (++spins >= kSpinLimit) {  // timed out: report, and stop here so the kernel drains
                atomicOr(err, kErrTimeout);
#pragma unroll
                for (int k = 0; k < kLookWords; ++k)
                    if ((w[k] >> 62) == 0) w[k] = kFlagInc;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int k = 0; k < kLookWords; ++k)
                if ((w[k] >> 62) == 0)
                    w[k] = __hip_atomic_load(&words[base - k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // this lane's sum up to and including its nearest inclusive word
        u64 part = 0;
        bool inc = false;
#pragma unroll
        for (int k = 0; k < kLookWords; ++k) {
            if (!inc) part += w[k] & kValMask;
            inc |= (w[k] >> 62) == 2;
        }
        const u64 incs = __ballot(inc);
        if (incs) {
            const int pl = __ffsll((long long)incs) - 1;
            excl += wave_sum_u64(lane <= pl ? part : 0);
            break;
        }
        excl += wave_sum_u64(part);
        base -= 64 * kLookWords;
    }
    if (lane == 0) __hip_atomic_store(&words[tile], kFlagInc | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// Look-back for two columns at once: lanes 0-31 serve column 0, lanes 32-63 column 1, each lane
// checking kLookWords2 predecessors (a 512-tile window per half-wave and step).  Returns this
// lane's column's exclusive prefix.
constexpr int kLookWords2 = 16;
__device__ u64 lookback2(u64* words0, u64* words1, u64 tile, u64 agg0, u64 agg1, unsigned* err, int lane) {
    const int h = lane >> 5, hl = lane & 31;
    u64* words = h ? words1 : words0;
    const u64 agg = h ? agg1 : agg0;
    if (tile == 0) {
        if (hl == 0) __hip_atomic_store(&words[0], kFlagInc | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (hl == 0) __hip_atomic_store(&words[tile], kFlagAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u64 excl = 0;
    bool done = false;
    i64 base = (i64)tile - 1 - (i64)hl * kLookWords2;
    for (;;) {
        u64 part = 0;
        bool inc = false;
        if (!done) {
            u64 w[kLookWords2];
#pragma unroll
            for (int k = 0; k < kLookWords2; ++k)
                w[k] = base - k >= 0 ? __hip_atomic_load(&words[base - k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : kFlagInc;  // virtual predecessor of tile 0
            unsigned spins = 0;
            for (;;) {
                bool pending = false;
#pragma unroll
                for (int k = 0; k < kLookWords2; ++k) pending |= (w[k] >> 62) == 0;
                if (!pending) break;
                if (++spins >= kSpinLimit) {  // timed out: report, and stop here so the kernel drains
                    atomicOr(err, kErrTimeout);
#pragma unroll
                    for (int k = 0; k < kLookWords2; ++k)
                        if ((w[k] >> 62) == 0) w[k] = kFlagInc;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int k = 0; k < kLookWords2; ++k)
                    if ((w[k] >> 62) == 0)
                        w[k] = __hip_atomic_load(&words[base - k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int k = 0; k < kLookWords2; ++k) {
                if (!inc) part += w[k] & kValMask;
                inc |= (w[k] >> 62) == 2;
            }
        }
        const u64 incs = __ballot(inc);
        const u32 mine = h ? (u32)(incs >> 32) : (u32)incs;
        const int pl = mine ? __ffs((int)mine) - 1 : 31;
        const u64 s = wave_incl_scan_u64(!done && hl <= pl ? part : 0, lane);
        const u64 s31 = (u64)__shfl((long long)s, 31, 64), s63 = (u64)__shfl((long long)s, 63, 64);
        if (!done) excl += h ? s63 - s31 : s31;
        done = done || mine != 0;
        if (__ballot(!done) == 0) break;
        base -= 32 * kLookWords2;
    }
    if (hl == 0) __hip_atomic_store(&words[tile], kFlagInc | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

template <int NV>
struct alignas(16) DecWaveLds {
    uint8_t win[kWaveRecs * kWin];  // first kWin bytes of each record (parse)
    int dst[NV][kWaveRecs + 1];     // field start in the wave's column range; [cnt..] = wave aggregate
    int cs[NV][kWaveRecs];          // field's first copy chunk (exclusive scan of chunk counts)
    u64 src[NV][kWaveRecs];         // payload position in the input stream
    u32 mark[64];                   // record index + 1 at its first chunk, per copy step
};

// Two-way pick with wave-uniform selector (keeps small register arrays out of scratch).
template <int NV, typename T>
__device__ __forceinline__ T pick(const T (&a)[NV], bool second) {
    if constexpr (NV == 1) return a[0];
    else return second ? a[1] : a[0];
}

// DIAG (timing diagnostics only, tools/kbench.py, tools/decode_timeline.py): 1 = skip the copy,
// 2 = skip the look-back, 4 = full decode plus per-wave phase timestamps into p.dbg.
template <int NF, int NV, int DIAG, int KRB = kRB>
__global__ __launch_bounds__(kThreads) void decode_kernel(DecodeParams p) {
    static_assert(NV == 1 || NV == 2, "decode handles one or two string columns");
    __shared__ DecWaveLds<NV> lds_all[kWaves];
    __shared__ MaskTable masks;
    __shared__ u64 s_wagg[NV][kWaves];  // wave aggregates
    __shared__ u64 s_tile_prefix[NV];
    __shared__ u32 s_ticket;

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 ntiles = (p.n + kTileRecs - 1) / kTileRecs;
    DecodeWsHeader* hdr = (DecodeWsHeader*)p.ws;
    u64* look = (u64*)((char*)p.ws + sizeof(DecodeWsHeader));

    const u64 t_entry = DIAG == 4 ? __builtin_amdgcn_s_memrealtime() : 0;
    if (threadIdx.x == 0) s_ticket = atomicAdd(&hdr->ticket, 1u);
    mask_table_init(masks, threadIdx.x);
    __syncthreads();
    const u64 tile = (u64)__builtin_amdgcn_readfirstlane(s_ticket);  // grid size == ntiles
    auto mark = [&](int slot) {
        if constexpr (DIAG == 4) {
            if (lane == 0) p.dbg[(tile * (kWaves + 1) + wave) * 8 + slot] = __builtin_amdgcn_s_memrealtime();
        }
    };
    if constexpr (DIAG == 4) {
        if (lane == 0) p.dbg[(tile * (kWaves + 1) + wave) * 8] = t_entry;
    }
    mark(1);

    if (wave == kWaves) {
        // ---------------- look-back wave: runs while the record waves' copy loads fly ----------------
        __syncthreads();  // A: wave aggregates are in s_wagg
        mark(4);
        u64 tsum[NV];
#pragma unroll
        for (int f = 0; f < NV; ++f)
            tsum[f] = (u64)uniform_i64((i64)wave_sum_u64(lane < kWaves ? s_wagg[f][lane] : 0));
        if constexpr (DIAG == 2) {  // timing only: no look-back (offsets wrong unless tiles are equal)
            if (lane == 0) {
#pragma unroll
                for (int f = 0; f < NV; ++f) s_tile_prefix[f] = tile * tsum[f];
            }
        } else if constexpr (NV == 2) {  // both columns at once, one half-wave each
            const u64 pre = lookback2(look, look + ntiles, tile, tsum[0], tsum[1], p.err, lane);
            if ((lane & 31) == 0) s_tile_prefix[lane >> 5] = pre;
        } else {
            const u64 pre = lookback(look, tile, tsum[0], p.err, lane);
            if (lane == 0) s_tile_prefix[0] = pre;
        }
        mark(5);
        __syncthreads();  // B: tile prefix is in s_tile_prefix
        return;
    }

    DecWaveLds<NV>& S = lds_all[wave];
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

    mark(2);
    // ---------------- wave scan: column positions relative to this wave's range ----------------
    u64 agg[NV], excl[NV];
    u32 nch[NV];
    bool too_large = false;
    // field lengths are < 2^32 (Symphony's u32 length prefix): split 32-bit DPP scans
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u64 inc = wave_incl_scan_u32w_dpp((u32)flen[f]);
        agg[f] = (u64)uniform_i64((i64)__shfl((long long)inc, 63, 64));
        excl[f] = inc - flen[f];
        too_large |= agg[f] >= ((u64)1 << 31);  // positions inside a wave's range are 32-bit
        nch[f] = (u32)((flen[f] + 15) >> 4);     // copy chunks of this field
    }
    int T[NV];  // copy chunks per column
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u32 cinc = too_large ? 0u : wave_incl_scan_u32_dpp(nch[f]);
        T[f] = (int)__builtin_amdgcn_readlane(cinc, 63);
        S.dst[f][lane] = (int)excl[f];  // lanes >= cnt hold the aggregate
        S.cs[f][lane] = (int)(cinc - nch[f]);
        S.src[f][lane] = fsrc[f];
    }
    if (lane == 0) {
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            S.dst[f][kWaveRecs] = (int)agg[f];
            s_wagg[f][wave] = agg[f];
        }
    }
    S.mark[lane] = 0;
    wave_sync();

    // ---------------- copy: each field as its own run of 16-byte chunks ----------------
    // A field of L >= 16 bytes is ceil(L/16) chunks at field offsets 0, 16, ... with the last one
    // moved back to end at the field end (it rewrites bytes of the same field with the same
    // values); a shorter field is one chunk stored bytewise.  No chunk mixes two fields, so each
    // is one byte-unaligned load and one store, and all loads of a step fly together.
    // Step g = 64 consecutive chunks of one column: column 0's steps, then column 1's.
    int nsub[NV];
    int G = 0;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        nsub[f] = too_large || DIAG == 1 ? 0 : (T[f] + 63) >> 6;
        G += nsub[f];
    }
    // last 16-byte block holding stream bytes (readable: ABI rule, header "Memory rules")
    const uintptr_t in_last = (((uintptr_t)(p.in + p.rec_off[p.n]) + 15) & ~(uintptr_t)15) - 16;
    int myc[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) myc[f] = lane < cnt && nch[f] > 0 ? (int)(S.cs[f][lane]) : -1;

    // Chunk `lane` of step g: returns the data, its position P in the wave's column range
    // (-1: no chunk) and, packed in `nbs`, the valid byte count (16, or a short field's length)
    // plus a byte shift.  The load is unconditional and branch-free (lanes without a chunk read
    // a block inside the stream), so no wait is forced until the data is stored: a short field
    // at the very end of the stream is read from the stream's last 16 bytes and shifted later.
    auto load_step = [&](int g, int& P, int& nbs) -> u32x4 {
        const bool second = NV == 2 && g >= nsub[0];
        const int f = second ? 1 : 0;
        const int c0 = (second ? g - nsub[0] : g) * 64;
        const int mc = pick<NV>(myc, second);
        // record owning chunk c0+lane: forward fill of first-chunk marks (max-scan of k+1);
        // a step's first chunk always starts a field or continues the previous step's last one
        if (mc >= c0 && mc < c0 + 64) S.mark[mc - c0] = (u32)lane + 1u;
        wave_sync();
        const u32 m = wave_incl_max_u32_dpp(S.mark[lane]);
        S.mark[lane] = 0;
        const int c = c0 + lane;
        const bool has = c < pick<NV>(T, second);
        // m == 0 only when the step's first fields continue from the previous step: the owning
        // record then is the last one whose first chunk precedes c0
        const int k = m != 0 ? (int)m - 1 : (has ? lds_search_64(S.cs[f], cnt, c0) : 0);
        const int dk = S.dst[f][k], L = S.dst[f][k + 1] - dk;
        const int q = c - S.cs[f][k];
        const int off = L >= 16 ? min(16 * q, L - 16) : 0;
        const uintptr_t X = has ? (uintptr_t)(p.in + S.src[f][k]) + (uintptr_t)off : in_last;
        const uintptr_t Xc = X < in_last ? X : in_last;
        P = has ? dk + off : -1;
        nbs = min(L, 16) | (int)((X - Xc) << 5);
        return ld16u(Xc);
    };

    __syncthreads();  // A: wave aggregates published; the look-back wave runs while the loads fly
    mark(3);
    u32x4 buf[KRB];
    int bP[KRB], bN[KRB];
#pragma unroll
    for (int i = 0; i < KRB; ++i) {
        bP[i] = -1;
        bN[i] = 0;
        buf[i] = i < G ? load_step(i, bP[i], bN[i]) : u32x4{0, 0, 0, 0};
    }
    mark(4);
    __syncthreads();  // B: tile prefix ready
    mark(5);

    i64 pre[NV], lim[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        u64 t = s_tile_prefix[f];
        for (int w = 0; w < wave; ++w) t += s_wagg[f][w];
        pre[f] = uniform_i64((i64)t);
        const i64 cap = (i64)p.cap[f];
        if (lane == 0 && pre[f] + (i64)agg[f] > cap && agg[f] > 0) atomicOr(p.err, kErrCapacity);
        lim[f] = max((i64)0, min((i64)agg[f], cap - pre[f]));
    }
    if (lane < cnt) {
        const u64 r = r0 + lane;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            p.offs[f][r] = (u64)pre[f] + excl[f];
            if (r == p.n - 1) p.offs[f][p.n] = (u64)pre[f] + agg[f];
        }
    }
    if (too_large) {
        if (lane == 0) atomicOr(p.err, kErrTooLarge);
        return;
    }

    // 16-byte stores at any byte alignment; byte stores (behind a wave-uniform test) only for
    // short fields and capacity clips.
    auto store_step = [&](int g, u32x4 v, int P, int nbs) {
        const bool second = NV == 2 && g >= nsub[0];
        const int nb = nbs & 31;
        const u32 sh = (u32)nbs >> 5;
        if (__ballot(sh != 0)) {  // short field read from the stream's last block: shift down
            u32 w[4];
            funnel16(v, u32x4{0, 0, 0, 0}, sh, w);
            v = u32x4{w[0], w[1], w[2], w[3]};
        }
        const i64 hi = min((i64)(P + nb), pick<NV>(lim, second));
        uint8_t* base = (second ? p.bytes[NV - 1] : p.bytes[0]) + pick<NV>(pre, second);
        const bool full = P >= 0 && (i64)P + 16 <= hi;
        if (full) *(g_u4*)(base + P) = v;
        const bool part = P >= 0 && !full && (i64)P < hi;
        if (__ballot(part)) {
            const u32 rr[4] = {v.x, v.y, v.z, v.w};
            if (part) store_chunk(base, P, 0, hi, rr);
        }
    };
    // Rolling pipeline: slot i stores step g, then reloads with step g + KRB, so every wave keeps
    // KRB steps of loads in flight until its columns are done.
    for (int g0 = 0; g0 < G; g0 += KRB) {
#pragma unroll
        for (int i = 0; i < KRB; ++i) {
            const int g = g0 + i;
            if (g < G) {
                store_step(g, buf[i], bP[i], bN[i]);
                if (g + KRB < G) buf[i] = load_step(g + KRB, bP[i], bN[i]);
            }
        }
    }
    mark(6);
}

template <int NF, int NV>
static void launch_layout(const DecodeParams& p, dim3 grid, dim3 block, hipStream_t stream) {
    if (p.variant == 101)
        hipLaunchKernelGGL((decode_kernel<NF, NV, 1>), grid, block, 0, stream, p);
    else if (p.variant == 102)
        hipLaunchKernelGGL((decode_kernel<NF, NV, 2>), grid, block, 0, stream, p);
    else if (p.variant == 104 && p.dbg)
        hipLaunchKernelGGL((decode_kernel<NF, NV, 4>), grid, block, 0, stream, p);
    else if (p.variant == 105)
        hipLaunchKernelGGL((decode_kernel<NF, NV, 0, 5>), grid, block, 0, stream, p);
    else if (p.variant == 106)
        hipLaunchKernelGGL((decode_kernel<NF, NV, 0, 4>), grid, block, 0, stream, p);
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
    const dim3 block(kThreads);
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
