// decode.hip -- batched Symphony UnmarshalSymphony for flat schemas on gfx950: the three-kernel
// path (decode variant 300).  The default decode is decode_pipe.hip; this file also holds the
// decode dispatch (launch_decode).
//
// Restates, for n records at once, the generated per-record unmarshaller into a fresh
// struct: benchmark/kv-store-symphony/symphony/kv.syn.go:680-745 (SetRequest; Get/Resp
// analogous), examples/echo_symphony/symphony/echo.syn.go:186-263 (int32 fields), from the
// generator's rules cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:622-694, :734-793.
//
// A string field's output position is the sum of all earlier lengths in its column, so decode
// is a scan.  It runs as three stream-ordered kernels with no inter-workgroup waiting:
//  1. parse (lane = record, 2 records per lane): the record's first 32 (48 with int32 fields)
//     bytes land in LDS with byte-unaligned 16-byte loads; Go's header checks and, per field,
//     the table-entry / length-prefix bounds checks (64-bit arithmetic, as Go's int) read
//     from there, or from global memory past the window.  Writes the status byte and int32 fields,
//     each string field's (length, offset in the record) to the workspace, and each tile's
//     per-column aggregate (one DPP wave scan).
//  2. scan: one workgroup per column turns tile aggregates into tile prefixes (and the final
//     offsets[n]).
//  3. copy (wave = 64-record tile): re-scans the tile's lengths, writes the output offsets,
//     and copies every field as a run of 16-byte chunks (the last one moved back to end at
//     the field end), so each chunk is one byte-unaligned 16-byte load and one 16-byte store.
//     Chunks are enumerated record-major (a record's key chunks, then its value chunks), so
//     the lines a record spans are fetched together; each wave keeps kRB steps (64 chunks
//     each) of loads in flight in a rolling register pipeline.
// No wave ever waits on another; the price is a second read of every record's header sectors
// (the parse pass) before any byte moves, which the pipelined default overlaps with the copy.
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

constexpr int kWaveRecs = 64;  // records per tile (one wave)
constexpr int kWaves = 4;      // tiles per workgroup (parse, copy)
constexpr int kThreads = 64 * kWaves;
constexpr int kRB = 4;         // copy steps (64 chunks each) in flight per wave
constexpr int kScanThreads = 1024;

// Workspace (per call, every slot written before it is read):
//   agg[nvar][tiles] u64 tile aggregates, pre[nvar][tiles] u64 tile prefixes,
//   flen[nvar][n] u32 field length, fpos[nvar][n] u32 field offset in its record (past the
//   length prefix).
struct DecodeWs {
    uint32_t* flen;
    uint32_t* fpos;
    u64* agg;
    u64* pre;
};
__host__ __device__ static inline uint64_t num_tiles(uint64_t n) { return (n + kWaveRecs - 1) / kWaveRecs; }
static DecodeWs ws_layout(void* ws, int nvar, uint64_t n) {
    const uint64_t t = num_tiles(n);
    DecodeWs w;
    w.agg = (u64*)ws;
    w.pre = w.agg + (size_t)nvar * t;
    w.flen = (uint32_t*)(w.pre + (size_t)nvar * t);
    w.fpos = w.flen + (size_t)nvar * n;
    return w;
}
size_t decode_workspace_bytes(int nvar, uint64_t n) {
    const size_t bytes = (size_t)nvar * (16 * num_tiles(n) + 8 * n);
    return (bytes + 255) & ~(size_t)255;
}

// ------------------------------------------------------------------ 1. parse
// Mixed kv batches (MIX, p.type != null): a record of type 0 is a GetRequest (one string field,
// kv.syn.go:134-185), any other a SetRequest (two, :680-745).
// Each lane parses kParseRecs records (tile t's record `lane` for the wave's kParseRecs tiles),
// in phases so that every record's loads of one kind are in flight together: offsets, then the
// header windows, then the length prefixes that lie past the window.
constexpr int kParseRecs = 2;
template <int NF>
constexpr int parse_win() { return NF > 0 ? 48 : 32; }  // table + first length prefix fit

template <int NF, int NV, bool MIX>
__global__ __launch_bounds__(kThreads) void decode_parse_kernel(DecodeParams p, DecodeWs w, u64 tb, u64 te) {
    constexpr int kW = parse_win<NF>();
    constexpr int R = kParseRecs;
    __shared__ uint8_t win_all[kWaves][R][kWaveRecs * kW];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 ntiles = num_tiles(p.n);
    const u64 tile0 = tb + ((u64)blockIdx.x * kWaves + wave) * R;
    if (tile0 >= te) return;

    // Loads are unconditional (exec-masked loads would make the compiler drain every load before
    // the next dependent use); lanes with nothing to read use `safe`, the workspace's first
    // 256 bytes (always allocated; the data read there is never used).
    const uintptr_t safe = (uintptr_t)w.agg;
    u64 start[R], len[R];
    bool live[R], win[R];
    u64 endv[R];
    int nvr[R];
#pragma unroll
    for (int h = 0; h < R; ++h) {
        const u64 r = (tile0 + h) * kWaveRecs + lane;
        live[h] = r < p.n && tile0 + h < te;
        const u64 rc = live[h] ? r : p.n;  // branch-free loads: rec_off has n+1 entries
        start[h] = p.rec_off[rc];
        endv[h] = p.rec_off[live[h] ? rc + 1 : rc];
        nvr[h] = MIX ? (p.type[live[h] ? r : 0] != 0 ? NV : 1) : NV;
    }
    __builtin_amdgcn_sched_barrier(0);  // issue every record's offset loads before using any
#pragma unroll
    for (int h = 0; h < R; ++h) {
        len[h] = endv[h] - start[h];
        win[h] = live[h] && len[h] >= (u64)kW;  // window loads stay inside the record
    }
    {
        u32x4 wv[R][kW / 16];
#pragma unroll
        for (int h = 0; h < R; ++h)
#pragma unroll
            for (int k = 0; k < kW / 16; ++k)
                wv[h][k] = ld16u((win[h] ? (uintptr_t)(p.in + start[h]) : safe) + 16 * k);
#pragma unroll
        for (int h = 0; h < R; ++h)
#pragma unroll
            for (int k = 0; k < kW / 16; ++k) *(u32x4*)&win_all[wave][h][lane * kW + 16 * k] = wv[h][k];
    }
    wave_sync();

    // header checks and table entries (window reads; global only for adversarial offsets)
    u32 st[R];
    int32_t fx[R][NF > 0 ? NF : 1];
    u64 po[R][NV];
#pragma unroll
    for (int h = 0; h < R; ++h) {
        const uintptr_t d = (uintptr_t)(p.in + start[h]);
        const uint8_t* wb = &win_all[wave][h][lane * kW];
        const bool wh = win[h];
        const u64 L = len[h];
        auto rd8 = [&](u64 q) -> u32 { return (wh && q < (u64)kW) ? (u32)wb[q] : ld_u8(d + q); };
        auto rd32 = [&](u64 q) -> u32 {
            return (wh && q + 4 <= (u64)kW) ? *(const u32*)(wb + q) : *(gc_u32*)(d + q);  // unaligned OK
        };
        st[h] = 0;
#pragma unroll
        for (int f = 0; f < (NF > 0 ? NF : 1); ++f) fx[h][f] = 0;
#pragma unroll
        for (int f = 0; f < NV; ++f) po[h][f] = 0;
        if (!live[h]) continue;
        if (L < 13) {
            st[h] = 1;  // "invalid data: too short"
        } else if (rd8(0) != 0x01) {
            st[h] = 2;  // "invalid data: wrong public version"
        } else {
            const u64 off2p = rd32(1);
            if (off2p >= L || rd8(off2p) != 0x01) {
                st[h] = 3;  // "missing private segment"
            } else {
                const u64 pts = off2p + 1;
                u64 toff = 0;
#pragma unroll
                for (int f = 0; f < NF; ++f, toff += 4) {
                    if (st[h] == 0) {
                        if (L < pts + toff + 4) st[h] = 4;  // "invalid data: too short for field"
                        else fx[h][f] = (int32_t)rd32(pts + toff);
                    }
                }
                if (st[h] == 0) {
#pragma unroll
                    for (int f = 0; f < NV; ++f, toff += 4) {
                        if (f < nvr[h] && L >= pts + toff + 4) {
                            u64 q = rd32(pts + toff);
                            if (q > 0) q += off2p;
                            if (q > 0 && L >= q + 4) po[h][f] = q;  // length prefix at q
                        }
                    }
                }
            }
        }
    }
    // length prefixes: from the window, else one global load each, all issued together
    u32 nbg[R][NV], nbw[R][NV];
#pragma unroll
    for (int h = 0; h < R; ++h)
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 q = po[h][f];
            const bool inwin = win[h] && q + 4 <= (u64)kW;
            nbg[h][f] = *(gc_u32*)(q > 0 && !inwin ? (uintptr_t)(p.in + start[h] + q) : safe);  // unaligned OK
            nbw[h][f] = inwin ? *(const u32*)&win_all[wave][h][lane * kW + (inwin ? q : 0)] : 0u;
        }
    bool too_large = false;
#pragma unroll
    for (int h = 0; h < R; ++h) {
        const u64 r = (tile0 + h) * kWaveRecs + lane;
        u64 flen[NV], fpos[NV];
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 q = po[h][f];
            const u64 nb = win[h] && q + 4 <= (u64)kW ? nbw[h][f] : nbg[h][f];
            const bool ok = q > 0 && len[h] >= q + 4 + nb;
            flen[f] = ok ? nb : 0;
            fpos[f] = ok ? q + 4 : 0;
        }
        if (live[h]) {
            p.status[r] = (uint8_t)st[h];
#pragma unroll
            for (int f = 0; f < NF; ++f) p.fixed[f][r] = fx[h][f];
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                too_large |= fpos[f] >= ((u64)1 << 32);  // field offset inside a >= 4 GiB record
                w.flen[(size_t)f * p.n + r] = (uint32_t)flen[f];
                w.fpos[(size_t)f * p.n + r] = (uint32_t)fpos[f];
            }
        }
        // tile aggregates (field lengths are < 2^32: split 32-bit DPP scans)
        if (tile0 + h < te) {
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                const u64 inc = wave_incl_scan_u32w_dpp((u32)flen[f]);
                if (lane == 63) {
                    w.agg[(size_t)f * ntiles + tile0 + h] = inc;
                    too_large |= inc >= ((u64)1 << 31);  // positions inside a tile's range are 32-bit
                }
            }
        }
    }
    if (__ballot(too_large) && lane == 0) atomicOr(p.err, kErrTooLarge);
}

// ------------------------------------------------------------------ 2. scan
// One workgroup per column: exclusive scan of the tile aggregates (each < 2^31, checked by the
// parse kernel).  Wave w owns 1024 consecutive tiles of a block, lane-interleaved (element
// k*64 + lane), so every load and store instruction is one coalesced 512-byte access; rows are
// scanned with DPP and carried across k, waves combine through LDS.
__global__ __launch_bounds__(kScanThreads) void decode_scan_kernel(DecodeParams p, DecodeWs w, u64 tb, u64 te) {
    constexpr int kRows = 16;
    constexpr int kWavesScan = kScanThreads / 64;
    constexpr u64 kBlock = (u64)kScanThreads * kRows;
    __shared__ u64 s_wsum[kWavesScan];
    const int f = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 ntiles = num_tiles(p.n);
    const u64* agg = w.agg + (size_t)f * ntiles;
    u64* pre = w.pre + (size_t)f * ntiles;
    u64 carry = 0;  // total of all earlier blocks (uniform)
    for (u64 base = tb; base < te; base += kBlock) {
        const u64 e0 = base + (u64)wave * (64 * kRows) + lane;
        u32 v[kRows];
#pragma unroll
        for (int k = 0; k < kRows; ++k)  // unconditional (clamped) loads: all rows in flight at once
            v[k] = (u32)agg[min(e0 + 64 * k, te - 1)];
        u64 run = 0, ex[kRows];
#pragma unroll
        for (int k = 0; k < kRows; ++k) {
            if (e0 + 64 * k >= te) v[k] = 0;
            const u64 inc = wave_incl_scan_u32w_dpp(v[k]);
            ex[k] = run + inc - v[k];
            run += (u64)(u32)__builtin_amdgcn_readlane((u32)inc, 63) | ((u64)(u32)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
        }
        if (lane == 0) s_wsum[wave] = run;
        __syncthreads();
        u64 wpre = carry, tot = 0;
#pragma unroll
        for (int q = 0; q < kWavesScan; ++q) {
            const u64 t = s_wsum[q];
            if (q < wave) wpre += t;
            tot += t;
        }
#pragma unroll
        for (int k = 0; k < kRows; ++k)
            if (e0 + 64 * k < te) pre[e0 + 64 * k] = wpre + ex[k];
        carry += tot;
        __syncthreads();  // s_wsum is rewritten by the next block
    }
    if (threadIdx.x == 0 && te == ntiles) p.offs[f][p.n] = carry;
}

// ------------------------------------------------------------------ 3. copy
template <int NV>
struct alignas(16) CopyWaveLds {
    u64 src[NV][kWaveRecs];      // field position in the input stream
    int dst[NV][kWaveRecs + 1];  // field start in the tile's column range; [cnt..] = aggregate
    int cs[kWaveRecs + 1];       // record's first copy chunk (record-major chunk sequence)
    int nch0[kWaveRecs];         // chunks of the record's first string field
    u32 mark[64];                // record index + 1 at its first chunk, per copy step
};

template <int NV, typename T>
__device__ __forceinline__ T pick(const T (&a)[NV], bool second) {
    if constexpr (NV == 1) return a[0];
    else return second ? a[1] : a[0];
}

template <int NV, int KRB = kRB>
__global__ __launch_bounds__(kThreads) void decode_copy_kernel(DecodeParams p, DecodeWs w, u64 tb, u64 te) {
    static_assert(NV == 1 || NV == 2, "decode handles one or two string columns");
    __shared__ CopyWaveLds<NV> lds_all[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 tile = tb + (u64)blockIdx.x * kWaves + wave;
    const u64 ntiles = num_tiles(p.n);
    if (tile >= te) return;
    CopyWaveLds<NV>& S = lds_all[wave];
    const u64 r0 = tile * kWaveRecs;
    const int cnt = (int)min((u64)kWaveRecs, p.n - r0);

    u32 flen[NV];
    i64 pre[NV];
    u64 start = 0;
    if (lane < cnt) start = p.rec_off[r0 + lane];
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        flen[f] = lane < cnt ? w.flen[(size_t)f * p.n + r0 + lane] : 0u;
        S.src[f][lane] = start + (lane < cnt ? w.fpos[(size_t)f * p.n + r0 + lane] : 0u);
        pre[f] = uniform_i64((i64)w.pre[(size_t)f * ntiles + tile]);
    }
    // tile scan: column positions relative to the tile, and the output offsets
    u64 agg[NV];
    u32 nch[NV];
    bool too_large = false;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u64 inc = wave_incl_scan_u32w_dpp(flen[f]);
        agg[f] = (u64)uniform_i64((i64)__shfl((long long)inc, 63, 64));
        const u64 excl = inc - flen[f];
        too_large |= agg[f] >= ((u64)1 << 31);
        if (lane < cnt) p.offs[f][r0 + lane] = (u64)pre[f] + excl;
        S.dst[f][lane] = (int)excl;  // lanes >= cnt hold the aggregate
        nch[f] = (flen[f] + 15) >> 4;
    }
    if (too_large) return;  // reported by the parse kernel (kErrTooLarge)
    const u32 nrec = nch[0] + (NV == 2 ? nch[NV - 1] : 0u);
    const u32 cinc = wave_incl_scan_u32_dpp(nrec);
    const int T = (int)__builtin_amdgcn_readlane(cinc, 63);  // chunks in this tile
    S.cs[lane] = (int)(cinc - nrec);
    S.nch0[lane] = (int)nch[0];
    S.mark[lane] = 0;
    if (lane == 0) {
#pragma unroll
        for (int f = 0; f < NV; ++f) S.dst[f][kWaveRecs] = (int)agg[f];
        S.cs[kWaveRecs] = T;
    }
    i64 lim[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const i64 cap = (i64)p.cap[f];
        if (lane == 0 && agg[f] > 0 && pre[f] + (i64)agg[f] > cap) atomicOr(p.err, kErrCapacity);
        lim[f] = max((i64)0, min((i64)agg[f], cap - pre[f]));
    }
    wave_sync();

    // last 16-byte block holding stream bytes (readable: ABI rule, header "Memory rules")
    const uintptr_t in_last = (((uintptr_t)(p.in + p.rec_off[p.n]) + 15) & ~(uintptr_t)15) - 16;
    const int myc = lane < cnt && nrec > 0 ? (int)(cinc - nrec) : -1;
    const int G = (T + 63) >> 6;  // copy steps

    // Chunk c0+lane of the record-major sequence: returns the data; P = its position in its
    // column's tile range (-1: none); `code` packs the valid byte count (16, or a short field's
    // length), the byte shift of a short field read from the stream's last block, and the
    // column.  The load is unconditional and branch-free, so nothing waits until the store.
    auto load_step = [&](int g, int& P, int& code) -> u32x4 {
        const int c0 = g * 64;
        // owning record: forward fill of first-chunk marks (max-scan of k+1); lanes before the
        // step's first mark continue the last record whose first chunk precedes c0
        if (myc >= c0 && myc < c0 + 64) S.mark[myc - c0] = (u32)lane + 1u;
        wave_sync();
        const u32 m = wave_incl_max_u32_dpp(S.mark[lane]);
        S.mark[lane] = 0;
        const int c = c0 + lane;
        const bool has = c < T;
        const int k = m != 0 ? (int)m - 1 : (has ? lds_search_64(S.cs, cnt, c0) : 0);
        int q = c - S.cs[k];
        const bool second = NV == 2 && q >= S.nch0[k];
        if (second) q -= S.nch0[k];
        const int f = second ? 1 : 0;
        const int dk = S.dst[f][k], L = S.dst[f][k + 1] - dk;
        const int off = L >= 16 ? min(16 * q, L - 16) : 0;
        const uintptr_t X = has ? (uintptr_t)(p.in + S.src[f][k]) + (uintptr_t)off : in_last;
        const uintptr_t Xc = X < in_last ? X : in_last;
        P = has ? dk + off : -1;
        code = min(L, 16) | (int)((X - Xc) << 5) | (second ? 1 << 10 : 0);
        return ld16u(Xc);
    };
    // 16-byte stores at any byte alignment; byte stores (behind a wave-uniform test) only for
    // short fields and capacity clips.
    auto store_step = [&](u32x4 v, int P, int code) {
        const bool second = (code >> 10) & 1;
        const int nb = code & 31;
        const u32 sh = ((u32)code >> 5) & 31u;
        if (__ballot(sh != 0)) {  // short field read from the stream's last block: shift down
            u32 t[4];
            funnel16(v, u32x4{0, 0, 0, 0}, sh, t);
            v = u32x4{t[0], t[1], t[2], t[3]};
        }
        const i64 hi = min((i64)(P + nb), pick<NV>(lim, second));
        uint8_t* base = (second ? p.bytes[NV - 1] : p.bytes[0]) + pick<NV>(pre, second);
        const bool full = P >= 0 && (i64)P + 16 <= hi;
        if (full) st16(base + P, v, true);  // (nontemporal: measured on, DESIGN.md section 4 Stores)
        const bool part = P >= 0 && !full && (i64)P < hi;
        if (__ballot(part)) {
            const u32 rr[4] = {v.x, v.y, v.z, v.w};
            if (part) store_chunk(base, P, 0, hi, rr, true);
        }
    };

    u32x4 buf[KRB];
    int bP[KRB], bC[KRB];
#pragma unroll
    for (int i = 0; i < KRB; ++i) {
        bP[i] = -1;
        bC[i] = 0;
        buf[i] = i < G ? load_step(i, bP[i], bC[i]) : u32x4{0, 0, 0, 0};
    }
    // rolling pipeline: slot i stores step g, then reloads with step g + KRB
    for (int g0 = 0; g0 < G; g0 += KRB) {
#pragma unroll
        for (int i = 0; i < KRB; ++i) {
            const int g = g0 + i;
            if (g < G) {
                store_step(buf[i], bP[i], bC[i]);
                if (g + KRB < G) buf[i] = load_step(g + KRB, bP[i], bC[i]);
            }
        }
    }
}

// ------------------------------------------------------------------ launch
template <int NF, int NV, bool MIX>
static hipError_t launch_layout(const DecodeParams& p, const DecodeWs& w, hipStream_t stream) {
    const u64 ntiles = num_tiles(p.n);
    constexpr u64 kGroup = kWaves * kParseRecs;  // tiles per parse workgroup
    const unsigned pg = (unsigned)((ntiles + kGroup - 1) / kGroup);
    const unsigned cg = (unsigned)((ntiles + kWaves - 1) / kWaves);
    hipLaunchKernelGGL((decode_parse_kernel<NF, NV, MIX>), dim3(pg), dim3(kThreads), 0, stream, p, w, (u64)0, ntiles);
    hipLaunchKernelGGL(decode_scan_kernel, dim3(NV), dim3(kScanThreads), 0, stream, p, w, (u64)0, ntiles);
#ifdef SYMHIP_TUNING
    if (p.variant == 301) return hipGetLastError();  // timing of parse + scan alone
#endif
    hipLaunchKernelGGL((decode_copy_kernel<NV>), dim3(cg), dim3(kThreads), 0, stream, p, w, (u64)0, ntiles);
    return hipGetLastError();
}

// Decode dispatch by the ctx's implementation (sym_ctx_set_decode_impl): the single-launch pipeline
// (decode_pipe.hip) by default, or its forced look-back mode; kImplThreeKernel runs the path above
// (parse -> scan -> copy), kept as a second, independently tested implementation of the contract.
hipError_t launch_decode(const DecodeParams& p, hipStream_t stream) {
    if (p.n == 0) {
        for (int f = 0; f < p.lay.nvar; ++f) {
            hipError_t e = hipMemsetAsync(p.offs[f], 0, sizeof(uint64_t), stream);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    bool three = p.impl == kImplThreeKernel;
#ifdef SYMHIP_TUNING
    three = three || p.variant == 300 || p.variant == 301;
#endif
    if (!three) return launch_decode_pipe(p, p.flags, p.epoch, stream);
    const DecodeWs w = ws_layout(p.ws, p.lay.nvar, p.n);
    if (p.type) return p.lay.nfixed == 0 && p.lay.nvar == 2 ? launch_layout<0, 2, true>(p, w, stream) : hipErrorInvalidValue;
    if (p.lay.nfixed == 0 && p.lay.nvar == 1) return launch_layout<0, 1, false>(p, w, stream);
    if (p.lay.nfixed == 0 && p.lay.nvar == 2) return launch_layout<0, 2, false>(p, w, stream);
    if (p.lay.nfixed == 2 && p.lay.nvar == 2) return launch_layout<2, 2, false>(p, w, stream);
    return hipErrorInvalidValue;
}

}  // namespace symhip
