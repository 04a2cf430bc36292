// raw_fields.hip -- batched zero-copy field reads of Symphony records on gfx950.
//
// The generated XxxRaw getters (cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:984-1099,
// 1259-1294, 1517-1565) read one field of one buffer in place; aRPC's proxy elements call them on
// every buffered request (cmd/proxy/element/firewall.go:44-47: GetRequestRaw(payload).GetScore()).
// Here n buffers are handled per launch:
//  * fixed-width fields: one thread per record, the field's bytes read straight from the record
//    (at most two dword loads), one coalesced store of the column;
//  * string / bytes fields: a thread per record resolves (source offset, length) with the getter's
//    bounds checks and its tile's byte total; one small kernel scans the tile totals; the gather
//    kernel rescans its tile's lengths in registers (DPP / shuffles), writes the value offsets and
//    copies the values;
//  * the firewall element: score + verdict per record and per-tile (kept bytes, kept records)
//    totals, the same tile scan, and the gather kernel compacts the passing records into a
//    forwardable batch (offsets, input positions, bytes).
//
// The gather kernel is output-stationary like encode_kernel and the packetizer: a wave owns 64
// consecutive segments whose outputs are contiguous, lane = aligned 16-byte output chunk, each
// chunk assembled from byte-unaligned 16-byte loads of the (one or more) segments it covers and
// written with one global_store_dwordx4.  Per-record scan inputs never round-trip through HBM
// (only 16 bytes per 256-record tile do), which is what a device-wide library scan would cost.
#include "../../include/symphony_hip.h"
#include <algorithm>

#include "codec.hpp"
#include "device_util.hpp"
#include "gather_tile.hpp"

namespace symhip {

namespace raw {

// The private getters' complete-buffer assertion (main.go:1003-1013); sets off2p when it holds.
__device__ inline uint8_t private_check(uintptr_t m, u64 L, u64& off2p) {
    if (L < 5) return SYM_RAW_INVALID_BUFFER;
    const u64 o = ld_u32(m + 1);
    if (o >= L || ld_u8(m + o) != 0x01) return SYM_RAW_PUBLIC_ONLY;
    off2p = o;
    return SYM_RAW_OK;
}

// ---- fixed-width getters: `if len(m) < off+W { return 0 }; return LE(m[off:])` (main.go:1272-1293)
template <int W>
__global__ __launch_bounds__(256) void fixed_kernel(const uint8_t* in, const u64* rec_off, u64 n, int priv, u32 toff,
                                                    void* out, uint8_t* status) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const u64 s = rec_off[i], L = rec_off[i + 1] - s;
    const uintptr_t m = (uintptr_t)(in + s);
    uint8_t st = SYM_RAW_OK;
    u64 base = toff;
    if (priv) {
        u64 o = 0;
        st = private_check(m, L, o);
        base = o + toff;  // offsetToPrivate + tableOffset (main.go:1266-1269)
    }
    u64 v = 0;
    if (st == SYM_RAW_OK && L >= base + W) {
        if constexpr (W == 1) v = ld_u8(m + base);
        if constexpr (W == 4) v = ld_u32(m + base);
        if constexpr (W == 8) v = (u64)ld_u32(m + base) | ((u64)ld_u32(m + base + 4) << 32);
    }
    if constexpr (W == 1) ((uint8_t*)out)[i] = (uint8_t)v;
    if constexpr (W == 4) ((u32*)out)[i] = (u32)v;
    if constexpr (W == 8) ((u64*)out)[i] = v;
    if (status) status[i] = st;
}

// Tile total of a per-record (bytes, count) over the 256 threads of a workgroup -> agg[tile].
__device__ inline void tile_total(u64 b, u64 c, Pair* agg, u64* red_b, u64* red_c) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    b = wave_sum_u64(b);
    c = wave_sum_u64(c);
    if (lane == 0) {
        red_b[wave] = b;
        red_c[wave] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0)
        agg[blockIdx.x] = Pair{red_b[0] + red_b[1] + red_b[2] + red_b[3], red_c[0] + red_c[1] + red_c[2] + red_c[3]};
}

// ---- string / bytes getters: resolve each value's source and length (main.go:1527-1555)
__global__ __launch_bounds__(256) void var_locate_kernel(const uint8_t* in, const u64* rec_off, u64 n, int priv,
                                                         u32 toff, u64* seg_src, u64* seg_len, uint8_t* status,
                                                         Pair* agg) {
    __shared__ u64 red_b[4], red_c[4];
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    u64 len = 0;
    if (i < n) {
        const u64 s = rec_off[i], L = rec_off[i + 1] - s;
        const uintptr_t m = (uintptr_t)(in + s);
        uint8_t st = SYM_RAW_OK;
        u64 base = toff, o = 0;
        if (priv) {
            st = private_check(m, L, o);
            base = o + toff;
        }
        u64 src = s;
        if (st == SYM_RAW_OK && L >= base + 4) {
            u64 po = ld_u32(m + base);
            if (po != 0) {          // 0 = unset (:1537-1539)
                if (priv) po += o;  // relative -> absolute (:1542-1544)
                if (L >= po + 4) {
                    const u64 d = ld_u32(m + po);
                    if (L >= po + 4 + d) {
                        src = s + po + 4;
                        len = d;
                    }
                }
            }
        }
        seg_src[i] = src;
        seg_len[i] = len;
        if (status) status[i] = st;
    }
    tile_total(len, 0, agg, red_b, red_c);
}

// ---- firewall element: GetScore, shouldBlock, verdict (firewall.go:34-52)
__global__ __launch_bounds__(256) void firewall_mark_kernel(const uint8_t* in, const u64* rec_off, u64 n, u32 toff,
                                                            int32_t threshold, int32_t* score, uint8_t* verdict,
                                                            Pair* agg) {
    __shared__ u64 red_b[4], red_c[4];
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    u64 kb = 0, kc = 0;
    if (i < n) {
        const u64 s = rec_off[i], L = rec_off[i + 1] - s;
        const int32_t sc = L >= (u64)toff + 4 ? (int32_t)ld_u32((uintptr_t)(in + s) + toff) : 0;  // kv.syn.go:285-291
        const bool drop = sc >= threshold;
        if (score) score[i] = sc;
        verdict[i] = drop ? SYM_VERDICT_DROP : SYM_VERDICT_PASS;
        kb = drop ? 0 : L;
        kc = drop ? 0 : 1;
    }
    tile_total(kb, kc, agg, red_b, red_c);
}

// ---- exclusive scan of the tile totals (one workgroup; pre[ntiles] = grand total).  Each thread
// takes 4 consecutive tiles, so up to 4096 tiles (2^20 records) take one block-wide scan.
// nlim (optional): a device count of the scanned items; only its ceil(*nlim / 256) tiles are
// scanned (an item-capacity launch whose real count is known on the device only).
// rows > 1 (grid = rows): workgroup r scans row r, agg + r * agg_stride into pre + r * pre_stride.
__global__ __launch_bounds__(1024) void tile_scan_kernel(const Pair* agg, Pair* pre, u64 ntiles,
                                                        const unsigned* gate = nullptr, const u64* nlim = nullptr,
                                                        u64 agg_stride = 0, u64 pre_stride = 0) {
    if (gate && *gate == 0) return;  // a gated launch (reassembly's general path) with nothing to do
    agg += blockIdx.x * agg_stride;
    pre += blockIdx.x * pre_stride;
    if (nlim) ntiles = min(ntiles, (*nlim + 255) / 256);
    constexpr int kPer = 4;
    __shared__ u64 wb[16], wc[16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 carry_b = 0, carry_c = 0;
    for (u64 base = 0; base < ntiles; base += 1024 * kPer) {  // uniform loop
        const u64 t0 = base + (u64)threadIdx.x * kPer;
        Pair v[kPer];
        u64 sb = 0, sc = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            v[k] = t0 + k < ntiles ? agg[t0 + k] : Pair{0, 0};
            sb += v[k].bytes;
            sc += v[k].count;
        }
        const u64 ib = wave_incl_scan_u64(sb, lane), ic = wave_incl_scan_u64(sc, lane);
        if (lane == 63) {
            wb[wave] = ib;
            wc[wave] = ic;
        }
        __syncthreads();
        u64 pb = carry_b + ib - sb, pc = carry_c + ic - sc, tb = 0, tc = 0;
        for (int q = 0; q < 16; ++q) {
            if (q < wave) {
                pb += wb[q];
                pc += wc[q];
            }
            tb += wb[q];
            tc += wc[q];
        }
        __syncthreads();  // wb / wc are rewritten by the next round
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            if (t0 + k < ntiles) pre[t0 + k] = Pair{pb, pc};
            pb += v[k].bytes;
            pc += v[k].count;
        }
        carry_b += tb;
        carry_c += tc;
    }
    if (threadIdx.x == 0) pre[ntiles] = Pair{carry_b, carry_c};
}

// Grid-stride over the tiles of the segment count (*n_ptr when given, else n): a launch sized for a
// capacity far above the real count (nested item lists) does not dispatch a workgroup per empty tile.
template <bool FW, int KU = 4, bool NT = false>
__global__ __launch_bounds__(kWaves * 64) void gather_kernel(GatherArgs a) {
    __shared__ WaveLds lds_all[kWaves];
    __shared__ MaskTable masks;
    __shared__ u64 wsum_b[kWaves], wsum_c[kWaves];
    const u64 n = a.n_ptr ? *a.n_ptr : a.n;  // segments
    const u64 ntiles = (n + 255) / 256;
    if (n == 0) return;  // nothing to place (and the scan of an empty count may not have run)
    mask_table_init(masks, threadIdx.x);
    for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {  // workgroup-uniform loop
        gather_tile<FW, KU, NT>(a, t, n, ntiles, lds_all, masks, wsum_b, wsum_c);
        __syncthreads();  // wsum_* and the wave slots are rewritten by the next tile
    }
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
inline u64 tiles_of(u64 n) { return (n + 255) / 256; }

}  // namespace raw

hipError_t launch_raw_fixed(const uint8_t* in, const u64* rec_off, u64 n, int priv, u32 table_off, u32 width,
                            void* out, uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    switch (width) {
        case 1: hipLaunchKernelGGL(raw::fixed_kernel<1>, grid, block, 0, stream, in, rec_off, n, priv, table_off, out, status); break;
        case 4: hipLaunchKernelGGL(raw::fixed_kernel<4>, grid, block, 0, stream, in, rec_off, n, priv, table_off, out, status); break;
        case 8: hipLaunchKernelGGL(raw::fixed_kernel<8>, grid, block, 0, stream, in, rec_off, n, priv, table_off, out, status); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// workspace: [tile totals (ntiles) | tile prefixes (ntiles+1) | VAR: value sources (n) | lengths (n)]
static size_t tile_ws(u64 n) { return 2 * raw::al256((raw::tiles_of(n) + 1) * sizeof(raw::Pair)); }

size_t raw_bytes_ws_bytes(u64 n) { return tile_ws(n) + 2 * raw::al256(n * sizeof(u64)); }

size_t firewall_ws_bytes(u64 n) { return tile_ws(n); }

hipError_t launch_tile_scan(const raw::Pair* agg, raw::Pair* pre, u64 ntiles, hipStream_t stream) {
    hipLaunchKernelGGL(raw::tile_scan_kernel, dim3(1), dim3(1024), 0, stream, agg, pre, ntiles, nullptr);
    return hipGetLastError();
}

hipError_t launch_tile_scan_gated(const raw::Pair* agg, raw::Pair* pre, u64 ntiles, const unsigned* gate,
                                  hipStream_t stream) {
    hipLaunchKernelGGL(raw::tile_scan_kernel, dim3(1), dim3(1024), 0, stream, agg, pre, ntiles, gate);
    return hipGetLastError();
}

hipError_t launch_segment_gather(const raw::GatherArgs& a, hipStream_t stream) {
    // a workgroup per tile of the capacity, up to 16384 (a 2^22-segment batch); past that (item
    // capacities of nested lists, far above their real counts) the workgroups stride over the tiles
    const dim3 grid((unsigned)std::min<u64>(raw::tiles_of(a.n), 16384));
    // segments of ~640 bytes (config-3 datagram payloads) ran faster with 2 chunks per lane per step
    // (more waves per SIMD: reassembly config 3 0.718 -> 0.689 ms); ~350-byte ones with 4 (config 2
    // 0.302 vs 0.313 ms, flat decode 0.339 vs 0.349 ms; r04h, SYMHIP_GATHER_VARIANT 1 / 2 below)
    int ku = a.seg_bytes_hint >= 512 ? 2 : 4;
#ifdef SYMHIP_TUNING
    if (const int v = tuning_variant("SYMHIP_GATHER_VARIANT")) ku = v == 1 ? 2 : v == 2 ? 8 : 4;
#endif
    if (ku == 2 && a.nt) hipLaunchKernelGGL((raw::gather_kernel<false, 2, true>), grid, dim3(256), 0, stream, a);
    else if (ku == 2) hipLaunchKernelGGL((raw::gather_kernel<false, 2>), grid, dim3(256), 0, stream, a);
#ifdef SYMHIP_TUNING
    else if (ku == 8) hipLaunchKernelGGL((raw::gather_kernel<false, 8>), grid, dim3(256), 0, stream, a);
#endif
    else if (a.nt) hipLaunchKernelGGL((raw::gather_kernel<false, 4, true>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL(raw::gather_kernel<false>, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_tile_scan_limited(const raw::Pair* agg, raw::Pair* pre, u64 ntiles, const u64* nlim, hipStream_t stream) {
    hipLaunchKernelGGL(raw::tile_scan_kernel, dim3(1), dim3(1024), 0, stream, agg, pre, ntiles, nullptr, nlim);
    return hipGetLastError();
}

hipError_t launch_tile_scan_rows(const raw::Pair* agg, u64 agg_stride, raw::Pair* pre, u64 pre_stride, u64 ntiles,
                                 int rows, const u64* nlim, hipStream_t stream) {
    hipLaunchKernelGGL(raw::tile_scan_kernel, dim3((unsigned)rows), dim3(1024), 0, stream, agg, pre, ntiles, nullptr,
                       nlim, agg_stride, pre_stride);
    return hipGetLastError();
}

static hipError_t scan_and_gather(raw::GatherArgs& a, bool fw, raw::Pair* agg, raw::Pair* pre, hipStream_t stream) {
    const u64 nt = raw::tiles_of(a.n);
    hipLaunchKernelGGL(raw::tile_scan_kernel, dim3(1), dim3(1024), 0, stream, agg, pre, nt, nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    a.pre = pre;
    if (fw) hipLaunchKernelGGL((raw::gather_kernel<true, 4, true>), dim3((unsigned)nt), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((raw::gather_kernel<false, 4, true>), dim3((unsigned)nt), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_raw_bytes(const uint8_t* in, const u64* rec_off, u64 n, int priv, u32 table_off, uint8_t* out,
                            u64 cap, u64* out_off, uint8_t* status, void* ws, unsigned* err, hipStream_t stream) {
    if (n == 0) return hipMemsetAsync(out_off, 0, sizeof(u64), stream);
    const size_t pc = raw::al256((raw::tiles_of(n) + 1) * sizeof(raw::Pair));
    raw::Pair* agg = (raw::Pair*)ws;
    raw::Pair* pre = (raw::Pair*)((char*)ws + pc);
    u64* seg_src = (u64*)((char*)ws + 2 * pc);
    u64* seg_len = (u64*)((char*)ws + 2 * pc + raw::al256(n * sizeof(u64)));
    hipLaunchKernelGGL(raw::var_locate_kernel, dim3((unsigned)raw::tiles_of(n)), dim3(256), 0, stream, in, rec_off, n,
                       priv, table_off, seg_src, seg_len, status, agg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    raw::GatherArgs a{};
    a.in = in;
    a.rec_off = rec_off;
    a.n = n;
    a.lo_ptr = rec_off;
    a.hi_ptr = rec_off + n;
    a.seg_src = seg_src;
    a.seg_len = seg_len;
    a.out = out;
    a.cap = cap;
    a.out_off = out_off;
    a.err = err;
    return scan_and_gather(a, false, agg, pre, stream);
}

hipError_t launch_firewall(const uint8_t* in, const u64* rec_off, u64 n, u32 score_table_off, int32_t threshold,
                           int32_t* score, uint8_t* verdict, uint8_t* kept, u64 cap, u64* kept_off, u64* kept_index,
                           u64* nkept, void* ws, unsigned* err, hipStream_t stream) {
    const size_t pc = raw::al256((raw::tiles_of(n) + 1) * sizeof(raw::Pair));
    raw::Pair* agg = (raw::Pair*)ws;
    raw::Pair* pre = (raw::Pair*)((char*)ws + pc);
    hipLaunchKernelGGL(raw::firewall_mark_kernel, dim3((unsigned)raw::tiles_of(n)), dim3(256), 0, stream, in, rec_off,
                       n, score_table_off, threshold, score, verdict, agg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    raw::GatherArgs a{};
    a.in = in;
    a.rec_off = rec_off;
    a.n = n;
    a.lo_ptr = rec_off;
    a.hi_ptr = rec_off + n;
    a.verdict = verdict;
    a.out = kept;
    a.cap = cap;
    a.out_off = kept_off;
    a.kept_index = kept_index;
    a.nkept = nkept;
    a.err = err;
    return scan_and_gather(a, true, agg, pre, stream);
}

}  // namespace symhip
