// raw_fields.hip -- batched zero-copy field reads of Symphony records on gfx950.
//
// The generated XxxRaw getters (cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:984-1099,
// 1259-1294, 1517-1565) read one field of one buffer in place; aRPC's proxy elements call them on
// every buffered request (cmd/proxy/element/firewall.go:44-47: GetRequestRaw(payload).GetScore()).
// Here n buffers are handled per launch:
//  * fixed-width fields: one thread per record, the field's bytes read straight from the record
//    (at most two dword loads), one coalesced store of the column;
//  * string / bytes fields: a thread per record resolves (source offset, length) with the getter's
//    bounds checks, a device-wide exclusive scan (rocPRIM) places the values, and a gather kernel
//    copies them out;
//  * the firewall element: score + verdict per record, one scan over (kept bytes, kept count)
//    pairs, and the same gather kernel compacts the passing records into a forwardable batch.
//
// The gather kernel is output-stationary like encode_kernel and the packetizer: a wave owns 64
// consecutive segments whose outputs are contiguous, lane = aligned 16-byte output chunk, each
// chunk assembled from byte-unaligned 16-byte loads of the (one or more) segments it covers and
// written with one global_store_dwordx4.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses memset

#include <rocprim/device/device_scan.hpp>

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

namespace raw {

constexpr int kSegs = 64;  // segments per wave tile
constexpr int kWaves = 4;

struct Pair {  // firewall scan element: kept bytes, kept records
    u64 bytes, count;
};
struct PairPlus {
    __host__ __device__ Pair operator()(const Pair& a, const Pair& b) const {
        return Pair{a.bytes + b.bytes, a.count + b.count};
    }
};

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

// ---- string / bytes getters: resolve each value's source and length (main.go:1527-1555)
__global__ __launch_bounds__(256) void var_locate_kernel(const uint8_t* in, const u64* rec_off, u64 n, int priv,
                                                         u32 toff, u64* seg_src, u64* seg_len, uint8_t* status) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i > n) return;
    if (i == n) {  // n+1 scan inputs: the last exclusive prefix is the total
        seg_len[n] = 0;
        return;
    }
    const u64 s = rec_off[i], L = rec_off[i + 1] - s;
    const uintptr_t m = (uintptr_t)(in + s);
    uint8_t st = SYM_RAW_OK;
    u64 base = toff, o = 0;
    if (priv) {
        st = private_check(m, L, o);
        base = o + toff;
    }
    u64 src = s, len = 0;
    if (st == SYM_RAW_OK && L >= base + 4) {
        u64 po = ld_u32(m + base);
        if (po != 0) {             // 0 = unset (:1537-1539)
            if (priv) po += o;     // relative -> absolute (:1542-1544)
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

// ---- firewall element: GetScore, shouldBlock, verdict (firewall.go:34-52)
__global__ __launch_bounds__(256) void firewall_mark_kernel(const uint8_t* in, const u64* rec_off, u64 n, u32 toff,
                                                            int32_t threshold, int32_t* score, uint8_t* verdict,
                                                            Pair* kept) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i > n) return;
    if (i == n) {
        kept[n] = Pair{0, 0};
        return;
    }
    const u64 s = rec_off[i], L = rec_off[i + 1] - s;
    const int32_t sc = L >= (u64)toff + 4 ? (int32_t)ld_u32((uintptr_t)(in + s) + toff) : 0;  // kv.syn.go:285-291
    const bool drop = sc >= threshold;
    if (score) score[i] = sc;
    verdict[i] = drop ? SYM_VERDICT_DROP : SYM_VERDICT_PASS;
    kept[i] = drop ? Pair{0, 0} : Pair{L, 1};
}

// ---- gather: out[dst[i] .. dst[i+1]) = in[src[i] .. src[i] + dst[i+1] - dst[i])
struct GatherArgs {
    const uint8_t* in;
    const u64* rec_off;  // [0] and [n]: the readable input range (for the unconditional loads)
    const u64* src;      // per segment: source byte offset in `in`
    const u64* dst;      // n+1 output offsets, element stride `ds` u64s (1: offsets, 2: Pair.bytes)
    int ds;
    u64 n;
    uint8_t* out;
    u64 cap;
    u64* kept_off;    // FW: compacted record offsets (nkept+1)
    u64* kept_index;  // FW: input position of each kept record (nullable)
    u64* nkept;       // FW
    unsigned* err;
};

struct WaveLds {
    u64 addr[kSegs];  // segment's source address
    int o[kSegs + 1];  // segment's output start relative to the tile; [cnt] = span
};

template <bool FW>
__global__ __launch_bounds__(kWaves * 64) void gather_kernel(GatherArgs a) {
    __shared__ WaveLds lds_all[kWaves];
    __shared__ MaskTable masks;
    mask_table_init(masks, threadIdx.x);
    __syncthreads();  // the only workgroup barrier
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    WaveLds& S = lds_all[wave];
    const u64 r0 = ((u64)blockIdx.x * kWaves + wave) * kSegs;
    if (r0 >= a.n) return;  // wave-uniform
    const int cnt = (int)min((u64)kSegs, a.n - r0);
    const int ds = a.ds;
    if (a.dst[a.n * ds] > a.cap) {  // output does not fit: nothing is written
        if (lane == 0 && r0 == 0) atomicOr(a.err, kErrCapacity);
        return;
    }
    const u64 D0 = a.dst[r0 * ds], D1 = a.dst[(r0 + cnt) * ds];
    if (D1 - D0 >= ((u64)1 << 31)) {  // tile positions are 32-bit
        if (lane == 0) atomicOr(a.err, kErrTooLarge);
        return;
    }
    const u64 in_lo = a.rec_off[0], in_hi = a.rec_off[a.n];

    // ---- phase 1 (lane = segment)
    bool interior = true;
    if (lane < cnt) {
        const u64 i = r0 + lane;
        const u64 d = a.dst[i * ds], len = a.dst[(i + 1) * ds] - d;
        const u64 src = a.src[i];
        S.addr[lane] = (u64)(uintptr_t)(a.in + src);
        S.o[lane] = (int)(d - D0);
        if (lane == cnt - 1) S.o[cnt] = (int)(D1 - D0);
        // a 16-byte window reads up to 15 bytes either side of its segment
        interior = len == 0 || (src >= in_lo + 16 && src + len + 16 <= in_hi);
        if constexpr (FW) {
            const u64 c0 = a.dst[i * 2 + 1], c1 = a.dst[(i + 1) * 2 + 1];
            if (c1 > c0) {
                a.kept_off[c0] = d;
                if (a.kept_index) a.kept_index[c0] = i;
            }
            if (i == a.n - 1) {
                a.kept_off[c1] = d + len;
                *a.nkept = c1;
            }
        }
    }
    const bool safe = __all(interior);
    wave_sync();

    // ---- phase 2 (lane = aligned 16-byte output chunk)
    const int span = (int)(D1 - D0);
    const i64 mis = (i64)((uintptr_t)a.out & 15);
    const int firstc = (int)((((i64)D0 + mis) & ~(i64)15) - mis - (i64)D0);  // in (-16, 0]
    uint8_t* const out_t = a.out + D0;
    for (int B = firstc; B < span; B += 16 * 64) {  // wave-uniform loop
        const int P = B + 16 * lane;
        if (P >= span) continue;
        u32x4 r = {0, 0, 0, 0};
        for (int k = lds_search_64(S.o, cnt, max(P, 0)); k < cnt; ++k) {
            const int lo = S.o[k] - P;
            if (lo >= 16) break;
            const int hi = min(S.o[k + 1] - P, 16);
            if (hi <= max(lo, 0)) continue;  // empty segment
            const uintptr_t X0 = (uintptr_t)(S.addr[k] + (u64)(i64)(P - S.o[k]));  // chunk byte t <- X0 + t
            if (safe) {
                r |= ld16u(X0) & range_mask(masks, lo, hi);
            } else {  // batch-edge tiles: only the aligned blocks holding wanted bytes
                u32 t[4] = {r.x, r.y, r.z, r.w};
                or_window_global(X0, max(lo, 0), hi, t);
                r = u32x4{t[0], t[1], t[2], t[3]};
            }
        }
        const u32 rr[4] = {r.x, r.y, r.z, r.w};
        store_chunk(out_t, P, 0, span, rr);
    }
}

template <typename T, typename Op>
size_t scan_temp(u64 n, Op op) {
    size_t bytes = 0;
    (void)rocprim::exclusive_scan(nullptr, bytes, (const T*)nullptr, (T*)nullptr, T{}, (size_t)n + 1, op);
    return (bytes + 255) & ~(size_t)255;
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

hipError_t launch_gather(const GatherArgs& a, bool fw, hipStream_t stream) {
    const u64 tiles = (a.n + kSegs - 1) / kSegs;
    const dim3 grid((unsigned)((tiles + kWaves - 1) / kWaves)), block(kWaves * 64);
    if (fw) hipLaunchKernelGGL(gather_kernel<true>, grid, block, 0, stream, a);
    else hipLaunchKernelGGL(gather_kernel<false>, grid, block, 0, stream, a);
    return hipGetLastError();
}

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

size_t raw_bytes_ws_bytes(u64 n) {
    return 2 * raw::al256((n + 1) * sizeof(u64)) + raw::scan_temp<u64>(n, rocprim::plus<u64>());
}

hipError_t launch_raw_bytes(const uint8_t* in, const u64* rec_off, u64 n, int priv, u32 table_off, uint8_t* out,
                            u64 cap, u64* out_off, uint8_t* status, void* ws, unsigned* err, hipStream_t stream) {
    const size_t col = raw::al256((n + 1) * sizeof(u64));
    u64* seg_src = (u64*)ws;
    u64* seg_len = (u64*)((char*)ws + col);
    void* temp = (char*)ws + 2 * col;
    size_t tb = raw::scan_temp<u64>(n, rocprim::plus<u64>());
    hipLaunchKernelGGL(raw::var_locate_kernel, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, stream, in,
                       rec_off, n, priv, table_off, seg_src, seg_len, status);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan(temp, tb, (const u64*)seg_len, out_off, (u64)0, (size_t)n + 1, rocprim::plus<u64>(),
                                stream);
    if (e != hipSuccess || n == 0) return e;
    raw::GatherArgs a{};
    a.in = in;
    a.rec_off = rec_off;
    a.src = seg_src;
    a.dst = out_off;
    a.ds = 1;
    a.n = n;
    a.out = out;
    a.cap = cap;
    a.err = err;
    return raw::launch_gather(a, false, stream);
}

size_t firewall_ws_bytes(u64 n) {
    return 2 * raw::al256((n + 1) * sizeof(raw::Pair)) + raw::scan_temp<raw::Pair>(n, raw::PairPlus());
}

hipError_t launch_firewall(const uint8_t* in, const u64* rec_off, u64 n, u32 score_table_off, int32_t threshold,
                           int32_t* score, uint8_t* verdict, uint8_t* kept, u64 cap, u64* kept_off, u64* kept_index,
                           u64* nkept, void* ws, unsigned* err, hipStream_t stream) {
    const size_t col = raw::al256((n + 1) * sizeof(raw::Pair));
    raw::Pair* mark = (raw::Pair*)ws;
    raw::Pair* pre = (raw::Pair*)((char*)ws + col);
    void* temp = (char*)ws + 2 * col;
    size_t tb = raw::scan_temp<raw::Pair>(n, raw::PairPlus());
    hipLaunchKernelGGL(raw::firewall_mark_kernel, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, stream, in,
                       rec_off, n, score_table_off, threshold, score, verdict, mark);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan(temp, tb, (const raw::Pair*)mark, pre, raw::Pair{0, 0}, (size_t)n + 1,
                                raw::PairPlus(), stream);
    if (e != hipSuccess) return e;
    raw::GatherArgs a{};
    a.in = in;
    a.rec_off = rec_off;
    a.src = rec_off;
    a.dst = (const u64*)pre;
    a.ds = 2;
    a.n = n;
    a.out = kept;
    a.cap = cap;
    a.kept_off = kept_off;
    a.kept_index = kept_index;
    a.nkept = nkept;
    a.err = err;
    return raw::launch_gather(a, true, stream);
}

}  // namespace symhip
