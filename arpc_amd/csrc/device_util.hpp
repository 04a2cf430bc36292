// device_util.hpp -- byte-shuffle primitives for the gfx950 Symphony kernels.
//
// The codec is an HBM-bound byte shuffle: records start at arbitrary byte offsets,
// so every output 16-byte chunk is assembled in registers from (a) aligned 16-byte
// global loads funnel-shifted with v_alignbyte_b32 and (b) header bytes synthesized
// per record and staged in LDS.  No byte-granular global stores except at the two
// edges of a workgroup's output range.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace symhip {

typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t i64;

// Explicit global address space so loads/stores lower to global_* (not flat_*).
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gc_u4;
typedef __attribute__((address_space(1))) const u32 gc_u32;
typedef __attribute__((address_space(1))) const uint8_t gc_u8;
typedef __attribute__((address_space(1))) u32x4 g_u4;
typedef __attribute__((address_space(1))) uint8_t g_u8;

__device__ __forceinline__ u32 alignbyte(u32 hi, u32 lo, u32 sh) { return __builtin_amdgcn_alignbyte(hi, lo, sh); }

// u32 at byte q (q <= 4*NW-4) of a register window w[0..NW): bit-select the dword pair (a dynamic
// register index would go to scratch) and align.
template <int NW>
__device__ __forceinline__ u32 win_u32(const u32 (&w)[NW], u32 q) {
    const u32 d = q >> 2;
    u32 lo = w[0], hi = w[1];
#pragma unroll
    for (int k = 1; k < NW; ++k) {
        lo = d == (u32)k ? w[k] : lo;
        hi = d == (u32)k ? (k < NW - 1 ? w[k + 1] : 0u) : hi;
    }
    return alignbyte(hi, lo, q & 3);
}

// Mask selecting chunk bytes [lo, hi) inside dword k (lo, hi in [-inf, +inf], clamped).
__device__ __forceinline__ u32 dword_mask(int lo, int hi, int k) {
    const int a = min(max(lo - 4 * k, 0), 4);
    const int b = min(max(hi - 4 * k, 0), 4);
    const u64 m = ((1ull << (8 * b)) - 1ull) & ~((1ull << (8 * a)) - 1ull);
    return (u32)m;
}

// Bytes [s, s+16) of the 32-byte concatenation a|b (s in [0,16)).  The dword barrel
// shift by s>>2 is written as bit-selects (v_bfi_b32): a `c ? d[k+2] : d[k]` form gets
// folded into a dynamic index and spilled to scratch.
__device__ __forceinline__ void funnel16(const u32x4 a, const u32x4 b, u32 s, u32 out[4]) {
    const u32 d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const u32 m2 = (s & 8) ? ~0u : 0u, m1 = (s & 4) ? ~0u : 0u;
    u32 e[6], f[5];
#pragma unroll
    for (int k = 0; k < 6; ++k) e[k] = (d[k + 2] & m2) | (d[k] & ~m2);
#pragma unroll
    for (int k = 0; k < 5; ++k) f[k] = (e[k + 1] & m1) | (e[k] & ~m1);
    const u32 sh = s & 3;
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = alignbyte(f[k + 1], f[k], sh);
}

// OR into r the chunk bytes t in [t_lo, t_hi) (0 <= t_lo < t_hi <= 16) taken from
// global memory at X + t.  Only the aligned 16-byte blocks that hold at least one
// of those bytes are loaded, so a caller whose [X+t_lo, X+t_hi) lies inside a
// buffer never touches memory past that buffer's last 16-byte block.
__device__ __forceinline__ void or_window_global(uintptr_t X, int t_lo, int t_hi, u32 r[4]) {
    const uintptr_t B0 = X & ~(uintptr_t)15;
    u32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
    if (X + (uintptr_t)t_lo < B0 + 16) a = *(gc_u4*)B0;
    if (X + (uintptr_t)t_hi > B0 + 16) b = *(gc_u4*)(B0 + 16);
    u32 w[4];
    funnel16(a, b, (u32)(X & 15), w);
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] |= w[k] & dword_mask(t_lo, t_hi, k);
}

// The two aligned blocks an interior chunk (all 16 bytes at X valid) needs; the second
// only when X is unaligned (so it holds valid bytes too).
__device__ __forceinline__ void load_interior(uintptr_t X, u32x4& a, u32x4& b) {
    const uintptr_t B0 = X & ~(uintptr_t)15;
    a = *(gc_u4*)B0;
    b = u32x4{0, 0, 0, 0};
    if (X & 15) b = *(gc_u4*)(B0 + 16);
}

// Byte-unaligned 16-byte global load (gfx950 handles byte-aligned global_load_dwordx4 at
// full rate; tools/ubench_unaligned.hip).  The caller guarantees [X, X+16) is readable.
__device__ __forceinline__ u32x4 ld16u(uintptr_t X) { return *(gc_u4*)X; }

// Byte-unaligned 16-byte LDS read (ds_read_b128 at any byte address).
__device__ __forceinline__ u32x4 lds16u(const void* base, int byte_off) {
    return *(const u32x4*)((const char*)base + byte_off);
}

// Chunk byte masks from a 17-entry table: lowmask[n] has bytes [0, n) set.
struct MaskTable {
    u32x4 lm[17];
};
__device__ __forceinline__ void mask_table_init(MaskTable& t, int tid) {
    if (tid < 17) {
        u32 w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = dword_mask(0, tid, k);
        t.lm[tid] = u32x4{w[0], w[1], w[2], w[3]};
    }
}
// bytes [lo, hi) of a chunk, lo/hi clamped to [0, 16]
__device__ __forceinline__ u32x4 range_mask(const MaskTable& t, int lo, int hi) {
    lo = min(max(lo, 0), 16);
    hi = min(max(hi, 0), 16);
    return t.lm[hi] & ~t.lm[lo];
}

// OR into r the 16 bytes of an LDS byte image starting at byte address `addr`
// (dword-aligned reads + alignbyte).  Callers keep the image zero outside the
// bytes they want, so no mask is needed.
__device__ __forceinline__ void or_window_lds(const u32* img, int addr, u32 r[4]) {
    const int q = addr >> 2;
    const u32 sh = (u32)addr & 3u;
    u32 d[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) d[k] = img[q + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] |= alignbyte(d[k + 1], d[k], sh);
}

// OR a little-endian u32 into chunk bytes [t, t+4) clipped to [0, 16); t in (-4, 16).
__device__ __forceinline__ void or_u32_at(u32 v, int t, u32 r[4]) {
    const u64 vv = (u64)v << 32;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int sh = t - 4 * k;  // byte position of v's byte 0 relative to dword k
        if (sh > -4 && sh < 4) r[k] |= (u32)(vv >> (32 - 8 * sh));
    }
}

// Compile-time-positioned byte writes into a small dword image.
template <int POS>
__device__ __forceinline__ void img_put_u32(u32* h, u32 v) {
    constexpr int q = POS >> 2, sh = (POS & 3) * 8;
    h[q] |= v << sh;
    if constexpr (sh != 0) h[q + 1] |= v >> (32 - sh);
}
template <int POS>
__device__ __forceinline__ void img_put_u8(u32* h, u32 v) {
    h[POS >> 2] |= (v & 0xffu) << ((POS & 3) * 8);
}

__device__ __forceinline__ uint8_t chunk_byte(const u32 r[4], int t) {
    const u32 m1 = t >= 4 ? ~0u : 0u, m2 = t >= 8 ? ~0u : 0u, m3 = t >= 12 ? ~0u : 0u;
    u32 w = (r[1] & m1) | (r[0] & ~m1);
    w = (r[2] & m2) | (w & ~m2);
    w = (r[3] & m3) | (w & ~m3);
    return (uint8_t)(w >> ((t & 3) * 8));
}

// A 16-byte output store of the streaming kernels, nontemporal where it pays: nothing in the launch
// re-reads the written lines.  One-box A/B of libraries (round 5): with 22 KB or smaller tiles (config 2,
// the Get/Set mix) nontemporal stores took config 2's encode 145 -> 141 us, its decode 152.5 -> 145.5 us
// and the mix's pair 3.6 -> 3.8 TB/s; with tiles of tens to hundreds of KB (config 3, the trace replays)
// they cost 1-8 % (config3_trace decode 1.40 -> 1.51 ms), so the kernels pass nt = their tile's span
// <= kNtSpan.  `sc1` stores (the line leaves the XCD's L2) gained nothing.  Span-gated library against
// plain stores, two runs each on one box: headline 4995 -> 5100 GB/s (decode 151 -> 146 us), N3
// reassembly 2670 -> 2840 GB/s, config 3 / the trace replays / the N5 legs within +-2 %.  The threshold,
// two runs each: 16 KB loses config 2's 22 KB tiles (headline 5100 -> 4945 GB/s), 64 KB takes config 3's
// ~53 KB tiles (4590 -> 4525 GB/s).  Every call site passes nt explicitly: the span-gated kernels above,
// and `true` where the kernel was measured with nontemporal stores at every span (the cipher, the N5
// copies, the packetizer, the three-kernel decode; round-5 A/B of the libraries, every leg).
constexpr i64 kNtSpan = 32768;
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v, bool nt) {
    if (nt) {
        // the empty asm statements keep the compiler from hoisting or sinking the two stores into
        // one (merged, the store loses its nontemporal flag)
        asm volatile("");
        __builtin_nontemporal_store(v, (g_u4*)p);
        asm volatile("");
    } else {
        *(g_u4*)p = v;
    }
}

// Store a 16-byte chunk at dst (absolute, 16-byte aligned) keeping only the bytes
// whose position P+t lies in [lo, hi).  Full chunks use one global_store_dwordx4;
// the partial chunks at a workgroup's range edges fall back to byte stores.
__device__ __forceinline__ void store_chunk(uint8_t* base, i64 P, i64 lo, i64 hi, const u32 r[4], bool nt) {
    if (P >= lo && P + 16 <= hi) {
        st16(base + P, u32x4{r[0], r[1], r[2], r[3]}, nt);
    } else {
        for (int t = 0; t < 16; ++t) {
            const i64 q = P + t;
            if (q >= lo && q < hi) *(g_u8*)(base + q) = chunk_byte(r, t);
        }
    }
}

// Largest j in [0, cnt) with a[j] <= key (a ascending, a[0] <= key); cnt <= 256.
__device__ __forceinline__ int lds_search_256(const u64* a, int cnt, u64 key) {
    int j = 0;
#pragma unroll
    for (int step = 128; step > 0; step >>= 1) {
        const int c = j + step;
        if (c < cnt && a[c] <= key) j = c;
    }
    return j;
}

// Unaligned reads inside a record: only dwords holding at least one of the four
// requested bytes are touched.
__device__ __forceinline__ u32 ld_u8(uintptr_t p) { return *(gc_u8*)p; }
__device__ __forceinline__ u32 ld_u32(uintptr_t p) {
    const uintptr_t a = p & ~(uintptr_t)3;
    const u32 sh = (u32)(p & 3);
    const u32 lo = *(gc_u32*)a;
    const u32 hi = sh ? *(gc_u32*)(a + 4) : 0u;
    return alignbyte(hi, lo, sh);
}

// Broadcast lane 0's value as a provably wave-uniform (SGPR) value.
__device__ __forceinline__ i64 uniform_i64(i64 x) {
    const u32 lo = __builtin_amdgcn_readfirstlane((u32)(u64)x);
    const u32 hi = __builtin_amdgcn_readfirstlane((u32)((u64)x >> 32));
    return (i64)(((u64)hi << 32) | lo);
}

// Order LDS traffic between lanes of ONE wave (no workgroup barrier).  The fences name the
// local address space only: a wavefront fence over all address spaces makes the compiler wait for
// every global load in flight (s_waitcnt vmcnt(0)), which serialises software-pipelined loops.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
// The same for global memory as well (a global read by every lane before one lane's write).
__device__ __forceinline__ void wave_sync_global() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 64-lane inclusive scan of a u32 with DPP row shifts and row broadcasts (GFX9 wave64):
// six VALU ops, no LDS round trips.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ u32 dpp_add(u32 v) {
    return v + (u32)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWMASK, 0xf, false);
}
__device__ __forceinline__ u32 wave_incl_scan_u32_dpp(u32 v) {
    v = dpp_add<0x111, 0xf>(v);  // row_shr:1
    v = dpp_add<0x112, 0xf>(v);  // row_shr:2
    v = dpp_add<0x114, 0xf>(v);  // row_shr:4
    v = dpp_add<0x118, 0xf>(v);  // row_shr:8
    v = dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
    v = dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
    return v;
}

// 64-lane inclusive max-scan of a u32 (same DPP pattern; shifted-in lanes read 0).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ u32 dpp_max(u32 v) {
    return max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWMASK, 0xf, false));
}
__device__ __forceinline__ u32 wave_incl_max_u32_dpp(u32 v) {
    v = dpp_max<0x111, 0xf>(v);
    v = dpp_max<0x112, 0xf>(v);
    v = dpp_max<0x114, 0xf>(v);
    v = dpp_max<0x118, 0xf>(v);
    v = dpp_max<0x142, 0xa>(v);
    v = dpp_max<0x143, 0xc>(v);
    return v;
}

// 64-lane inclusive scan of values < 2^32 with a 64-bit result: two 32-bit DPP scans over a
// 25/7-bit split (64 * 2^25 fits in 32 bits), no shuffles, no branches.
__device__ __forceinline__ u64 wave_incl_scan_u32w_dpp(u32 v) {
    const u32 lo = wave_incl_scan_u32_dpp(v & 0x1FFFFFFu);
    const u32 hi = wave_incl_scan_u32_dpp(v >> 25);
    return ((u64)hi << 25) + lo;
}

// 64-lane inclusive scan of values < 2^43 with a 64-bit result: two 32-bit DPP scans over a
// 22/21-bit split (64 * 2^22 fits in 32 bits).  No shuffles: no permute-address registers held
// across a loop (the streaming scanner's, pipe_words.hpp).
__device__ __forceinline__ u64 wave_incl_scan_u43_dpp(u64 v) {
    const u32 lo = wave_incl_scan_u32_dpp((u32)v & 0x3FFFFFu);
    const u32 hi = wave_incl_scan_u32_dpp((u32)(v >> 22));
    return ((u64)hi << 22) + lo;
}

// 64-lane inclusive scan of a u32.
__device__ __forceinline__ u32 wave_incl_scan_u32(u32 v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// Largest j in [0, cnt) with a[j] <= key (a ascending, a[0] <= key); cnt <= 64.
template <typename T>
__device__ __forceinline__ int lds_search_64(const T* a, int cnt, T key) {
    int j = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1) {
        const int c = j + step;
        if (c < cnt && a[c] <= key) j = c;
    }
    return j;
}

// 64-lane inclusive scan of a u64 (two 32-bit shuffles per step).
__device__ __forceinline__ u64 wave_incl_scan_u64(u64 v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 lo = __shfl_up((u32)v, d, 64);
        const u32 hi = __shfl_up((u32)(v >> 32), d, 64);
        if (lane >= d) v += ((u64)hi << 32) | lo;
    }
    return v;
}

__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        const u32 lo = __shfl_xor((u32)v, d, 64);
        const u32 hi = __shfl_xor((u32)(v >> 32), d, 64);
        v += ((u64)hi << 32) | lo;
    }
    return v;
}

}  // namespace symhip
