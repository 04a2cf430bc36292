// encode.hip -- batched Symphony MarshalSymphony for flat schemas on gfx950.
//
// Restates, for n records at once, the generated per-record marshaller
//   benchmark/kv-store-symphony/symphony/kv.syn.go:611-678 (SetRequest; Get/Resp/Echo analogous)
// from the generator's layout rules (cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:196-330,
// :439-491) plus the client's ID patch (pkg/rpc/client.go:267-271).
//
// Design (output-stationary, one pass):
//  * A workgroup owns a tile of kTile=256 consecutive records.  Record i starts at
//      out_off[i] = i*OVH + sum_f (offs_f[i] - offs_f[0])
//    (an affine function of the input offsets: no scan needed on encode).
//  * Phase 1 (one thread per record): read the offsets, write out_off, and build the
//    record's header image -- version bytes, offset_to_private, IDs, the private
//    table and the first length prefix, H0 bytes -- in a zero-padded 64-byte LDS slot.
//  * Phase 2 (one thread per aligned 16-byte output chunk): locate the chunk's record
//    by binary search over the tile's record starts in LDS, OR together the header
//    window (LDS), the string payload windows (two aligned 16-byte global loads,
//    funnel-shifted with v_alignbyte) and the inner length prefixes (register
//    shifts), then issue one global_store_dwordx4.  Only the partial chunks at the
//    tile's two edges use byte stores, so no chunk is ever read-modified-written.
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

template <int NF, int NV>
__global__ __launch_bounds__(256) void encode_kernel(EncodeParams p) {
    constexpr int NT = NF + NV;
    constexpr int H0 = 14 + 4 * NT + 4;          // bytes before field 0's payload
    constexpr i64 OVH = 14 + 4 * NT + 4 * NV;    // fixed bytes per record
    constexpr int SLOT = 64;                     // header image bytes per record (H0 <= 34)
    static_assert(H0 + 20 <= SLOT && OVH >= 16, "layout assumptions");

    __shared__ u64 s_o[kTile + 1];               // tile record starts (stream positions)
    __shared__ u64 s_src[NV][kTile];             // offs_f[i]: payload start in column f
    __shared__ u64 s_len[NV][kTile];
    __shared__ __attribute__((aligned(16))) u32 s_hdr[(kTile + 2) * SLOT / 4];  // slot 0: zero pad

    const int tid = threadIdx.x;
    const u64 r0 = (u64)blockIdx.x * kTile;
    const int cnt = (int)min((u64)kTile, p.n - r0);

    // ---------------- phase 1: per-record offsets and header images ----------------
    if (tid < cnt) {
        const u64 r = r0 + tid;
        i64 o = (i64)r * OVH;
        u64 L[NV];
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 lo = p.offs[f][r];
            L[f] = p.offs[f][r + 1] - lo;
            o += (i64)(lo - p.offs[f][0]);
            s_src[f][tid] = lo;
            s_len[f][tid] = L[f];
        }
        s_o[tid] = (u64)o;
        p.out_off[r] = (u64)o;
        u64 size = (u64)OVH;
#pragma unroll
        for (int f = 0; f < NV; ++f) size += L[f];
        if (tid == cnt - 1) {
            s_o[cnt] = (u64)o + size;
            if (r == p.n - 1) p.out_off[p.n] = (u64)o + size;
        }
        // header image: [0]=1 | [1:5]=13 | [5:9]=sid | [9:13]=mid | [13]=1 | table | len(field 0)
        u32 h[SLOT / 4];
#pragma unroll
        for (int k = 0; k < SLOT / 4; ++k) h[k] = 0;
        img_put_u8<0>(h, 1);
        img_put_u32<1>(h, 13);
        img_put_u32<5>(h, p.service_id);
        img_put_u32<9>(h, p.method_id);
        img_put_u8<13>(h, 1);
        if constexpr (NF > 0) img_put_u32<14>(h, (u32)p.fixed[0][r]);
        if constexpr (NF > 1) img_put_u32<18>(h, (u32)p.fixed[1][r]);
        // private-table entries: offset of the field's length prefix relative to privateStart
        // (13), truncated to u32 (kv.syn.go:664, :671).  ps = start of field 0's payload.
        u64 ps = H0;
        img_put_u32<14 + 4 * NF>(h, (u32)(ps - 4 - 13));
        if constexpr (NV > 1) {
            ps += L[0] + 4;
            img_put_u32<18 + 4 * NF>(h, (u32)(ps - 4 - 13));
        }
        img_put_u32<H0 - 4>(h, (u32)L[0]);
        uint4* slot = (uint4*)&s_hdr[(tid + 1) * (SLOT / 4)];
#pragma unroll
        for (int k = 0; k < SLOT / 16; ++k) slot[k] = make_uint4(h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3]);
    }
    if (tid < SLOT / 4) s_hdr[tid] = 0;
    __syncthreads();

    // ---------------- phase 2: one aligned 16-byte output chunk per thread ----------------
    const i64 tile_lo = (i64)s_o[0];
    const i64 tile_hi = (i64)s_o[cnt];
    const i64 mis = (i64)((uintptr_t)p.out & 15);
    const i64 first = ((tile_lo + mis) & ~(i64)15) - mis;  // chunk grid is aligned in absolute addresses
    for (i64 P = first + 16 * tid; P < tile_hi; P += 16 * kTile) {
        const i64 Pc = P > tile_lo ? P : tile_lo;
        const int j = lds_search_256(s_o, cnt, (u64)Pc);
        const i64 b = P - (i64)s_o[j];  // chunk start relative to record j (> -16)
        u32 r[4] = {0, 0, 0, 0};
        if (b < H0) or_window_lds(s_hdr, (j + 1) * SLOT + (int)b, r);
        i64 ps = H0;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const i64 L = (i64)s_len[f][j];
            if (f > 0) {
                const i64 t = ps - 4 - b;  // inner length prefix of field f
                if (t > -4 && t < 16) or_u32_at((u32)L, (int)t, r);
            }
            const i64 tlo = ps - b > 0 ? ps - b : 0;
            const i64 thi = ps + L - b < 16 ? ps + L - b : 16;
            if (tlo < thi) {
                const uintptr_t X = (uintptr_t)(p.bytes[f] + s_src[f][j]) + (uintptr_t)(b - ps);
                or_window_global(X, (int)tlo, (int)thi, r);
            }
            ps += L + 4;
        }
        if (j + 1 < cnt) {  // the next record's header may start inside this chunk
            const i64 nb = P - (i64)s_o[j + 1];
            if (nb > -16) or_window_lds(s_hdr, (j + 2) * SLOT + (int)nb, r);
        }
        store_chunk(p.out, P, tile_lo, tile_hi, r);
    }
}

hipError_t launch_encode(const EncodeParams& p, hipStream_t stream) {
    if (p.n == 0) return hipMemsetAsync(p.out_off, 0, sizeof(uint64_t), stream);
    const dim3 grid((unsigned)((p.n + kTile - 1) / kTile));
    const dim3 block(256);
    if (p.lay.nfixed == 0 && p.lay.nvar == 1)
        hipLaunchKernelGGL((encode_kernel<0, 1>), grid, block, 0, stream, p);
    else if (p.lay.nfixed == 0 && p.lay.nvar == 2)
        hipLaunchKernelGGL((encode_kernel<0, 2>), grid, block, 0, stream, p);
    else if (p.lay.nfixed == 2 && p.lay.nvar == 2)
        hipLaunchKernelGGL((encode_kernel<2, 2>), grid, block, 0, stream, p);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace symhip
