// encode.hip -- batched Symphony MarshalSymphony for flat schemas on gfx950.
//
// Restates, for n records at once, the generated per-record marshaller
//   benchmark/kv-store-symphony/symphony/kv.syn.go:611-678 (SetRequest; Get/Resp/Echo analogous)
// from the generator's layout rules (cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:196-330,
// :439-491) plus the client's ID patch (pkg/rpc/client.go:267-271).
//
// Design (output-stationary, one pass, one independent tile per wave):
//  * Each wave owns kWaveRecs=64 consecutive records; the 4 waves of a workgroup never
//    synchronize after setup.  Record i starts at
//      out_off[i] = i*OVH + sum_f (offs_f[i] - offs_f[0])
//    (affine in the input offsets: no scan on encode).
//  * Phase 1 (lane = record): read offsets, write out_off, and build the record's header
//    image -- version bytes, offset_to_private, IDs, private table, first length prefix --
//    in a zero-padded LDS slot.
//  * Phase 2 (lane = aligned 16-byte output chunk, natural order, 2 chunks per lane per
//    step): binary-search the chunk's record in LDS, then
//      chunk = header window (one unaligned ds_read_b128 of the record's slot)
//            | payload f window (one byte-unaligned global_load_dwordx4) & byte mask
//            | inner length prefixes (register shifts)
//            | next record's header window.
//    gfx950 serves byte-unaligned 16-byte loads at full rate, so there is no funnel shift.
//    One global_store_dwordx4 per chunk, consecutive lanes on consecutive chunks: every
//    wave store instruction writes 1 KiB of whole lines.  Only the partial chunks at a
//    tile's two edges use byte stores, so nothing is read-modify-written.
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

constexpr int kWaveRecs = 64;  // records per wave tile
constexpr int kWaves = 4;      // wave tiles per 256-thread workgroup

// Header slot for H0 header bytes: a 16-byte window starting at any b < H0 stays in the slot,
// and one starting up to 15 bytes before a slot reads only the previous slot's zero tail.
constexpr int slot_bytes(int H0) { return ((H0 + 16) + 7) & ~7; }

// A tile's stream span must stay below 2^31 (64 records; positions are 32-bit), and string
// fields are < 2^32 bytes (Symphony's u32 length prefix).
template <int NV, int SLOT>
struct EncWaveLds {
    char hdr[(kWaveRecs + 1) * SLOT];  // slot 0 = zero pad, slot i+1 = record i
    int o[kWaveRecs + 1];              // record start relative to the tile start; [cnt] = span
    u32 len[NV][kWaveRecs];
    u64 delta[NV][kWaveRecs];          // payload byte address = delta + chunk position
    uint8_t flags[64];                 // record-start marks of one phase-2 step
};

template <int NF, int NV, int kVariant>
__global__ __launch_bounds__(256) void encode_kernel(EncodeParams p) {
    constexpr int NT = NF + NV;
    constexpr int H0 = 14 + 4 * NT + 4;        // bytes before field 0's payload
    constexpr i64 OVH = 14 + 4 * NT + 4 * NV;  // fixed bytes per record
    constexpr int SLOT = slot_bytes(H0);
    static_assert(SLOT - 16 >= H0 && OVH >= 16, "layout assumptions");

    __shared__ EncWaveLds<NV, SLOT> lds_all[kWaves];
    __shared__ MaskTable masks;
    mask_table_init(masks, threadIdx.x);
    __syncthreads();  // the only workgroup barrier

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    EncWaveLds<NV, SLOT>& S = lds_all[wave];
    const u64 r0 = ((u64)blockIdx.x * kWaves + wave) * kWaveRecs;
    if (r0 >= p.n) return;  // wave-uniform
    const int cnt = (int)min((u64)kWaveRecs, p.n - r0);

    // ---------------- phase 1: per-record offsets and header image ----------------
    i64 o = 0, size = 0;
    u64 L[NV];
    if (lane < cnt) {
        const u64 r = r0 + lane;
        o = (i64)r * OVH;
        size = OVH;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 lo = p.offs[f][r];
            L[f] = p.offs[f][r + 1] - lo;
            o += (i64)(lo - p.offs[f][0]);
            size += (i64)L[f];
            S.len[f][lane] = (u32)L[f];
        }
        p.out_off[r] = (u64)o;
        if (r == p.n - 1) p.out_off[p.n] = (u64)(o + size);
    }
    // wave-uniform: readfirstlane keeps them (and the phase-2 loop bounds) in SGPRs
    const i64 T0 = uniform_i64((i64)__shfl((long long)o, 0, 64));
    const i64 T1 = uniform_i64((i64)__shfl((long long)(o + size), cnt - 1, 64));
    if (T1 - T0 >= (i64)1 << 31) {  // positions are 32-bit inside a tile
        if (lane == 0) atomicOr(p.err, kErrTooLarge);
        return;
    }
    if (lane < cnt) {
        const u64 r = r0 + lane;
        const int orel = (int)(o - T0);
        S.o[lane] = orel;
        if (lane == cnt - 1) S.o[cnt] = (int)(T1 - T0);
        int ps = H0;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            S.delta[f][lane] = (u64)(uintptr_t)(p.bytes[f] + p.offs[f][r]) - (u64)(i64)(orel + ps);
            ps += (int)L[f] + 4;
        }
        // header image: [0]=1 | [1:5]=13 | [5:9]=sid | [9:13]=mid | [13]=1 | table | len(field 0)
        u32 h[SLOT / 4 + 1];
#pragma unroll
        for (int k = 0; k < SLOT / 4 + 1; ++k) h[k] = 0;
        img_put_u8<0>(h, 1);
        img_put_u32<1>(h, 13);
        img_put_u32<5>(h, p.service_id);
        img_put_u32<9>(h, p.method_id);
        img_put_u8<13>(h, 1);
        if constexpr (NF > 0) img_put_u32<14>(h, (u32)p.fixed[0][r]);
        if constexpr (NF > 1) img_put_u32<18>(h, (u32)p.fixed[1][r]);
        // private-table entries: offset of the field's length prefix relative to privateStart
        // (13), truncated to u32 (kv.syn.go:664, :671).
        img_put_u32<14 + 4 * NF>(h, (u32)(H0 - 4 - 13));
        if constexpr (NV > 1) img_put_u32<18 + 4 * NF>(h, (u32)(H0 + L[0] + 4 - 4 - 13));
        img_put_u32<H0 - 4>(h, (u32)L[0]);
        uint2* slot = (uint2*)&S.hdr[(lane + 1) * SLOT];
#pragma unroll
        for (int k = 0; k < SLOT / 8; ++k) slot[k] = make_uint2(h[2 * k], h[2 * k + 1]);
    }
    if (lane < SLOT / 4) ((u32*)S.hdr)[lane] = 0;
    S.flags[lane] = 0;
    wave_sync();

    // ---------------- phase 2: natural-order output chunks ----------------
    const int span = (int)(T1 - T0);
    const i64 mis = (i64)((uintptr_t)p.out & 15);
    const int first = (int)(((T0 + mis) & ~(i64)15) - mis - T0);  // in (-16, 0]
    uint8_t* const out_t = p.out + T0;
    const uintptr_t dummy = (uintptr_t)p.out & ~(uintptr_t)15;  // readable; its bytes get masked off
    // A payload window reads up to 15 bytes beyond its field; that stays inside the column
    // unless the tile's fields sit within 16 bytes of the column's ends (batch edges).
    bool tile_safe = true;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u64 c0 = p.offs[f][0], c1 = p.offs[f][p.n];
        const u64 t0 = p.offs[f][r0], t1 = p.offs[f][r0 + cnt];
        tile_safe = tile_safe && t0 >= c0 + 16 && t1 + 16 <= c1;
    }
    const i64 my_o = lane < cnt ? (i64)S.o[lane] : ((i64)1 << 40);  // record-role register

    // Chunk -> record without searching: records are >= 22 bytes, so at most one record starts
    // inside any 16-byte chunk.  Record k first owns chunk ceil((o_k - B)/16) of this step; a
    // ballot of those marks plus mbcnt gives every lane its record.
    auto locate = [&](int B) -> int {
        const i64 ck = (my_o - B + 15) >> 4;
        const u64 before = __ballot(ck <= 0);
        if (ck >= 1 && ck <= 63) S.flags[ck] = 1;
        wave_sync();
        const bool mine = S.flags[lane] != 0;
        const u64 m = __ballot(mine);
        if (mine) S.flags[lane] = 0;  // clean for the next step (each lane its own byte)
        const int below = (int)__builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
        // (int) casts matter: __popcll is unsigned and max(unsigned, int) picks the double overload
        const int counted = (int)__popcll(before) + below + (mine ? 1 : 0);
        return counted > 0 ? counted - 1 : 0;  // 0 only for the chunk straddling the tile start
    };

    auto chunk = [&](int P, int j, bool careful) {
        const int oj = S.o[j];
        const int b = P - oj;  // chunk start relative to record j (> -16)
        int t = H0 - b;        // chunk offset where field 0's payload starts
        int Lf[NV];
        uintptr_t X[NV];
        bool need[NV], fast[NV];
        u32x4 w[NV];
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            Lf[f] = (int)S.len[f][j];
            X[f] = (uintptr_t)(S.delta[f][j] + (u64)(i64)P);
            need[f] = t < 16 && t + Lf[f] > 0;
            fast[f] = need[f];
            if (careful) {  // the 16-byte window must lie inside the column's 16-byte-rounded extent
                const uintptr_t c0 = (uintptr_t)(p.bytes[f] + p.offs[f][0]) & ~(uintptr_t)15;
                const uintptr_t c1 = ((uintptr_t)(p.bytes[f] + p.offs[f][p.n]) + 15) & ~(uintptr_t)15;
                fast[f] = need[f] && X[f] >= c0 && X[f] + 16 <= c1;
            }
            w[f] = ld16u(fast[f] ? X[f] : dummy);  // unconditional: both loads issue together
            t += Lf[f] + 4;
        }
        u32x4 r = {0, 0, 0, 0};
        if (b < H0) r = lds16u(S.hdr, (j + 1) * SLOT + b);
        t = H0 - b;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            if (f > 0 && t > 0 && t < 20) {  // inner length prefix of field f at [t-4, t)
                u32 tmp[4] = {r.x, r.y, r.z, r.w};
                or_u32_at((u32)Lf[f], t - 4, tmp);
                r = u32x4{tmp[0], tmp[1], tmp[2], tmp[3]};
            }
            if (need[f]) {
                u32x4 v = w[f];
                if (careful && !fast[f]) {  // batch edges: aligned blocks holding valid bytes only
                    u32 tmp[4] = {0, 0, 0, 0};
                    or_window_global(X[f], max(t, 0), min(t + Lf[f], 16), tmp);
                    v = u32x4{tmp[0], tmp[1], tmp[2], tmp[3]};
                }
                r |= v & range_mask(masks, t, t + Lf[f]);
            }
            t += Lf[f] + 4;
        }
        if (j + 1 < cnt) {  // the next record's header may start inside this chunk
            const int nb = P - S.o[j + 1];
            if (nb > -16) r |= lds16u(S.hdr, (j + 2) * SLOT + nb);
        }
        const u32 rr[4] = {r.x, r.y, r.z, r.w};
        store_chunk(out_t, P, 0, span, rr);
    };

    if constexpr (kVariant == 0) {
        for (int B = first; B < span; B += 16 * 64) {  // wave-uniform loop
            const int j = locate(B);
            const int P = B + 16 * lane;
            if (P < span) chunk(P, j, !tile_safe);
        }
        return;
    }
    if (!tile_safe) {  // batch-edge tiles (two per batch): the careful one-step path
        for (int B = first; B < span; B += 16 * 64) {
            const int j = locate(B);
            const int P = B + 16 * lane;
            if (P < span) chunk(P, j, true);
        }
        return;
    }
    // Interior tiles: kU steps per round.  Every payload load of the round is issued before the
    // first store (unconditional loads, so the compiler waits only once), keeping kU KiB of
    // loads in flight per wave instead of one.
    constexpr int kU = kVariant > 0 ? kVariant : 1;
    for (int B0 = first; B0 < span; B0 += 16 * 64 * kU) {  // wave-uniform loop
        int jj[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) jj[u] = locate(B0 + 16 * 64 * u);
        u32x4 w[kU][NV];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int P = B0 + 16 * 64 * u + 16 * lane;
            const int j = jj[u];
            int t = H0 - (P - S.o[j]);
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                const int Lf = (int)S.len[f][j];
                const bool need = P < span && t < 16 && t + Lf > 0;
                w[u][f] = ld16u(need ? (uintptr_t)(S.delta[f][j] + (u64)(i64)P) : dummy);
                t += Lf + 4;
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int P = B0 + 16 * 64 * u + 16 * lane;
            if (P >= span) continue;
            const int j = jj[u];
            const int b = P - S.o[j];
            u32x4 r = {0, 0, 0, 0};
            if (b < H0) r = lds16u(S.hdr, (j + 1) * SLOT + b);
            int t = H0 - b;
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                const int Lf = (int)S.len[f][j];
                if (f > 0 && t > 0 && t < 20) {  // inner length prefix of field f at [t-4, t)
                    u32 tmp[4] = {r.x, r.y, r.z, r.w};
                    or_u32_at((u32)Lf, t - 4, tmp);
                    r = u32x4{tmp[0], tmp[1], tmp[2], tmp[3]};
                }
                if (t < 16 && t + Lf > 0) r |= w[u][f] & range_mask(masks, t, t + Lf);
                t += Lf + 4;
            }
            if (j + 1 < cnt) {
                const int nb = P - S.o[j + 1];
                if (nb > -16) r |= lds16u(S.hdr, (j + 2) * SLOT + nb);
            }
            const u32 rr[4] = {r.x, r.y, r.z, r.w};
            store_chunk(out_t, P, 0, span, rr);
        }
    }
}

template <int NF, int NV>
static void launch_layout(const EncodeParams& p, dim3 grid, dim3 block, hipStream_t stream) {
    // variants 2/4: that many steps' loads in flight per wave (measured no faster on MI355X: the
    // one-step loop already runs at ~92 % of a plain 350 MB copy, tools/ubench_copy.hip)
    switch (p.variant) {
        case 2: hipLaunchKernelGGL((encode_kernel<NF, NV, 2>), grid, block, 0, stream, p); break;
        case 4: hipLaunchKernelGGL((encode_kernel<NF, NV, 4>), grid, block, 0, stream, p); break;
        default: hipLaunchKernelGGL((encode_kernel<NF, NV, 0>), grid, block, 0, stream, p); break;
    }
}

hipError_t launch_encode(const EncodeParams& p, hipStream_t stream) {
    if (p.n == 0) return hipMemsetAsync(p.out_off, 0, sizeof(uint64_t), stream);
    const u64 tiles = (p.n + kWaveRecs - 1) / kWaveRecs;
    const dim3 grid((unsigned)((tiles + kWaves - 1) / kWaves));
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
