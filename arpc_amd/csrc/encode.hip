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
#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"
#include "pipe_words.hpp"

namespace symhip {

constexpr int kWaveRecs = 64;  // records per wave tile
constexpr int kWaves = 4;      // wave tiles per 256-thread workgroup
constexpr int kGroupShift = 4; // mixed batches: 2^kGroupShift tiles per size-pass group (1024 records)

// Header slot for H0 header bytes: a 16-byte window starting at any b < H0 stays in the slot,
// and one starting up to 15 bytes before a slot reads only the previous slot's zero tail.
constexpr int slot_bytes(int H0) { return ((H0 + 16) + 7) & ~7; }

// ---------------------------------------------------------------- mixed Get/Set batches: record sizes
// Record sizes depend on the type column, so record offsets are a scan.  One launch
// (encode_pipe_kernel) runs it the way the default decode does (decode_pipe.hip), with three roles
// by workgroup index, over epoch-tagged words in the ctx's flag buffer (pipe_words.hpp):
//   [0, P)     sizers: workgroup takes a group of kPipeGroup 64-record tiles, computes every tile's
//              byte total, publishes each tile's exclusive prefix inside the group (a "local" word)
//              and the group's total (an aggregate word); groups g, g + P, ...  Never wait.
//   P          scanner: chains the group aggregates into exclusive group prefix words.
//   P + 1 + t  encode tile t: its stream position = group prefix + local prefix, both loaded when
//              the tile starts (normally published long before).  A word still missing after
//              kFallbackTicks is resolved by the tile itself (look-back over the group words, the
//              local prefix recomputed), so progress never depends on residency.
// Layout (u64 words): aggregate[ngroups], prefix[ngroups], 32 words of scanner store sink, local[ntiles].
constexpr int kPipeGroup = 8;  // tiles per sizer group (512 records)
__host__ __device__ static inline u64 mixed_ntiles(u64 n) { return (n + 63) / 64; }
__host__ __device__ static inline u64 mixed_npgroups(u64 n) { return (mixed_ntiles(n) + kPipeGroup - 1) / kPipeGroup; }
struct PipeWords {
    u64 *aw, *pw, *lw;
    u64 ng, nt;
};
__device__ __forceinline__ PipeWords pipe_words(const EncodeParams& p) {
    PipeWords w;
    w.nt = mixed_ntiles(p.n);
    w.ng = mixed_npgroups(p.n);
    w.aw = (u64*)p.flags;
    w.pw = w.aw + w.ng;
    w.lw = w.pw + w.ng + 32;  // <= 2 ng + 32 + nt <= 4 nt + 32 words: within decode_pipe_flag_bytes(2, n)
    return w;
}

// Byte totals of 64-record tiles t[k] (< ntiles), whole wave, wave-uniform result: 22 + K bytes per
// record (kv.syn.go:74-132) plus 8 + V per SetRequest (:611-678); K from the key offsets at the
// tile's edges.  Every load of the R tiles is in flight before any is used.
template <int R>
__device__ __forceinline__ void mixed_tile_totals(const EncodeParams& p, const u64 (&t)[R], u64 (&agg)[R]) {
    const int lane = threadIdx.x & 63;
    const u64 n = p.n;
    uint8_t ty[R];
    u64 v0[R], v1[R], ke[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const u64 a = t[k] * 64, b = min(a + 64, n);
        const u64 r = min(a + lane, n - 1);
        ty[k] = p.type[r];
        v0[k] = p.offs[1][r];
        v1[k] = p.offs[1][r + 1];
        ke[k] = p.offs[0][lane == 0 ? a : b];  // lanes 0 and 1: the key offsets at the tile's edges
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const u64 a = t[k] * 64, b = min(a + 64, n);
        const u32 extra = a + lane < b && ty[k] != 0 ? (u32)(8 + (v1[k] - v0[k])) : 0u;  // < 2^32 (u32 lengths)
        const u64 sets = pipe::lane_u64_pub(wave_incl_scan_u32w_dpp(extra), 63);
        const u64 keys = pipe::lane_u64_pub(ke[k], 1) - pipe::lane_u64_pub(ke[k], 0);
        agg[k] = 22 * (b - a) + keys + sets;
    }
}

// Sizer role: one group per step (wave w sizes tiles 2w, 2w + 1 of it).
__device__ void mixed_sizer(const EncodeParams& p, const PipeWords& W, u64* s_tot) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (u64 g = blockIdx.x; g < W.ng; g += p.pipe_sizers) {
        const u64 tb = g * kPipeGroup + 2 * (u64)wave;
        u64 t[2], agg[2];
        t[0] = min(tb, W.nt - 1);
        t[1] = min(tb + 1, W.nt - 1);
        mixed_tile_totals<2>(p, t, agg);
        if (lane < 2) s_tot[2 * wave + lane] = tb + lane < W.nt ? agg[lane] : 0;
        __syncthreads();
        if (wave == 0 && lane < kPipeGroup) {
            u64 excl = 0, tot = 0;
#pragma unroll
            for (int k = 0; k < kPipeGroup; ++k) {
                const u64 x = s_tot[k];
                excl += k < lane ? x : 0;
                tot += x;
            }
            const u64 tile = g * kPipeGroup + lane;
            if (tile < W.nt) pipe::store_word(&W.lw[tile], pipe::make_word(p.epoch, pipe::kStAgg, excl));
            if (lane == 0) {
                pipe::store_word(&W.aw[g], pipe::make_word(p.epoch, pipe::kStAgg, tot));
                if (p.dbg) p.dbg[(W.nt + g) * 8 + 4] = pipe::now_ticks();  // tools/mixed_timeline.py
            }
        }
        __syncthreads();  // s_tot is rewritten for the next group
    }
}

// Byte total of tiles [t0, t1) (whole wave, wave-uniform; t1 - t0 <= kPipeGroup).
__device__ u64 mixed_range_total(const EncodeParams& p, u64 t0, u64 t1) {
    u64 sum = 0;
    for (u64 t = t0; t < t1; ++t) {
        const u64 tt[1] = {t};
        u64 a[1];
        mixed_tile_totals<1>(p, tt, a);
        sum += a[0];
    }
    return sum;
}

// The stream position of mixed tile `tile` (wave 0 of its workgroup).  wg / wl: its group's prefix
// word and its local word, as loaded when the tile started.
__device__ i64 mixed_tile_prefix(const EncodeParams& p, u64 tile, u64 wg, u64 wl) {
    const u32 ep = p.epoch;
    if (__builtin_amdgcn_readfirstlane(pipe::tagged(wg, ep) && pipe::tagged(wl, ep)))
        return uniform_i64((i64)((wg & pipe::kValMask) + (wl & pipe::kValMask)));
    const int lane = threadIdx.x & 63;
    const PipeWords W = pipe_words(p);
    const u64 g = tile / kPipeGroup;
    if (!p.pipe_lookback && lane == 0) {
        for (const u64 t0 = pipe::now_ticks(); !(pipe::tagged(wg, ep) && pipe::tagged(wl, ep)) &&
                                               pipe::now_ticks() - t0 <= pipe::kFallbackTicks;) {
            __builtin_amdgcn_s_sleep(2);
            if (!pipe::tagged(wg, ep)) wg = pipe::load_word(&W.pw[g]);
            if (!pipe::tagged(wl, ep)) wl = pipe::load_word(&W.lw[tile]);
        }
    }
    wg = pipe::lane_u64_pub(wg, 0);
    wl = pipe::lane_u64_pub(wl, 0);
    u64 gpre, lpre;
    if (pipe::tagged(wg, ep)) {
        gpre = wg & pipe::kValMask;
    } else {  // resolve the group prefix here (never waits) and publish it
        i64 pre[1];
        pipe::lookback_with<1>(W.aw, W.pw, W.ng, g, ep, pre, [&](u64 gi, u64 (&a)[1]) {
            a[0] = mixed_range_total(p, gi * kPipeGroup, min((gi + 1) * kPipeGroup, W.nt));
        });
        gpre = (u64)pre[0];
        if (lane == 0) pipe::store_word(&W.pw[g], pipe::make_word(ep, pipe::kStPre, gpre));
    }
    lpre = pipe::tagged(wl, ep) ? wl & pipe::kValMask : mixed_range_total(p, g * kPipeGroup, tile);
    return uniform_i64((i64)(gpre + lpre));
}

// A tile's stream span must stay below 2^31 (64 records; positions are 32-bit), and string
// fields are < 2^32 bytes (Symphony's u32 length prefix).
template <int NV, int SLOT, int TR = kWaveRecs>
struct EncWaveLds {
    char hdr[(TR + 1) * SLOT];  // slot 0 = zero pad, slot i+1 = record i
    int o[TR + 1];              // record start relative to the tile start; [cnt] = span
    u32 len[NV][TR];
    u64 delta[NV][TR];          // payload byte address = delta + chunk position
    uint8_t h0[TR];             // mixed batches: the record's bytes before field 0's payload
    i64 t0;                     // the tile's stream start
    int span, ok;               // its length; 0 if it is too long for 32-bit positions
    int safe;                   // no payload window of the tile reaches past a column end
    int safe_h[TR / kWaveRecs]; // per header wave (TR > 64)
    i64 end_h[TR / kWaveRecs];  // per header wave: the end of its last record
};

// MIXED: a kv batch of GetRequests (type 0: 22 + K bytes, kv.syn.go:74-132) and SetRequests (else:
// 30 + K + V bytes, :611-678); the layout constants below are the SetRequest's, and every per-record
// difference (header image, table, where the key payload starts, no value) is taken per record.
// WPT (waves per tile): 1 = each wave owns a tile; kWaves = the workgroup owns one tile, wave 0
// builds it and the waves take its output steps round-robin (4x shorter-lived workgroups, so a
// 2^20-record launch runs ~8 rounds of workgroups instead of ~2 and its tail is short).
// TR: records per tile (64, or 128 with whole-workgroup tiles: waves 0 and 1 build the headers of
// 64 records each, so a tile of short records -- mixed Get/Set batches -- moves about as many bytes
// as a 64-record tile of SetRequests).
// PIPE (mixed batches, workgroup tiles): the one-launch size scan above -- blocks [0, P) are sizers,
// block P the scanner, block P + 1 + t encodes tile t (P = p.pipe_sizers; no sizers or scanner when
// p.pipe_lookback).  SSK: the scanner's tiles per thread per step.

// The prefetching encode (PF): one tile's input rows staged in LDS by global_load_lds while the
// previous tile is copied -- offsets [rb, rb + 64] of every string column (as dwords: three
// 64-lane dword loads, 130 dwords used), the type bytes (mixed batches), the int32 fields.
template <int NF, int NV>
struct alignas(16) EncStage {
    u32 offs[NV][3 * 64];
    u32 type[64];  // a byte load lands in its lane's dword (LDS-DMA writes base + 4 * lane below dword size)
    int32_t fixed[NF > 0 ? NF : 1][64];
};
template <int NF, int NV>
__device__ __forceinline__ u64 stage_off(const EncStage<NF, NV>* s, int f, u64 i) {
    return ((const u64*)s->offs[f])[i];
}
#define SYMHIP_LDS(ptr) ((__attribute__((address_space(3))) void*)(ptr))
// Whole wave: issue the loads of tile rows [rb, rb + 64) into s (they land asynchronously; wait
// with s_waitcnt vmcnt(0) before reading).  Source addresses are clamped into the columns.
template <int NF, int NV, bool MIXED>
__device__ __forceinline__ void enc_stage_issue(const EncodeParams& p, u64 rb, EncStage<NF, NV>& s, int lane) {
    const u64 n = p.n;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u32* src = (const u32*)p.offs[f];
#pragma unroll
        for (int k = 0; k < 3; ++k)
            __builtin_amdgcn_global_load_lds((const void*)(src + min(2 * rb + (u64)(64 * k + lane), 2 * n + 1)),
                                             SYMHIP_LDS(&s.offs[f][64 * k]), 4, 0, 0);
    }
    const u64 r = min(rb + (u64)lane, n - 1);
    if constexpr (MIXED) __builtin_amdgcn_global_load_lds((const void*)(p.type + r), SYMHIP_LDS(s.type), 1, 0, 0);
#pragma unroll
    for (int f = 0; f < NF; ++f)
        __builtin_amdgcn_global_load_lds((const void*)(p.fixed[f] + r), SYMHIP_LDS(s.fixed[f]), 4, 0, 0);
}

// Phase 1 of a tile (header waves; every wave calls it when HW > 1, for its barriers): per-record
// offsets and header image into S.  stg: the staged rows (PF) or null (read from HBM); wg_in /
// wl_in: the PIPE prefix words loaded with the staged rows (PF).

#define OFF(f, r) (PF ? stage_off(stg, (f), (r) - rb) : p.offs[(f)][(r)])
#define TYP(r) (PF ? (uint8_t)stg->type[(r) - rb] : p.type[(r)])
#define FIX(f, r) (PF ? stg->fixed[(f)][(r) - rb] : p.fixed[(f)][(r)])
template <int NF, int NV, bool MIXED, int WPT, bool DIAG, int TR, bool PIPE, bool PF>
__device__ __forceinline__ void enc_phase1(const EncodeParams& p, EncWaveLds<NV, slot_bytes(14 + 4 * (NF + NV) + 4), TR>& S,
                                           u64 r0, int cnt, int lane, int wave, u64* stamp,
                                           const EncStage<NF, NV>* stg, u64 wg_in, u64 wl_in) {
    constexpr int HW = TR / kWaveRecs;  // waves that build headers
    constexpr int NT = NF + NV;
    constexpr int H0 = 14 + 4 * NT + 4;        // bytes before field 0's payload (the largest, in mixed batches)
    constexpr i64 OVH = 14 + 4 * NT + 4 * NV;  // fixed bytes per record
    constexpr int SLOT = slot_bytes(H0);
    (void)OVH;
    // ---------------- phase 1: per-record offsets and header image ----------------
    // header wave h (h < HW) takes the tile's records [64 h, 64 h + 64): record rec = 64 h + lane
    const int hw = WPT == 1 ? 0 : wave;
    const u64 rb = r0 + (u64)hw * kWaveRecs;   // the header wave's first record
    const int hcnt = (int)min((u64)kWaveRecs, rb < p.n ? p.n - rb : (u64)0);
    const int rec = hw * kWaveRecs + lane;
    const bool hdr_wave = (WPT == 1 || wave < HW) && hcnt > 0;
    // A payload window reads up to 15 bytes beyond its field; that stays inside the column
    // unless the tile's fields sit within 16 bytes of the column's ends (batch edges).  Scalar
    // loads, issued with the per-record ones.
    bool part_safe = true;
    i64 o = 0, size = 0;
    u64 L[NV], lo[NV];  // the record's field lengths and first payload offsets (kept: a re-read after
                        // the out_off stores or the prefix-word polls is another trip to memory)
#pragma unroll
    for (int f = 0; f < NV; ++f) L[f] = lo[f] = 0;
    bool isset = true;  // mixed batches: SetRequest (else GetRequest)
    if (hdr_wave) {
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 c0 = p.offs[f][0], c1 = p.offs[f][p.n];
            const u64 t0 = OFF(f, rb), t1 = OFF(f, rb + hcnt);
            part_safe = part_safe && t0 >= c0 + 16 && t1 + 16 <= c1;
        }
        if constexpr (MIXED) {
            // sizes depend on the type: the size scan's prefix of this 64-record part plus a wave scan
            u64 wg = 0, wl = 0;  // PIPE: the prefix words, loaded first so their round trip overlaps the size loads
            if constexpr (PIPE && PF) {  // loaded with the staged rows
                wg = wg_in;
                wl = wl_in;
            } else if constexpr (PIPE) {
                const PipeWords W = pipe_words(p);
                wg = pipe::load_word(&W.pw[rb / kWaveRecs / kPipeGroup]);
                wl = pipe::load_word(&W.lw[rb / kWaveRecs]);
            }
            if (lane < hcnt) {
                const u64 r = rb + lane;
                isset = TYP(r) != 0;
                lo[0] = OFF(0, r);
                L[0] = OFF(0, r + 1) - lo[0];
                // the value offsets are loaded whatever the type (a select, not a branch): behind a
                // test of the type byte they would wait for its load, a second round trip per tile
                lo[1] = OFF(1, r);
                const u64 l1 = OFF(1, r + 1) - lo[1];
                L[1] = isset ? l1 : 0;
                size = (i64)(22 + L[0] + (isset ? 8 + L[1] : 0));
            }
            const u64 part = rb / kWaveRecs;  // the size scan's 64-record tiles
            const u64 incl = wave_incl_scan_u64((u64)size, lane);
            i64 tp;
            if constexpr (PIPE) {
                tp = mixed_tile_prefix(p, part, wg, wl);
                if (DIAG && lane == 0) stamp[7] = __builtin_amdgcn_s_memrealtime();
            } else {
                tp = uniform_i64((i64)(p.group_pre[part >> kGroupShift] + p.tile_loc[part]));
            }
            o = tp + (i64)(incl - (u64)size);
            if (lane < hcnt) {
                const u64 r = rb + lane;
#pragma unroll
                for (int f = 0; f < NV; ++f) S.len[f][rec] = (u32)L[f];
                p.out_off[r] = p.out_base + (u64)o;
                if (r == p.n - 1) p.out_off[p.n] = p.out_base + (u64)(o + size);
            }
        } else if (lane < hcnt) {
            const u64 r = rb + lane;
            o = (i64)r * OVH;
            size = OVH;
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                lo[f] = OFF(f, r);
                L[f] = OFF(f, r + 1) - lo[f];
                o += (i64)(lo[f] - p.offs[f][0]);
                size += (i64)L[f];
                S.len[f][rec] = (u32)L[f];
            }
            p.out_off[r] = p.out_base + (u64)o;
            if (r == p.n - 1) p.out_off[p.n] = p.out_base + (u64)(o + size);
        }
        if constexpr (HW > 1) {  // the parts meet in LDS: tile start, part ends, edge checks
            const i64 t0 = uniform_i64((i64)__shfl((long long)o, 0, 64));
            const i64 t1 = uniform_i64((i64)__shfl((long long)(o + size), hcnt - 1, 64));
            if (lane == 0) {
                if (hw == 0) S.t0 = t0;
                S.end_h[hw] = t1;
                S.safe_h[hw] = part_safe;
            }
        }
    }
    if constexpr (HW > 1) {
        __syncthreads();
        if (hdr_wave && lane == 0 && rb + hcnt == min(r0 + (u64)TR, p.n)) {  // the header wave of the tile's last part
            const i64 t0 = S.t0, t1 = S.end_h[hw];
            bool safe = true;
            for (int h = 0; h <= hw; ++h) safe = safe && S.safe_h[h] != 0;
            const bool ok = t1 - t0 < (i64)1 << 31;
            S.span = (int)(t1 - t0);
            S.ok = ok;
            S.safe = safe;
            if (!ok) atomicOr(p.err, kErrTooLarge);
        }
        __syncthreads();
    }
    if (hdr_wave) {
        // wave-uniform: readfirstlane keeps them (and the phase-2 loop bounds) in SGPRs
        i64 T0, T1;
        bool ok;
        if constexpr (HW > 1) {
            T0 = uniform_i64(S.t0);
            T1 = T0 + __builtin_amdgcn_readfirstlane(S.span);
            ok = S.ok != 0;
        } else {
            T0 = uniform_i64((i64)__shfl((long long)o, 0, 64));
            T1 = uniform_i64((i64)__shfl((long long)(o + size), hcnt - 1, 64));
            ok = T1 - T0 < (i64)1 << 31;  // positions are 32-bit inside a tile
            if (lane == 0) {
                S.t0 = T0;
                S.span = (int)(T1 - T0);
                S.ok = ok;
                S.safe = part_safe;
                if (!ok) atomicOr(p.err, kErrTooLarge);
            }
        }
        if (ok && lane < hcnt) {
            const u64 r = rb + lane;
            const int orel = (int)(o - T0);
            S.o[rec] = orel;
            if (rec == cnt - 1) S.o[cnt] = (int)(T1 - T0);
            const int h0 = MIXED && !isset ? 22 : H0;
            int ps = h0;
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                S.delta[f][rec] = (u64)(uintptr_t)(p.bytes[f] + lo[f]) - (u64)(i64)(orel + ps);
                ps += (int)L[f] + 4;
            }
            // header image: [0]=1 | [1:5]=13 | [5:9]=sid | [9:13]=mid | [13]=1 | table | len(field 0)
            u32 h[SLOT / 4 + 1];
#pragma unroll
            for (int k = 0; k < SLOT / 4 + 1; ++k) h[k] = 0;
            img_put_u8<0>(h, 1);
            img_put_u32<1>(h, 13);
            img_put_u32<5>(h, p.service_id);
            img_put_u32<9>(h, MIXED && !isset ? p.method_get : p.method_id);
            img_put_u8<13>(h, 1);
            if constexpr (NF > 0) img_put_u32<14>(h, (u32)FIX(0, r));
            if constexpr (NF > 1) img_put_u32<18>(h, (u32)FIX(1, r));
            // private-table entries: offset of the field's length prefix relative to privateStart
            // (13), truncated to u32 (kv.syn.go:664, :671).
            if (MIXED && !isset) {  // GetRequest{Key} (kv.syn.go:119-127)
                img_put_u32<14>(h, 5u);
                img_put_u32<18>(h, (u32)L[0]);
            } else {
                img_put_u32<14 + 4 * NF>(h, (u32)(H0 - 4 - 13));
                if constexpr (NV > 1) img_put_u32<18 + 4 * NF>(h, (u32)(H0 + L[0] + 4 - 4 - 13));
                img_put_u32<H0 - 4>(h, (u32)L[0]);
            }
            if constexpr (MIXED) S.h0[rec] = (uint8_t)h0;
            uint2* slot = (uint2*)&S.hdr[(rec + 1) * SLOT];
#pragma unroll
            for (int k = 0; k < SLOT / 8; ++k) slot[k] = make_uint2(h[2 * k], h[2 * k + 1]);
        }
        if (hw == 0 && lane < SLOT / 4) ((u32*)S.hdr)[lane] = 0;
    }
}
#undef OFF
#undef TYP
#undef FIX

// Phase 2 of a tile: natural-order output chunks.  OW output waves take the steps round-robin;
// this one is number ow.
template <int NF, int NV, int kVariant, bool MIXED, int WPT, bool DIAG, int TR, int OW>
__device__ __forceinline__ void enc_phase2(const EncodeParams& p, EncWaveLds<NV, slot_bytes(14 + 4 * (NF + NV) + 4), TR>& S,
                                           int cnt, int lane, int wave, int ow, uint8_t* const flg, const MaskTable& masks,
                                           u64* stamp) {
    constexpr int HW = TR / kWaveRecs;  // waves that build headers
    constexpr int NT = NF + NV;
    constexpr int H0 = 14 + 4 * NT + 4;        // bytes before field 0's payload (the largest, in mixed batches)
    constexpr i64 OVH = 14 + 4 * NT + 4 * NV;  // fixed bytes per record
    constexpr int SLOT = slot_bytes(H0);
    (void)OVH;
    // ---------------- phase 2: natural-order output chunks ----------------
    const i64 T0 = uniform_i64(S.t0);
    const int span = __builtin_amdgcn_readfirstlane(S.span);
    const bool nt = span <= kNtSpan;  // (st16)
    const i64 mis = (i64)((uintptr_t)p.out & 15);
    const int first = (int)(((T0 + mis) & ~(i64)15) - mis - T0);  // in (-16, 0]
    uint8_t* const out_t = p.out + T0;
    const uintptr_t dummy = (uintptr_t)p.out & ~(uintptr_t)15;  // readable; its bytes get masked off
    const bool tile_safe = S.safe != 0;
    const i64 my_o = lane < cnt ? (i64)S.o[lane] : ((i64)1 << 40);  // record-role registers
    const i64 my_o2 = HW > 1 && 64 + lane < cnt ? (i64)S.o[64 + (HW > 1 ? lane : 0)] : ((i64)1 << 40);

    // Chunk -> record without searching: records are >= 22 bytes, so at most one record starts
    // inside any 16-byte chunk.  Record k first owns chunk ceil((o_k - B)/16) of this step; a
    // ballot of those marks plus mbcnt gives every lane its record.
    u64 before2 = 0;
    auto locate = [&](int B) -> int {
        const i64 ck = (my_o - B + 15) >> 4;
        const u64 before = __ballot(ck <= 0);
        if (ck >= 1 && ck <= 63) flg[ck] = 1;
        if constexpr (HW > 1) {  // the tile's second 64 records
            const i64 ck2 = (my_o2 - B + 15) >> 4;
            before2 = __ballot(ck2 <= 0);
            if (ck2 >= 1 && ck2 <= 63) flg[ck2] = 1;
        }
        wave_sync();
        const bool mine = flg[lane] != 0;
        const u64 m = __ballot(mine);
        if (mine) flg[lane] = 0;  // clean for the next step (each lane its own byte)
        const int below = (int)__builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
        // (int) casts matter: __popcll is unsigned and max(unsigned, int) picks the double overload
        const int counted = (int)__popcll(before) + (HW > 1 ? (int)__popcll(before2) : 0) + below + (mine ? 1 : 0);
        return counted > 0 ? counted - 1 : 0;  // 0 only for the chunk straddling the tile start
    };

    // fetch: the chunk's payload windows (loads only); assemble: header | payloads | prefixes ->
    // one store.  Split so a pipelined loop can issue step s+1's loads before step s's store.
    auto fetch = [&](int P, int j, bool careful, u32x4 (&w)[NV]) {
        const int b = P - S.o[j];  // chunk start relative to record j (> -16)
        int t = (MIXED ? (int)S.h0[j] : H0) - b;  // chunk offset where field 0's payload starts
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const int Lf = (int)S.len[f][j];
            const uintptr_t X = (uintptr_t)(S.delta[f][j] + (u64)(i64)P);
            bool fast = P < span && t < 16 && t + Lf > 0 && (!MIXED || Lf > 0);  // a GetRequest has no value
            if (careful) {  // the 16-byte window must lie inside the column's 16-byte-rounded extent
                const uintptr_t c0 = (uintptr_t)(p.bytes[f] + p.offs[f][0]) & ~(uintptr_t)15;
                const uintptr_t c1 = ((uintptr_t)(p.bytes[f] + p.offs[f][p.n]) + 15) & ~(uintptr_t)15;
                fast = fast && X >= c0 && X + 16 <= c1;
            }
            w[f] = ld16u(fast ? X : dummy);  // unconditional: the loads issue together
            t += Lf + 4;
        }
    };
    auto assemble = [&](int P, int j, bool careful, const u32x4 (&w)[NV]) {
        const int b = P - S.o[j];
        const int h0j = MIXED ? (int)S.h0[j] : H0;
        u32x4 r = {0, 0, 0, 0};
        if (b < H0) r = lds16u(S.hdr, (j + 1) * SLOT + b);  // a GetRequest's slot is zero past its 22 bytes
        int t = h0j - b;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const int Lf = (int)S.len[f][j];
            if (f > 0 && t > 0 && t < 20) {  // inner length prefix of field f at [t-4, t)
                u32 tmp[4] = {r.x, r.y, r.z, r.w};
                or_u32_at((u32)Lf, t - 4, tmp);
                r = u32x4{tmp[0], tmp[1], tmp[2], tmp[3]};
            }
            if (!careful) {
                // unconditional use of the load (the mask is zero where the field is absent): a use
                // inside a skippable branch would leave the load pending on that path, and the
                // pipelined loop would wait for it at the loop head
                r |= w[f] & range_mask(masks, t, t + Lf);
            } else if (t < 16 && t + Lf > 0 && (!MIXED || Lf > 0)) {
                u32x4 v = w[f];
                {  // batch edges: windows reaching outside the column are read blockwise
                    const uintptr_t X = (uintptr_t)(S.delta[f][j] + (u64)(i64)P);
                    const uintptr_t c0 = (uintptr_t)(p.bytes[f] + p.offs[f][0]) & ~(uintptr_t)15;
                    const uintptr_t c1 = ((uintptr_t)(p.bytes[f] + p.offs[f][p.n]) + 15) & ~(uintptr_t)15;
                    if (!(X >= c0 && X + 16 <= c1)) {  // aligned blocks holding valid bytes only
                        u32 tmp[4] = {0, 0, 0, 0};
                        or_window_global(X, max(t, 0), min(t + Lf, 16), tmp);
                        v = u32x4{tmp[0], tmp[1], tmp[2], tmp[3]};
                    }
                }
                r |= v & range_mask(masks, t, t + Lf);
            }
            t += Lf + 4;
        }
        if (j + 1 < cnt) {  // the next record's header may start inside this chunk
            const int nb = P - S.o[j + 1];
            if (nb > -16) r |= lds16u(S.hdr, (j + 2) * SLOT + nb);
        }
        const u32 rr[4] = {r.x, r.y, r.z, r.w};
        store_chunk(out_t, P, 0, span, rr, nt);
    };
    auto chunk = [&](int P, int j, bool careful) {
        u32x4 w[NV];
        fetch(P, j, careful, w);
        assemble(P, j, careful, w);
    };

    if constexpr (kVariant == 1) {  // pipelined: step s+1's loads are in flight across step s's store
        if (!tile_safe) {
            for (int B = first + 16 * 64 * ow; B < span; B += 16 * 64 * OW) {
                const int j = locate(B);
                const int P = B + 16 * lane;
                if (P < span) chunk(P, j, true);
            }
            return;
        }
        // Straight-line software pipeline over the first kPipe steps (ping-pong registers): step
        // s+1's loads are issued before step s is assembled and stored.  Every path that fetches
        // a register set also consumes it and no value of a pending load reaches a join or a loop
        // head (the compiler would copy it there, waiting for every load in flight); steps past
        // kPipe run in a plain loop (the last pipelined fetch is then simply not used).
        constexpr int kStep = 16 * 64 * OW, kPipe = 8;
        int B = first + 16 * 64 * ow;  // the next step to store
        if (B < span) {
            u32x4 wa[NV], wb[NV];
            int ja = locate(B);
            fetch(B + 16 * lane, ja, false, wa);
#pragma unroll
            for (int st = 0; st < kPipe; st += 2) {
                if (B + kStep >= span) {
                    assemble(B + 16 * lane, ja, false, wa);  // lanes past the span store nothing
                    B = span;
                    break;
                }
                const int jb = locate(B + kStep);
                fetch(B + kStep + 16 * lane, jb, false, wb);
                assemble(B + 16 * lane, ja, false, wa);
                B += kStep;
                if (B + kStep >= span) {
                    assemble(B + 16 * lane, jb, false, wb);
                    B = span;
                    break;
                }
                ja = locate(B + kStep);
                fetch(B + kStep + 16 * lane, ja, false, wa);
                assemble(B + 16 * lane, jb, false, wb);
                B += kStep;
            }
        }
        for (; B < span; B += kStep) {  // wave-uniform loop
            const int j = locate(B);
            if (B + 16 * lane < span) chunk(B + 16 * lane, j, false);
        }
        if (DIAG && lane == 0) stamp[2 + (WPT == 1 ? 0 : wave)] = __builtin_amdgcn_s_memrealtime();
        return;
    }
    if constexpr (kVariant == 0) {
        for (int B = first + 16 * 64 * ow; B < span; B += 16 * 64 * OW) {  // wave-uniform loop
            const int j = locate(B);
            const int P = B + 16 * lane;
            if (P < span) chunk(P, j, !tile_safe);
        }
        if (DIAG && lane == 0) stamp[2 + (WPT == 1 ? 0 : wave)] = __builtin_amdgcn_s_memrealtime();
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
            store_chunk(out_t, P, 0, span, rr, nt);
        }
    }
}

// A real call from the persistent loop: inlined into the loop, the loop-invariant parts of the
// unrolled copy steps are hoisted out of it and held in registers (114 VGPRs instead of 54).
template <int NF, int NV, int kVariant, bool MIXED, int WPT, bool DIAG, int TR, int OW>
__device__ __attribute__((noinline)) void enc_phase2_call(const EncodeParams& p, EncWaveLds<NV, slot_bytes(14 + 4 * (NF + NV) + 4), TR>& S,
                                                          int cnt, int lane, int wave, int ow, uint8_t* const flg,
                                                          const MaskTable& masks, u64* stamp) {
    enc_phase2<NF, NV, kVariant, MIXED, WPT, DIAG, TR, OW>(p, S, cnt, lane, wave, ow, flg, masks, stamp);
}

template <int NF, int NV, int kVariant, bool MIXED = false, int WPT = 1, bool DIAG = false, int TR = kWaveRecs,
          bool PIPE = false, int SSK = 8, bool PF = false>
__device__ __forceinline__ void encode_body(const EncodeParams& p) {
    static_assert(!PF || (WPT == kWaves && TR == kWaveRecs && kVariant == 1), "the prefetching encode takes 64-record workgroup tiles");
    static_assert(!PIPE || (MIXED && WPT == kWaves && (TR == kWaveRecs || TR == 2 * kWaveRecs)),
                  "the pipelined size scan is for mixed 64- or 128-record workgroup tiles");
    static_assert(!MIXED || (NF == 0 && NV == 2 && kVariant <= 1), "mixed batches are kv Get/Set");
    static_assert(WPT == 1 || (WPT == kWaves && kVariant <= 1), "whole-workgroup tiles take one step per wave");
    static_assert(TR == kWaveRecs || (TR == 2 * kWaveRecs && WPT == kWaves), "128-record tiles are workgroup tiles");
    constexpr int NT = NF + NV;
    constexpr int H0 = 14 + 4 * NT + 4;        // bytes before field 0's payload (the largest, in mixed batches)
    constexpr i64 OVH = 14 + 4 * NT + 4 * NV;  // fixed bytes per record
    constexpr int SLOT = slot_bytes(H0);
    static_assert(SLOT - 16 >= H0 && OVH >= 16, "layout assumptions");

    __shared__ EncWaveLds<NV, SLOT, TR> lds_all[PF ? 2 : kWaves / WPT];
    __shared__ EncStage<NF, NV> stg_all[PF ? 2 : 1];
    __shared__ uint8_t flags_all[kWaves][64];  // record-start marks of one phase-2 step, per wave
    __shared__ MaskTable masks;
    u64 blk = blockIdx.x;
    if constexpr (PIPE) {
        if (!p.pipe_lookback) {
            const PipeWords W = pipe_words(p);
            if (blockIdx.x < p.pipe_sizers) {
                __shared__ u64 s_tot[kPipeGroup];
                mixed_sizer(p, W, s_tot);
                return;
            }
            if (blockIdx.x == p.pipe_sizers) {
                __shared__ pipe::ScanLds SL;
                pipe::scanner<1, SSK>(W.aw, W.pw, W.ng, p.epoch, SL, DIAG ? p.dbg + W.nt * 8 : nullptr);  // 256 * SSK groups per step
                return;
            }
            blk = blockIdx.x - p.pipe_sizers - 1;
        }
    }
    mask_table_init(masks, threadIdx.x);
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint8_t* const flg = flags_all[wave];
    flg[lane] = 0;
    if constexpr (!PF) {
        (void)stg_all;
        EncWaveLds<NV, SLOT, TR>& S = lds_all[WPT == 1 ? wave : 0];
        const u64 r0 = (WPT == 1 ? blk * kWaves + wave : blk) * TR;
        if (r0 >= p.n) return;  // wave-uniform (workgroup-uniform when WPT > 1)
        const int cnt = (int)min((u64)TR, p.n - r0);
        u64* const stamp = DIAG ? p.dbg + (r0 / kWaveRecs) * 8 : nullptr;  // tools/enc_timeline.py
        if (DIAG && lane == 0 && (WPT == 1 || wave == 0)) {
            stamp[0] = __builtin_amdgcn_s_memrealtime();
            stamp[6] = blockIdx.x;
        }
        enc_phase1<NF, NV, MIXED, WPT, DIAG, TR, PIPE, false>(p, S, r0, cnt, lane, wave, stamp, nullptr, 0, 0);
        if constexpr (WPT == 1) wave_sync();
        else __syncthreads();
        if (!S.ok) return;  // uniform
        if (DIAG && lane == 0 && (WPT == 1 || wave == 0)) stamp[1] = __builtin_amdgcn_s_memrealtime();
        enc_phase2<NF, NV, kVariant, MIXED, WPT, DIAG, TR, WPT>(p, S, cnt, lane, wave, WPT == 1 ? 0 : wave, flg, masks, stamp);
    } else {
        // Persistent workgroups, wave-specialised: wave 0 builds tile t (phase 1, from rows staged
        // one tile ahead) while waves 1-3 copy tile t - G (phase 2); one barrier per tile hands S[b]
        // over.  S and the stage are double-buffered, so phase 1 of tile t + G may overwrite S[b]
        // only after that barrier -- by which waves 1-3 have finished tile t - G.
        const u64 nt = (p.n + kWaveRecs - 1) / kWaveRecs;
        const u64 G = gridDim.x - (PIPE && !p.pipe_lookback ? p.pipe_sizers + 1 : 0);
        if (wave == 0) {
            u64 wg = 0, wl = 0;
            const auto issue = [&](u64 t, int b) {
                enc_stage_issue<NF, NV, MIXED>(p, t * kWaveRecs, stg_all[b], lane);
                if constexpr (PIPE) {
                    const PipeWords W = pipe_words(p);
                    wg = pipe::load_word(&W.pw[t / kPipeGroup]);
                    wl = pipe::load_word(&W.lw[t]);
                }
            };
            if (blk < nt) issue(blk, 0);
            int b = 0;
#pragma unroll 1
            for (u64 t = blk; t < nt; t += G, b ^= 1) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this tile's rows and words have landed
                const u64 cg = wg, cl = wl;
                if (t + G < nt) issue(t + G, b ^ 1);  // in flight while this tile is built and copied
                const u64 r0 = t * kWaveRecs;
                const int cnt = (int)min((u64)kWaveRecs, p.n - r0);
                u64* const stamp = DIAG ? p.dbg + t * 8 : nullptr;
                if (DIAG && lane == 0) {
                    stamp[0] = __builtin_amdgcn_s_memrealtime();
                    stamp[6] = blockIdx.x;
                }
                int ln = lane;  // opaque per iteration (see the copier loop below)
                asm volatile("" : "+v"(ln));
                enc_phase1<NF, NV, MIXED, WPT, DIAG, TR, PIPE, true>(p, lds_all[b], r0, cnt, ln, 0, stamp, &stg_all[b], cg, cl);
                if (DIAG && lane == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();
                pipe::lds_barrier();  // S[b] built (LDS writes done; stores and the prefetch stay in flight)
            }
        } else {
            int b = 0;
#pragma unroll 1
            for (u64 t = blk; t < nt; t += G, b ^= 1) {
                pipe::lds_barrier();
                EncWaveLds<NV, SLOT, TR>& S = lds_all[b];
                if (!S.ok) continue;  // uniform
                const int cnt = (int)min((u64)kWaveRecs, p.n - t * kWaveRecs);
                u64* const stamp = DIAG ? p.dbg + t * 8 : nullptr;
                int ln = lane;  // opaque per iteration: keeps the lane-derived constants of the copy steps
                asm volatile("" : "+v"(ln));  // from being hoisted out of the loop (~32 VGPRs held across it)
                enc_phase2<NF, NV, kVariant, MIXED, WPT, DIAG, TR, kWaves - 1>(p, S, cnt, ln, wave, wave - 1, flg, masks, stamp);
            }
        }
    }
}


template <int NF, int NV, int kVariant, bool MIXED = false, int WPT = 1, bool DIAG = false, int TR = kWaveRecs>
__global__ __launch_bounds__(256) void encode_kernel(EncodeParams p) {
    encode_body<NF, NV, kVariant, MIXED, WPT, DIAG, TR>(p);
}

// The one-launch mixed encode: its role code (sizer, scanner, look-back) would otherwise lift the
// kernel past 64 VGPRs, i.e. from 8 to 6 waves per SIMD, and the encode tiles are latency-bound
// (tools/mixed_timeline.py: resident tiles x lifetime sets the rate).
template <bool DIAG = false, int SSK = 1, int TR = kWaveRecs>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void encode_pipe_kernel(EncodeParams p) {
    encode_body<0, 2, 1, true, kWaves, DIAG, TR, true, SSK>(p);
}

// The prefetching encode (tuning variants 50-53): persistent wave-specialised workgroups, see
// encode_body PF.  Measured slower than the default (config 2: 174 vs 154 us, config 3: 377 vs
// 360 us, mixed: 119 vs 111 us; profiles/r03_pf_*): phase 1 drops from ~6 to ~2 us per tile, but
// the copier loop holds 82-89 VGPRs (occupancy 5-6 instead of 8) and each copier waits for its
// stores at every tile boundary (vmcnt counts stores; the next tile's loads are issued after them),
// where a retiring workgroup leaves its stores draining behind it.
template <int NF, int NV, bool MIXED, bool PIPE, bool DIAG = false>
__global__ __launch_bounds__(256) void encode_pf_kernel(EncodeParams p) {
    encode_body<NF, NV, 1, MIXED, kWaves, DIAG, kWaveRecs, PIPE, 1, true>(p);
}

static int device_cus();
// Tile workgroups of a persistent launch: all of them resident at once, next to `others` resident
// workgroups of the same launch (sizers, scanner).
template <int NF, int NV, bool MIXED, bool PIPE, bool DIAG>
static u64 pf_tile_groups(u64 ntiles, u64 others) {
    static int occ[16] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    int& o = occ[dev & 15];
    if (o == 0 && hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, encode_pf_kernel<NF, NV, MIXED, PIPE, DIAG>, 256, 0) != hipSuccess)
        o = 0;
    const u64 slots = (u64)device_cus() * (u64)max(o, 1);
    const u64 g = slots > others + 1 ? slots - others : 1;
    return min(g, ntiles);
}
template <int NF, int NV, bool MIXED, bool PIPE, bool DIAG = false>
static void launch_pf(EncodeParams p, hipStream_t stream) {
    const u64 nt = (p.n + kWaveRecs - 1) / kWaveRecs;
    const u64 others = PIPE && !p.pipe_lookback ? (u64)p.pipe_sizers + 1 : 0;
    const u64 g = pf_tile_groups<NF, NV, MIXED, PIPE, DIAG>(nt, others);
    hipLaunchKernelGGL((encode_pf_kernel<NF, NV, MIXED, PIPE, DIAG>), dim3((unsigned)(others + g)), dim3(256), 0, stream, p);
}

static dim3 encode_grid(u64 n, int wpt) {
    const u64 tiles = (n + kWaveRecs - 1) / kWaveRecs;
    return dim3((unsigned)(wpt == 1 ? (tiles + kWaves - 1) / kWaves : tiles));
}

template <int NF, int NV>
static void launch_layout(const EncodeParams& p, hipStream_t stream) {
    const dim3 block(64 * kWaves);
#ifdef SYMHIP_TUNING
    // variants 2/4: that many steps' loads in flight per wave (measured no faster on MI355X: the
    // one-step loop already runs at ~92 % of a plain 350 MB copy, tools/ubench_copy.hip);
    // 5: one tile per wave (the round-1 layout)
    switch (p.variant) {
        case 2: hipLaunchKernelGGL((encode_kernel<NF, NV, 2>), encode_grid(p.n, 1), block, 0, stream, p); return;
        case 4: hipLaunchKernelGGL((encode_kernel<NF, NV, 4>), encode_grid(p.n, 1), block, 0, stream, p); return;
        case 5: hipLaunchKernelGGL((encode_kernel<NF, NV, 0>), encode_grid(p.n, 1), block, 0, stream, p); return;
        // 6/7: per-tile timestamps into p.dbg (tools/enc_timeline.py), workgroup tiles / wave tiles
        case 6: hipLaunchKernelGGL((encode_kernel<NF, NV, 0, false, kWaves, true>), encode_grid(p.n, kWaves), block, 0, stream, p); return;
        case 7: hipLaunchKernelGGL((encode_kernel<NF, NV, 0, false, 1, true>), encode_grid(p.n, 1), block, 0, stream, p); return;
        // 8/9: pipelined steps, workgroup tiles / wave tiles; 10: 8 with timestamps
        case 8: hipLaunchKernelGGL((encode_kernel<NF, NV, 1, false, kWaves>), encode_grid(p.n, kWaves), block, 0, stream, p); return;
        case 9: hipLaunchKernelGGL((encode_kernel<NF, NV, 1, false, 1>), encode_grid(p.n, 1), block, 0, stream, p); return;
        case 10: hipLaunchKernelGGL((encode_kernel<NF, NV, 1, false, kWaves, true>), encode_grid(p.n, kWaves), block, 0, stream, p); return;
        // 21: 128-record workgroup tiles (two header waves)
        case 21: hipLaunchKernelGGL((encode_kernel<NF, NV, 1, false, kWaves, false, 2 * kWaveRecs>), dim3((unsigned)((p.n + 127) / 128)), block, 0, stream, p); return;
        // 50: the prefetching persistent encode; 53: with timestamps
        case 50: launch_pf<NF, NV, false, false>(p, stream); return;
        case 53: launch_pf<NF, NV, false, false, true>(p, stream); return;
        // 15: workgroup tiles, one step at a time (no software pipeline)
        case 15: hipLaunchKernelGGL((encode_kernel<NF, NV, 0, false, kWaves>), encode_grid(p.n, kWaves), block, 0, stream, p); return;
        default: break;
    }
#endif
    hipLaunchKernelGGL((encode_kernel<NF, NV, 1, false, kWaves>), encode_grid(p.n, kWaves), block, 0, stream, p);
}

hipError_t launch_encode(const EncodeParams& p, hipStream_t stream) {
    if (p.n == 0) return hipMemsetAsync(p.out_off, 0, sizeof(uint64_t), stream);
    if (p.lay.nfixed == 0 && p.lay.nvar == 1)
        launch_layout<0, 1>(p, stream);
    else if (p.lay.nfixed == 0 && p.lay.nvar == 2)
        launch_layout<0, 2>(p, stream);
    else if (p.lay.nfixed == 2 && p.lay.nvar == 2)
        launch_layout<2, 2>(p, stream);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// ---------------------------------------------------------------- mixed Get/Set batches
static int device_cus() {
    static int cus[16] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    int& ncu = cus[dev & 15];
    if (ncu == 0 && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 0;
    return ncu;
}

// SYM_ENCODE_THREE_KERNEL: the size scan as two launches before the encode (no inter-workgroup
// waiting at all).  The size pass reads the type bytes and the value offsets and writes, per 64-record
// tile, its exclusive size prefix inside its group of kGroupTiles tiles, and per group its total;
// one workgroup then scans the group totals.  The encode kernel starts tile t at
// group_pre[t >> kGroupShift] + tile_loc[t].
constexpr int kGroupTiles = 1 << kGroupShift;   // tiles per size-pass workgroup (1024 records)
constexpr int kTilesPerWave = kGroupTiles / 4;  // 4

struct MixedWs {
    u64* group_pre;
    u64* tile_loc;
    u64* group_tot;
};
__host__ __device__ static inline u64 mixed_ngroups(u64 n) { return (mixed_ntiles(n) + kGroupTiles - 1) / kGroupTiles; }
static MixedWs mixed_layout(void* ws, u64 n) {
    MixedWs w;
    w.group_pre = (u64*)ws;
    w.group_tot = w.group_pre + mixed_ngroups(n);
    w.tile_loc = w.group_tot + mixed_ngroups(n);
    return w;
}
size_t encode_mixed_ws_bytes(uint64_t n) { return (size_t)(2 * mixed_ngroups(n) + mixed_ntiles(n)) * 8; }

__global__ __launch_bounds__(256) void mixed_size_kernel(EncodeParams p, MixedWs w) {
    __shared__ u64 s_agg[kGroupTiles];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u64 n = p.n, ntiles = mixed_ntiles(n), g = blockIdx.x;
    const u64 t0 = g * kGroupTiles + (u64)wave * kTilesPerWave;  // this wave's first tile
    // every load of the wave's tiles in flight before any is used (clamped, unconditional); lane 0
    // also loads the key offsets at the tiles' edges
    uint8_t ty[kTilesPerWave];
    u64 v0[kTilesPerWave], v1[kTilesPerWave], ka[kTilesPerWave], kb[kTilesPerWave];
#pragma unroll
    for (int k = 0; k < kTilesPerWave; ++k) {
        const u64 a = min((t0 + k) * kWaveRecs, n), b = min(a + kWaveRecs, n);
        const u64 r = min(a + lane, n - 1);
        ty[k] = p.type[r];
        v0[k] = p.offs[1][r];
        v1[k] = p.offs[1][r + 1];
        ka[k] = p.offs[0][lane == 0 ? a : b];
        kb[k] = p.offs[0][b];
    }
#pragma unroll
    for (int k = 0; k < kTilesPerWave; ++k) {
        const u64 t = t0 + k, a = t * kWaveRecs, r = a + lane;
        const u32 extra = r < n && ty[k] != 0 ? (u32)(8 + (v1[k] - v0[k])) : 0u;  // < 2^32 (u32 lengths)
        const u64 inc = wave_incl_scan_u32w_dpp(extra);
        const u64 sum = (u64)(u32)__builtin_amdgcn_readlane((u32)inc, 63) | ((u64)(u32)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
        if (lane == 0)
            s_agg[wave * kTilesPerWave + k] = t < ntiles ? 22 * (min(a + kWaveRecs, n) - a) + (kb[k] - ka[k]) + sum : 0;
    }
    __syncthreads();
    if (wave == 0) {  // the group's tiles: exclusive prefixes inside the group, and its total
        const u64 v = lane < kGroupTiles ? s_agg[lane] : 0;
        const u64 inc = wave_incl_scan_u64(v, lane);
        const u64 t = g * kGroupTiles + lane;
        if (lane < kGroupTiles && t < ntiles) w.tile_loc[t] = inc - v;
        if (lane == 63) w.group_tot[g] = inc;
    }
}

// One workgroup: exclusive scan of the group totals (16 per thread per round).  A separate launch:
// the size pass's former "last workgroup scans" ticket made every workgroup do an acq_rel atomic on
// one word, and those serialised (30 us for 2^20 records).
__global__ __launch_bounds__(256) void mixed_group_scan_kernel(MixedWs w, u64 ng) {
    __shared__ u64 s_wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    u64 carry = 0;
    for (u64 base = 0; base < ng; base += 256 * 16) {
        u64 v[16], sum = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const u64 i = base + (u64)tid * 16 + k;
            v[k] = i < ng ? w.group_tot[i] : 0;
            sum += v[k];
        }
        const u64 inc = wave_incl_scan_u64(sum, lane);
        if (lane == 63) s_wsum[wave] = inc;
        __syncthreads();
        u64 wpre = 0, tot = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q < wave) wpre += s_wsum[q];
            tot += s_wsum[q];
        }
        __syncthreads();
        u64 run = carry + wpre + inc - sum;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const u64 i = base + (u64)tid * 16 + k;
            if (i < ng) w.group_pre[i] = run;
            run += v[k];
        }
        carry += tot;
    }
}

static void launch_encode_mixed_3(EncodeParams p, void* ws, hipStream_t stream) {
    const MixedWs w = mixed_layout(ws, p.n);
    hipLaunchKernelGGL(mixed_size_kernel, dim3((unsigned)mixed_ngroups(p.n)), dim3(256), 0, stream, p, w);
    hipLaunchKernelGGL(mixed_group_scan_kernel, dim3(1), dim3(256), 0, stream, w, mixed_ngroups(p.n));
    p.group_pre = w.group_pre;
    p.tile_loc = w.tile_loc;
#ifdef SYMHIP_TUNING
    switch (p.variant) {
        case 20:  // 128-record workgroup tiles
            hipLaunchKernelGGL((encode_kernel<0, 2, 1, true, kWaves, false, 2 * kWaveRecs>), dim3((unsigned)((p.n + 127) / 128)),
                               dim3(64 * kWaves), 0, stream, p);
            return;
        case 5: hipLaunchKernelGGL((encode_kernel<0, 2, 0, true>), encode_grid(p.n, 1), dim3(64 * kWaves), 0, stream, p); return;
        case 38: hipLaunchKernelGGL((encode_kernel<0, 2, 1, true, kWaves, true>), encode_grid(p.n, kWaves), dim3(64 * kWaves), 0, stream, p); return;  // + timestamps
        case 41: hipLaunchKernelGGL((encode_kernel<0, 2, 1, true, 1>), encode_grid(p.n, 1), dim3(64 * kWaves), 0, stream, p); return;  // wave tiles, pipelined steps
        case 15: hipLaunchKernelGGL((encode_kernel<0, 2, 0, true, kWaves>), encode_grid(p.n, kWaves), dim3(64 * kWaves), 0, stream, p); return;
        default: break;
    }
#endif
    hipLaunchKernelGGL((encode_kernel<0, 2, 1, true, kWaves>), encode_grid(p.n, kWaves), dim3(64 * kWaves), 0, stream, p);
}

hipError_t launch_encode_mixed(EncodeParams p, void* ws, hipStream_t stream) {
    if (p.n == 0) return hipMemsetAsync(p.out_off, 0, sizeof(uint64_t), stream);
    if (!p.type || p.lay.nfixed != 0 || p.lay.nvar != 2) return hipErrorInvalidValue;
    int impl = p.impl;
#ifdef SYMHIP_TUNING
    if (p.variant == 5 || p.variant == 15 || p.variant == 20 || p.variant == 38 || p.variant == 40 || p.variant == 41) impl = SYM_ENCODE_THREE_KERNEL;  // 40: its default kernel
#endif
    if (impl == SYM_ENCODE_THREE_KERNEL) {
        if (!ws) return hipErrorInvalidValue;
        launch_encode_mixed_3(p, ws, stream);
        return hipGetLastError();
    }
    if (!p.flags || p.epoch == 0) return hipErrorInvalidValue;
    const u64 nt = mixed_ntiles(p.n);
    const int ncu = device_cus();
    if (ncu <= 0) return hipErrorInvalidDevice;
    // sizers: two per CU (kPipeGroup tiles per workgroup step).  Round 5, tools/mixed_ab.py, 30
    // rounds: one per 2 CUs (round 4, variant 32) 102.7 us, one per CU (31) 101.2, two per CU 100.6;
    // the trace replay 563.0 / 561.4 / 560.4 us; four per CU (33) 99.9 vs 100.5 us, within noise
    u64 P = (u64)ncu * 2;
    p.pipe_lookback = impl == SYM_ENCODE_LOOKBACK;
#ifdef SYMHIP_TUNING
    if (p.variant == 30) P = (u64)ncu / 4;
    if (p.variant == 31) P = (u64)ncu;
    if (p.variant == 32) P = (u64)ncu / 2;
    if (p.variant == 33) P = (u64)ncu * 4;
#endif
    if (P > mixed_npgroups(p.n)) P = mixed_npgroups(p.n);
    p.pipe_sizers = (unsigned)P;
    const u64 grid = p.pipe_lookback ? nt : P + 1 + nt;
    if (grid > 0xFFFFFFFFull) return hipErrorInvalidValue;
#ifdef SYMHIP_TUNING
    if (p.variant == 25) {  // 128-record tiles (two header waves, each its 64-record part's prefix)
        const u64 nt2 = (p.n + 2 * kWaveRecs - 1) / (2 * kWaveRecs);
        hipLaunchKernelGGL((encode_pipe_kernel<false, 1, 2 * kWaveRecs>), dim3((unsigned)(p.pipe_lookback ? nt2 : P + 1 + nt2)),
                           dim3(64 * kWaves), 0, stream, p);
        return hipGetLastError();
    }
    if (p.variant == 51) {  // the prefetching persistent encode tiles
        launch_pf<0, 2, true, true>(p, stream);
        return hipGetLastError();
    }
    if (p.variant == 52) {  // the same with timestamps (tools/mixed_timeline.py --variant 52)
        if (!p.dbg) return hipErrorInvalidValue;
        launch_pf<0, 2, true, true, true>(p, stream);
        return hipGetLastError();
    }
    if (p.variant == 37) {  // per-tile timestamps (tools/mixed_timeline.py): p.dbg holds 16 u64 per tile
        if (!p.dbg) return hipErrorInvalidValue;
        hipLaunchKernelGGL((encode_pipe_kernel<true>), dim3((unsigned)grid), dim3(64 * kWaves), 0, stream, p);
        return hipGetLastError();
    }
    if (p.variant == 34 || p.variant == 35 || p.variant == 36) {  // scanner steps of 512 / 1024 / 2048 groups (default 256)
        if (p.variant == 34) hipLaunchKernelGGL((encode_pipe_kernel<false, 2>), dim3((unsigned)grid), dim3(64 * kWaves), 0, stream, p);
        if (p.variant == 35) hipLaunchKernelGGL((encode_pipe_kernel<false, 4>), dim3((unsigned)grid), dim3(64 * kWaves), 0, stream, p);
        if (p.variant == 36) hipLaunchKernelGGL((encode_pipe_kernel<false, 8>), dim3((unsigned)grid), dim3(64 * kWaves), 0, stream, p);
        return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL((encode_pipe_kernel<>), dim3((unsigned)grid),
                       dim3(64 * kWaves), 0, stream, p);
    return hipGetLastError();
}

}  // namespace symhip
