// decode_pipe.hip -- batched Symphony UnmarshalSymphony on gfx950: the default decode.
//
// Restates, for n records at once, the generated per-record unmarshaller into a fresh struct:
// benchmark/kv-store-symphony/symphony/kv.syn.go:680-745 (SetRequest; Get/Resp analogous),
// examples/echo_symphony/symphony/echo.syn.go:186-263 (int32 fields), from the generator's rules
// cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:622-694, :734-793.
//
// A string field's output position is the sum of all earlier lengths in its column, so decode is a
// scan.  Here it is ONE launch in which every stream byte is staged through LDS once, with three
// roles by workgroup index (lowest first, so producers are resident before their consumers):
//   [0, P)      parsers: a wave reads the headers of 64-record tiles (two 16-byte loads per record
//               into registers, global loads past that window), runs Go's checks for the field
//               lengths only, and publishes the tile's per-column aggregate word.  They never wait.
//               kv layouts (no int32 fields) by default parse SPECULATIVELY: the lengths a record
//               laid out as the generator writes it has, from its length alone and at most one
//               4-byte load (spec_flen) -- the parsers' header reads were ~10 % of the decode time --
//               and (round 6) that one load only once per tile, for the tile's first SetRequest
//               (tile-key speculation: the copier's stage is then the only read of a record's head).
//               Every copier checks them against Go's exact parse of its staged bytes; a second
//               launch (the gate) decodes the batch again exactly if any was wrong.
//   P           scanner: walks the tiles in order, 1024 per step, and publishes every tile's
//               exclusive prefix word up to the first tile whose aggregate is not yet published.
//   P + 1 + t   copier of tile t:
//                 1. stage: the tile's byte span -> LDS with aligned, coalesced 16-byte loads (up to
//                    kStage bytes; a longer span's tail is read from HBM at copy time);
//                 2. parse (wave 0, lane = record) from LDS: status byte, int32 fields, per-field
//                    (position, length), the tile scan (DPP); publishes its own aggregate too;
//                 3. waits for its prefix word (normally published long before), writes offsets;
//                 4. copy (all lanes): each field as a run of 16-byte chunks (the last one moved back
//                    to end at the field end): one byte-unaligned LDS read, one 16-byte store.
// Prefix words are 8-byte {epoch, status, value} words written and polled with agent-scope relaxed
// atomics -- the word is its own flag (MI355X_MICROARCH.md visibility, form "R2") -- tagged with the
// call's epoch so they never need clearing between calls.
//
// Progress does not depend on which workgroups are resident.  The fast path assumes the hardware's
// in-order dispatch (parsers and scanner resident before the copiers that wait on them); a copier
// whose prefix word has not appeared after kFallbackTicks resolves its prefix itself by a decoupled
// look-back that never waits: it walks back over earlier tiles' words, and a tile with no published
// aggregate is parsed from HBM on the spot (its aggregate then published for everyone).  The copier
// publishes the prefix it found, so later look-backs stop there.  kImplLookback forces this path
// (parsers and scanner exit at once) so the tests can exercise it.
//
// Mixed kv batches (p.type != null, sym_decode_kv_mixed): a record of type 0 is a GetRequest (one
// string field, kv.syn.go:134-185), any other a SetRequest (two, :680-745); column 1 is empty for
// GetRequests.
//
// Why this shape (measured on MI355X): a separate parse pass costs ~65 us of
// scattered header reads before any byte moves; an in-kernel decoupled look-back between copiers
// stalls on cross-XCD round trips (~2 us each) once ~1500 tiles are in flight; parsers that run
// ahead make the chain a single streaming scanner the copiers rarely wait on.
#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"
#include "pipe_words.hpp"

namespace symhip {

namespace pipe {

constexpr int kRecs = 64;       // records per tile
constexpr int kThreads = 256;   // 4 waves
constexpr int kStage = 22528;   // staged bytes per tile: a whole 64-record tile of 350-B records
constexpr int kU = 2;           // copy chunks per lane per step


__host__ __device__ inline u64 num_tiles(u64 n) { return (n + kRecs - 1) / kRecs; }

// Control words after the aggregate / prefix words and the scanner's 256-byte sink
// (decode_pipe_flag_bytes): [kCtrlMismatch] tagged with the call's epoch when a copier found a
// speculative length wrong; [kCtrlSpecErr] tagged when the speculative launch saw a capacity error
// (value: the kErr bits), merged into p.err by the gate or dropped with a re-decode.  Words of other
// calls (other tags, or another call's words where a larger batch put them) are ignored.
constexpr int kCtrlMismatch = 0;
constexpr int kCtrlSpecErr = 1;
constexpr int kCtrlTileMiss = 2;  // tile-key speculation: a record's own key length differed from its tile's
__device__ __forceinline__ u64* ctrl_words(u64* flags, int nv, u64 ntiles) { return flags + (size_t)2 * nv * ntiles + 32; }

template <int NV, int STG>
struct alignas(16) Lds {
    uint8_t stage[STG + 16];
    u64 src[NV][kRecs];      // field payload position (stream offset)
    int dst[NV][kRecs + 1];  // field start in the tile's column range; [cnt..] = aggregate
    int cs[kRecs + 1];       // record's first copy chunk (record-major chunk sequence)
    int nch0[kRecs];         // chunks of the record's first string field
    i64 pre[NV];             // tile prefix per column
    i64 lim[NV];             // bytes of the tile's column range that fit the output capacity
    int total;               // chunks in the tile (-1: tile skipped, error reported)
    u64 red[4];              // scanner: per-wave partial sums
    int first[4];            // scanner: per-wave first unpublished tile
};



// ---------------------------------------------------------------- parser role
// Step k covers tiles [k*4PR, (k+1)*4PR): wave (b, w) takes R consecutive tiles, lane = record; every
// load of the R records a lane handles is issued before any is used.  Field lengths follow the same
// Go checks as the copier's parse (kv.syn.go:681-745), so both publish identical aggregates.
// String fields of record r: NV, or 1 for a GetRequest of a mixed kv batch.
template <int NV, bool MIX>
__device__ __forceinline__ int rec_nvar(const DecodeParams& p, u64 r) {
    if constexpr (MIX) return p.type[r] != 0 ? NV : 1;
    else return NV;
}

// R tiles th[] by one wave (lane = record): the records' field lengths with Go's checks, then each
// tile's aggregate word per column.  Every load of the R records is issued before any is used.
template <int NF, int NV, bool MIX, int R, int WB>
__device__ __forceinline__ void parse_tiles(const DecodeParams& p, u64* aw, u64 ntiles, u32 epoch, const u64 (&th)[R]) {
    constexpr int NW = WB / 4;  // window dwords
    const int lane = threadIdx.x & 63;
    const u64 n = p.n;
    const uintptr_t in = (uintptr_t)p.in;
    bool live[R], win[R];
    u64 start[R], L[R];
    int nvr[R];
    u32 w[R][NW];
#pragma unroll
    for (int h = 0; h < R; ++h) {
        const u64 r = th[h] * kRecs + lane;
        live[h] = th[h] < ntiles && r < n;
        const u64 rc = live[h] ? r : n;
        start[h] = p.rec_off[rc];
        L[h] = p.rec_off[live[h] ? rc + 1 : rc] - start[h];
        nvr[h] = rec_nvar<NV, MIX>(p, live[h] ? r : 0);
    }
#pragma unroll
    for (int h = 0; h < R; ++h) {
        win[h] = live[h] && L[h] >= (u64)WB;
        const uintptr_t wa = win[h] ? in + start[h] : (uintptr_t)aw;  // readable filler (>= 256 B)
#pragma unroll
        for (int k = 0; k < WB / 16; ++k) {
            const u32x4 a = ld16u(wa + 16 * k);
            w[h][4 * k] = a.x;
            w[h][4 * k + 1] = a.y;
            w[h][4 * k + 2] = a.z;
            w[h][4 * k + 3] = a.w;
        }
    }
#pragma unroll
    for (int h = 0; h < R; ++h) {
        const uintptr_t A = in + start[h];
        const bool wh = win[h];
        const u64 Lh = L[h];
        auto rd8 = [&](u64 q) -> u32 {
            constexpr u64 M = WB - 4;
            return wh && q < (u64)WB ? (win_u32<NW>(w[h], (u32)min(q, M)) >> (8 * (q > M ? q - M : 0))) & 0xffu
                                     : ld_u8(A + q);
        };
        auto rd32 = [&](u64 q) -> u32 {
            return wh && q + 4 <= (u64)WB ? win_u32<NW>(w[h], (u32)q) : *(gc_u32*)(A + q);  // unaligned OK
        };
        u64 flen[NV];
#pragma unroll
        for (int f = 0; f < NV; ++f) flen[f] = 0;
        if (live[h] && Lh >= 13 && rd8(0) == 0x01) {
            const u64 off2p = rd32(1);
            if (off2p < Lh && rd8(off2p) == 0x01) {
                const u64 pts = off2p + 1;
                const u64 vt = pts + 4 * (u64)NF;  // var table: only if every int32 field fits
                if (Lh >= vt) {
#pragma unroll
                    for (int f = 0; f < NV; ++f) {
                        const u64 te = vt + 4 * (u64)f;
                        if (f < nvr[h] && Lh >= te + 4) {
                            u64 q = rd32(te);
                            if (q > 0) q += off2p;
                            if (q > 0 && Lh >= q + 4) {
                                const u64 nb = rd32(q);
                                if (Lh >= q + 4 + nb) flen[f] = nb;
                            }
                        }
                    }
                }
            }
        }
        if (th[h] < ntiles) {
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                const u64 inc = wave_incl_scan_u32w_dpp((u32)flen[f]);
                const u64 agg = (u64)(u32)__builtin_amdgcn_readlane((u32)inc, 63) |
                                ((u64)(u32)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
                if (lane == f) store_word(&aw[(size_t)f * ntiles + th[h]], make_word(epoch, kStAgg, agg));
            }
        }
    }
}

// Speculative field lengths of a kv record (NF == 0): in a record laid out as the generator writes it
// (public version, off2p = 13, ids, private version, table, then the string fields back to back up to
// the record's end; main.go:439-620), the last string field's length is the bytes left after the
// others: 14 + 8 * fields bytes of header, table and length prefixes.  So a one-field
// (GetRequest-shaped) record needs no header read, a two-field one only its first length prefix
// (bytes 22..25, k0).  The copier checks these against Go's exact parse of its
// staged bytes (spec_check) and a batch with any difference is decoded again exactly.
template <int NV>
__device__ __forceinline__ void spec_flen(u64 L, int nvr, u32 k0, u64 (&flen)[NV]) {
    flen[0] = 0;
    if constexpr (NV == 2) flen[1] = 0;
    if (nvr == 1) {
        if (L >= 22) flen[0] = L - 22;
    } else if (NV == 2 && L >= 30 && L - 30 >= (u64)k0) {
        flen[0] = k0;
        if constexpr (NV == 2) flen[NV - 1] = L - 30 - k0;
    }
}

// Speculation hold: after a batch whose speculative lengths missed, the gate stores in the ctx's
// error block (bytes 8..15, next to the error word) the number of the decode call kSpecHold calls
// ahead (p.seq counts a ctx's decode calls and is never reset); until the calls reach it the parsers
// parse exactly and the copiers skip the check, so a producer whose records do not follow the
// generator layout pays the re-decode once per kSpecHold calls, not on every batch.  The host makes a
// hold stale without touching the device: sym_ctx_set_decode_impl advances the ctx's call number past
// any hold an earlier call could have set.
constexpr u64 kSpecHold = kSpecHoldCalls;  // decode calls (codec.hpp)
__device__ __forceinline__ u64* spec_hold_word(const DecodeParams& p) { return (u64*)(p.err + 2); }
__device__ __forceinline__ bool spec_held(const DecodeParams& p) {
    const u64 h = *spec_hold_word(p);  // written by an earlier launch: visible at this launch's start
    return p.seq < h && h - p.seq <= kSpecHold;
}

// Tile-key speculation (PipeCfg::tilek): a speculative parser reads ONE first length prefix per tile
// -- the first two-field record's k0 -- and takes it for every two-field record of the tile, so the
// parsers touch one stream line per 64 records instead of one per SetRequest (the copier's stage is
// then the only other read of the record heads).  Every copier checks its records' own k0 (from the
// staged bytes) against its tile's; a difference tags ctrl[kCtrlTileMiss], the gate decodes the batch
// again exactly, and the next kTileHold calls read every record's own k0 (parse_tiles_spec's
// per-record form): a producer whose key lengths vary pays the re-decode once per kTileHold calls.
constexpr u64 kTileHold = kTileHoldCalls;  // decode calls (codec.hpp)
__device__ __forceinline__ u64* spec_tile_hold_word(const DecodeParams& p) { return (u64*)(p.err + 4); }
__device__ __forceinline__ bool spec_tile_held(const DecodeParams& p) {
    const u64 h = *spec_tile_hold_word(p);
    return p.seq < h && h - p.seq <= kTileHold;
}

// The tile's key length under tile-key speculation (wave-uniform; lane = record): the first length
// prefix of the first record that has two fields and at least 30 bytes (the only records spec_flen
// reads k0 for), 0 when there is none.  `cand` / `k0own`: this lane's record qualifies / its own k0.
__device__ __forceinline__ u32 tile_k0_of(bool cand, u32 k0own) {
    const u64 bm = __ballot(cand);
    return bm ? (u32)__builtin_amdgcn_readlane(k0own, (int)__builtin_ctzll(bm)) : 0u;
}

// parse_tiles with speculative lengths: the record offsets (and types), plus one 4-byte load per
// two-field record, or (TILEK) per tile: the first two-field record's, taken for the whole tile.
template <int NV, bool MIX, int R, bool TILEK = false>
__device__ __forceinline__ void parse_tiles_spec(const DecodeParams& p, u64* aw, u64 ntiles, u32 epoch, const u64 (&th)[R]) {
    const int lane = threadIdx.x & 63;
    const u64 n = p.n;
    const uintptr_t in = (uintptr_t)p.in;
    bool live[R];
    u64 L[R];
    int nvr[R];
    u32 k0[R];
    u64 st[R];
#pragma unroll
    for (int h = 0; h < R; ++h) {
        const u64 r = th[h] * kRecs + lane;
        live[h] = th[h] < ntiles && r < n;
        const u64 rc = live[h] ? r : n;
        st[h] = p.rec_off[rc];
        L[h] = p.rec_off[live[h] ? rc + 1 : rc] - st[h];
        nvr[h] = rec_nvar<NV, MIX>(p, live[h] ? r : 0);
        if constexpr (!TILEK) {
            const bool rd = live[h] && nvr[h] == 2 && L[h] >= 30;
            k0[h] = *(gc_u32*)(rd ? in + st[h] + 22 : (uintptr_t)aw);
        }
    }
    if constexpr (TILEK) {
        // one line per tile: the first qualifying record's start, broadcast, and one lane's load
#pragma unroll
        for (int h = 0; h < R; ++h) {
            const u64 bm = __ballot(NV == 2 && live[h] && nvr[h] == 2 && L[h] >= 30);
            const int fl = bm ? (int)__builtin_ctzll(bm) : 0;
            const u64 sf = (u64)(u32)__builtin_amdgcn_readlane((u32)st[h], fl) |
                           ((u64)(u32)__builtin_amdgcn_readlane((u32)(st[h] >> 32), fl) << 32);
            k0[h] = *(gc_u32*)(bm && lane == fl ? in + sf + 22 : (uintptr_t)aw);
        }
#pragma unroll
        for (int h = 0; h < R; ++h) {
            const u64 bm = __ballot(NV == 2 && live[h] && nvr[h] == 2 && L[h] >= 30);
            k0[h] = bm ? (u32)__builtin_amdgcn_readlane(k0[h], (int)__builtin_ctzll(bm)) : 0u;
        }
    }
#pragma unroll
    for (int h = 0; h < R; ++h) {
        u64 flen[NV];
        spec_flen<NV>(live[h] ? L[h] : 0, nvr[h], k0[h], flen);
        if (th[h] < ntiles) {
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                const u64 inc = wave_incl_scan_u32w_dpp((u32)flen[f]);
                const u64 agg = (u64)(u32)__builtin_amdgcn_readlane((u32)inc, 63) |
                                ((u64)(u32)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
                if (lane == f) store_word(&aw[(size_t)f * ntiles + th[h]], make_word(epoch, kStAgg, agg));
            }
        }
    }
}

// Parser workgroup blockIdx.x of P: each wave takes R consecutive tiles per step, steps P * 4 * R
// tiles apart.  SPEC: speculative lengths unless the ctx holds exact parsing (spec_held).
template <int NF, int NV, bool MIX, int R = 2, int WB = 32, bool SPEC = false, bool TILEK = false>
__device__ void parser(const DecodeParams& p, u64* aw, u64 ntiles, u32 epoch, u32 P) {
    const int wave = threadIdx.x >> 6;
    const bool held = SPEC && NF == 0 && spec_held(p);  // exact parsing this call (wave-uniform)
    const bool tile = TILEK && NV == 2 && SPEC && NF == 0 && !held && !spec_tile_held(p);  // one k0 per tile
    for (u64 j = ((u64)blockIdx.x * 4 + wave) * R; j < ntiles; j += (u64)P * 4 * R) {
        u64 th[R];
#pragma unroll
        for (int h = 0; h < R; ++h) th[h] = j + h < ntiles ? j + h : ntiles;  // past the end: skipped
        if (TILEK && tile) parse_tiles_spec<NV, MIX, R, true>(p, aw, ntiles, epoch, th);
        else if (SPEC && NF == 0 && !held) parse_tiles_spec<NV, MIX, R>(p, aw, ntiles, epoch, th);
        else parse_tiles<NF, NV, MIX, R, WB>(p, aw, ntiles, epoch, th);
    }
}

// ---------------------------------------------------------------- scanner role: pipe_words.hpp scanner()
constexpr int kScanPer = 2;   // the pipeline's scanner: tiles per thread per step (512-tile steps)

// ---------------------------------------------------------------- look-back (the fallback)
// Field lengths of record r with Go's checks (kv.syn.go:681-745, echo.syn.go:223-231), read straight
// from HBM: the same values the parsers and the copiers' parse compute.
template <int NF, int NV, bool MIX>
__device__ void record_flen_global(const DecodeParams& p, u64 r, u64 (&flen)[NV]) {
#pragma unroll
    for (int f = 0; f < NV; ++f) flen[f] = 0;
    const u64 start = p.rec_off[r], L = p.rec_off[r + 1] - start;
    const uintptr_t A = (uintptr_t)p.in + start;
    if (L < 13 || ld_u8(A) != 0x01) return;
    const u64 off2p = *(gc_u32*)(A + 1);  // unaligned OK
    if (off2p >= L || ld_u8(A + off2p) != 0x01) return;
    const u64 vt = off2p + 1 + 4 * (u64)NF;  // var table: only if every int32 field fits
    if (L < vt) return;
    const int nvr = rec_nvar<NV, MIX>(p, r);
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u64 te = vt + 4 * (u64)f;
        if (f < nvr && L >= te + 4) {
            u64 q = *(gc_u32*)(A + te);
            if (q > 0) q += off2p;
            if (q > 0 && L >= q + 4) {
                const u64 nb = *(gc_u32*)(A + q);
                if (L >= q + 4 + nb) flen[f] = nb;
            }
        }
    }
}

// Per-column aggregate of `tile` (whole wave, lane = record; wave-uniform result).
template <int NF, int NV, bool MIX>
__device__ void tile_agg_global(const DecodeParams& p, u64 tile, u64 (&agg)[NV]) {
    const int lane = threadIdx.x & 63;
    const u64 r = tile * kRecs + lane;
    u64 flen[NV];
    if (r < p.n) {
        record_flen_global<NF, NV, MIX>(p, r, flen);
    } else {
#pragma unroll
        for (int f = 0; f < NV; ++f) flen[f] = 0;
    }
#pragma unroll
    for (int f = 0; f < NV; ++f) agg[f] = (u64)uniform_i64((i64)wave_sum_u64(flen[f]));
}

// Exclusive prefix of `tile` per column (wave 0 of its copier): pipe_words.hpp lookback_with, a
// missing aggregate parsed from HBM.
template <int NF, int NV, bool MIX>
__device__ void lookback(const DecodeParams& p, u64* aw, u64* pw, u64 ntiles, u64 tile, u32 epoch, i64 (&pre)[NV]) {
    lookback_with<NV>(aw, pw, ntiles, tile, epoch, pre, [&](u64 t, u64 (&a)[NV]) { tile_agg_global<NF, NV, MIX>(p, t, a); });
}

// ---------------------------------------------------------------- Go's parse of one record
// kv.syn.go:681-745 (echo.syn.go:186-263 for int32 fields) on a record of L bytes read through
// rd8 / rd32 (lane = record): status, int32 fields, each string field's length and position.
template <int NF, int NV, typename Rd8, typename Rd32>
__device__ __forceinline__ void exact_parse(bool live, u64 L, int nvr, Rd8&& rd8, Rd32&& rd32, u32& st,
                                            int32_t (&fx)[NF > 0 ? NF : 1], u64 (&flen)[NV], u64 (&fpos)[NV]) {
    st = 0;
#pragma unroll
    for (int f = 0; f < NV; ++f) flen[f] = fpos[f] = 0;
    if (!live) return;
    if (L < 13) {
        st = SYM_STATUS_TOO_SHORT;  // "invalid data: too short" (kv.syn.go:681-683)
    } else if (rd8(0) != 0x01) {
        st = SYM_STATUS_BAD_VERSION;  // "invalid data: wrong public version" (:686-688)
    } else {
        const u64 off2p = rd32(1);
        if (off2p >= L || rd8(off2p) != 0x01) {
            st = SYM_STATUS_NO_PRIVATE;  // "missing private segment" (:696-698)
        } else {
            const u64 pts = off2p + 1;
            u64 toff = 0;
#pragma unroll
            for (int f = 0; f < NF; ++f, toff += 4) {  // echo.syn.go:223-231
                if (st == 0) {
                    if (L < pts + toff + 4) st = SYM_STATUS_FIELD_TOO_SHORT;
                    else fx[f] = (int32_t)rd32(pts + toff);
                }
            }
            if (st == 0) {
#pragma unroll
                for (int f = 0; f < NV; ++f, toff += 4) {  // kv.syn.go:717-742
                    if (f < nvr && L >= pts + toff + 4) {
                        u64 q = rd32(pts + toff);
                        if (q > 0) q += off2p;
                        if (q > 0 && L >= q + 4) {
                            const u64 nb = rd32(q);
                            if (L >= q + 4 + nb) {
                                flen[f] = nb;
                                fpos[f] = q + 4;
                            }
                        }
                    }
                }
            }
        }
    }
}

// Tile-key check (wave 0 of a copier, lane = record): `own` are the speculative lengths from the
// record's own first length prefix k0 (staged bytes); the parsers took the tile's k0 instead
// (tile_k0_of, the same rule).  Any record whose lengths differ tags ctrl[kCtrlTileMiss] (once).
template <int NV>
__device__ __forceinline__ void tile_check(u64* flags, u64 ntiles, u32 epoch, bool live, u64 L, int nvr, u32 k0,
                                           const u64 (&own)[NV]) {
    const bool cand = live && nvr == 2 && L >= 30;
    const u32 kt = tile_k0_of(cand, cand ? k0 : 0u);
    u64 tf[NV];
    spec_flen<NV>(live ? L : 0, nvr, kt, tf);
    bool tm = false;
#pragma unroll
    for (int f = 0; f < NV; ++f) tm |= tf[f] != own[f];
    u64* const ctrl = ctrl_words(flags, NV, ntiles);
    if (__ballot(tm) && (threadIdx.x & 63) == 0 && !tagged(load_word(&ctrl[kCtrlTileMiss]), epoch))
        store_word(&ctrl[kCtrlTileMiss], make_word(epoch, kStAgg, 1));
}

// ---------------------------------------------------------------- the copier
// Tile `tile`: stage, parse (wave 0), prefix, copy.  forced: no parsers / scanner in this launch, so
// the prefix comes from look-back at once.  SPEC: the parsers published speculative aggregates
// (parse_tiles_spec); wave 0 compares them record by record with Go's exact parse of the staged
// bytes and tags ctrl[kCtrlMismatch] on any difference (the gate then decodes the batch again), and
// a capacity error is tagged in ctrl[kCtrlSpecErr] (it may come from a speculative prefix), merged
// into p.err by the gate when the speculation held.
template <int NF, int NV, bool MIX, int MODE, int DIAG, int STG, bool SPEC, int UK = kU, bool FAST = false, bool LOC = false,
          bool CANON = false, bool TILEK = false>
__device__ __forceinline__ void copier(const DecodeParams& p, u64* flags, u32 epoch, u64 tile, bool forced, Lds<NV, STG>& S) {
    constexpr int kLoads = (STG / 16 + kThreads - 1) / kThreads;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u64 n = p.n, ntiles = num_tiles(n);
    const uintptr_t in = (uintptr_t)p.in;
    // readable limit of the stream: the 16-byte boundary past its last byte (ABI memory rule)
    const uintptr_t in_end16 = (in + p.rec_off[n] + 15) & ~(uintptr_t)15;
    const uintptr_t in_last = in_end16 - 16;
    const uintptr_t safe = (uintptr_t)flags;  // readable filler address for lanes with nothing to load
    u64* aw = flags;                          // aggregate words [NV][ntiles]
    u64* pw = flags + (size_t)NV * ntiles;    // prefix words [NV][ntiles]
    auto stamp = [&](int slot) {
        if constexpr (DIAG)
            if (tid == 0) p.dbg[tile * 8 + slot] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    const u64 r0 = tile * kRecs;
    const int cnt = (int)min((u64)kRecs, n - r0);
    const u64 s0 = p.rec_off[r0], s1 = p.rec_off[r0 + cnt];
    const uintptr_t base = (in + s0) & ~(uintptr_t)15;
    const uintptr_t stop = min((in + s1 + 15) & ~(uintptr_t)15, in_end16);
    const int nst = (int)min((u64)STG, (u64)(stop > base ? stop - base : 0));  // multiple of 16

    // ---- 1. stage (and wave 0's record offsets) ----
    u64 start = 0, endv = 0;
    const bool held = SPEC && spec_held(p);  // loaded beside the stage, used after the parse
    // FAST: the copy takes the speculative field positions (the generator's layout, spec_flen) right
    // after the stage, and wave 0 runs Go's exact parse as the check WHILE waves 1-3 copy
    const bool fast = FAST && SPEC && NF == 0 && !held;
    const bool canon = CANON && SPEC && NF == 0 && !held && !fast;
    // TILEK: the parsers took one key length per tile (spec_tile_held: unless held); the check also
    // compares every record's own k0 with its tile's
    const bool tilek_on = TILEK && NV == 2 && SPEC && NF == 0 && !held && !fast && !spec_tile_held(p);
    u32 ty = 1;  // mixed batches: the record's type, loaded with its offsets (not after the stage)
    if (wave == 0) {
        start = p.rec_off[r0 + min(lane, cnt)];
        endv = p.rec_off[r0 + min(lane + 1, cnt)];
        if constexpr (MIX) ty = p.type[lane < cnt ? r0 + lane : 0];
    }
    {
        u32x4 sv[kLoads];
#pragma unroll
        for (int k = 0; k < kLoads; ++k) {  // unconditional loads: all in flight together
            const int c = tid + kThreads * k;
            sv[k] = ld16u(16 * c < nst ? base + 16 * (uintptr_t)c : safe);
        }
#pragma unroll
        for (int k = 0; k < kLoads; ++k) {
            const int c = tid + kThreads * k;
            if (16 * c < nst) *(u32x4*)&S.stage[16 * c] = sv[k];
        }
    }
    lds_barrier();
    stamp(1);

    // ---- 2. parse + 3. prefix (wave 0) ----
    // wave 0, lane = record: its bytes from the stage (past the stage, from HBM)
    const bool live = lane < cnt;
    const u64 L = endv - start;
    const uintptr_t A = in + start;
    auto rd8 = [&](u64 q) -> u32 {
        const u64 a = (u64)(A - base) + q;
        return a < (u64)nst ? (u32)S.stage[a] : ld_u8(A + q);
    };
    auto rd32 = [&](u64 q) -> u32 {
        const u64 a = (u64)(A - base) + q;
        return a + 4 <= (u64)nst ? *(const u32*)&S.stage[a] : *(gc_u32*)(A + q);  // unaligned OK
    };
    const int nvr = MIX ? (ty != 0 ? NV : 1) : NV;  // rec_nvar
    u64 flen[NV], fpos[NV];  // (wave 0; fast: the speculative ones, kept for the check)
    if (wave == 0) {
        u32 st = 0;
        int32_t fx[NF > 0 ? NF : 1] = {};
        if (fast) {  // the generator's layout: fields back to back after the table (spec_flen)
            const u32 k0 = live && nvr == 2 && L >= 30 ? rd32(22) : 0u;
            spec_flen<NV>(live ? L : 0, nvr, k0, flen);
            fpos[0] = nvr == 2 ? 26 : 22;
            if constexpr (NV == 2) fpos[1] = 30 + (u64)k0;
            if (live) p.status[r0 + lane] = 0;  // (no int32 columns: NF == 0)
        } else if (canon) {
            // CANON: a record whose header is the generator's image (version bytes, off2p = 13, the
            // table pointing at back-to-back fields, the last length prefix = the bytes left) parses,
            // by Go's rules, to exactly its speculative lengths with status 0: six independent LDS
            // reads and one dependent one instead of Go's parse chain.  Any other record (wave-rare)
            // takes Go's exact parse, and a length it gives that differs from the speculation tags
            // the mismatch, as the check below does.
            u32 k0 = 0;
            bool ok = false;
            if (live && L >= (nvr == 2 ? 30u : 22u)) {
                const u32 b0 = rd8(0), o2 = rd32(1), b13 = rd8(13), t0 = rd32(14), t1 = rd32(18);
                const bool hdr = b0 == 1 && o2 == 13 && b13 == 1;
                if (nvr == 2) {
                    k0 = rd32(22);
                    ok = hdr && L - 30 >= (u64)k0 && t0 == 9 && t1 == 13 + k0 && rd32(26 + (u64)k0) == (u32)(L - 30 - k0);
                } else {
                    ok = hdr && t0 == 5 && t1 == (u32)(L - 22);
                }
            }
            spec_flen<NV>(live ? L : 0, nvr, k0, flen);
            fpos[0] = nvr == 2 ? 26 : 22;
            if constexpr (NV == 2) fpos[1] = 30 + (u64)k0;
            if (TILEK && tilek_on) tile_check<NV>(flags, ntiles, epoch, live, L, nvr, k0, flen);
            if (__ballot(live && !ok)) {
                if (DIAG && lane == 0) atomicAdd((unsigned long long*)&p.dbg[ntiles * 8], 1ull);  // waves off the image
                u64 elen[NV], epos[NV];
                exact_parse<NF, NV>(live, L, nvr, rd8, rd32, st, fx, elen, epos);
                bool mm = false;
                if (!ok) {
#pragma unroll
                    for (int f = 0; f < NV; ++f) {
                        mm |= elen[f] != flen[f];
                        flen[f] = elen[f];
                        fpos[f] = epos[f];
                    }
                } else {
                    st = 0;
                }
                u64* const ctrl = ctrl_words(flags, NV, ntiles);
                if (__ballot(mm) && lane == 0 && !tagged(load_word(&ctrl[kCtrlMismatch]), epoch))
                    store_word(&ctrl[kCtrlMismatch], make_word(epoch, kStAgg, 1));
            }
            if (live) p.status[r0 + lane] = (uint8_t)st;
        } else {
            exact_parse<NF, NV>(live, L, nvr, rd8, rd32, st, fx, flen, fpos);
            if (live) {
                p.status[r0 + lane] = (uint8_t)st;
#pragma unroll
                for (int f = 0; f < NF; ++f) p.fixed[f][r0 + lane] = fx[f];
            }
        }
        u64* const ctrl = ctrl_words(flags, NV, ntiles);
        if (SPEC && !held && !fast && !canon) {  // the parsers' speculative lengths of these records, from the same bytes
            const u32 k0 = live && nvr == 2 && L >= 30 ? rd32(22) : 0u;
            u64 sf[NV];
            spec_flen<NV>(live ? L : 0, nvr, k0, sf);
            bool mm = false;
#pragma unroll
            for (int f = 0; f < NV; ++f) mm |= sf[f] != flen[f];
            if (TILEK && tilek_on) tile_check<NV>(flags, ntiles, epoch, live, L, nvr, k0, sf);
            // (tag once: when every record misses, 16k copiers storing to one word contend)
            if (__ballot(mm) && lane == 0 && !tagged(load_word(&ctrl[kCtrlMismatch]), epoch))
                store_word(&ctrl[kCtrlMismatch], make_word(epoch, kStAgg, 1));
        }
        // tile scan of the field lengths (each < 2^32)
        u64 agg[NV], excl[NV];
        u32 nch[NV];
        bool too_large = false;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 inc = wave_incl_scan_u32w_dpp((u32)flen[f]);
            agg[f] = (u64)(u32)__builtin_amdgcn_readlane((u32)inc, 63) |
                     ((u64)(u32)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
            excl[f] = inc - flen[f];
            too_large |= agg[f] >= ((u64)1 << 31);  // positions inside a tile's range are 32-bit
            nch[f] = (u32)((flen[f] + 15) >> 4);
            S.src[f][lane] = start + fpos[f];
            S.dst[f][lane] = (int)excl[f];  // lanes >= cnt hold the aggregate
        }
        stamp(2);
        i64 pre[NV];
        if constexpr (MODE == 0) {
            u64 wv = 0;
            bool got = true;
            if (lane < NV) {
                // this tile's aggregate (a parser may have published the same value), then its prefix
                store_word(&aw[(size_t)lane * ntiles + tile], make_word(epoch, kStAgg, lane == 0 ? agg[0] : agg[NV - 1]));
                u64* a = &pw[(size_t)lane * ntiles + tile];
                wv = load_word(a);
                if (!forced && !tagged(wv, epoch)) {  // (the clock only when the word is not there yet)
                    const u64 t0 = now_ticks();
                    do {
                        __builtin_amdgcn_s_sleep(2);
                        wv = load_word(a);
                    } while (!tagged(wv, epoch) && now_ticks() - t0 <= kFallbackTicks);
                }
                got = tagged(wv, epoch);
            }
            if (__ballot(!got)) {  // no prefix from the scanner: resolve it here (never waits)
                lookback<NF, NV, MIX>(p, aw, pw, ntiles, tile, epoch, pre);
#pragma unroll
                for (int f = 0; f < NV; ++f)
                    if (lane == 0) store_word(&pw[(size_t)f * ntiles + tile], make_word(epoch, kStPre, (u64)pre[f]));
            } else {
                pre[0] = (i64)((u64)__shfl((long long)wv, 0, 64) & kValMask);
                if constexpr (NV == 2) pre[1] = (i64)((u64)__shfl((long long)wv, 1, 64) & kValMask);
            }
        } else {  // timing only: spread the tiles over the columns in proportion to their stream offset
            const double frac = (double)(s0 - p.rec_off[0]) / (double)(p.rec_off[n] - p.rec_off[0] + 1);
#pragma unroll
            for (int f = 0; f < NV; ++f) pre[f] = (i64)(frac * (double)p.cap[f]);
        }
        stamp(3);
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            if (live) p.offs[f][r0 + lane] = (u64)pre[f] + excl[f];
            if (lane == 0 && r0 + cnt == n) p.offs[f][n] = (u64)pre[f] + agg[f];
        }
        const u32 nrec = nch[0] + (NV == 2 ? nch[NV - 1] : 0u);
        const u32 cinc = wave_incl_scan_u32_dpp(nrec);
        S.cs[lane] = (int)(cinc - nrec);
        S.nch0[lane] = (int)nch[0];
        if (lane == 0) {
            const int T = (int)__builtin_amdgcn_readlane(cinc, 63);
            S.cs[kRecs] = T;
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                S.dst[f][kRecs] = (int)agg[f];
                S.pre[f] = pre[f];
                const i64 cap = (i64)p.cap[f];
                if (MODE == 0 && agg[f] > 0 && pre[f] + (i64)agg[f] > cap) {
                    if constexpr (SPEC) store_word(&ctrl[kCtrlSpecErr], make_word(epoch, kStAgg, kErrCapacity));
                    else atomicOr(p.err, kErrCapacity);
                }
                S.lim[f] = max((i64)0, min((i64)agg[f], cap - pre[f]));
            }
            S.total = too_large ? -1 : T;
        }
        if (__ballot(too_large) && lane == 0) atomicOr(p.err, kErrTooLarge);
    }
    lds_barrier();

    if (fast && wave == 0) {  // the check: Go's exact parse of the staged records, while waves 1-3 copy
        u32 st;
        int32_t fx[NF > 0 ? NF : 1] = {};
        u64 elen[NV], epos[NV];
        exact_parse<NF, NV>(live, L, nvr, rd8, rd32, st, fx, elen, epos);
        bool mm = live && st != 0;  // (the copy wrote status 0)
#pragma unroll
        for (int f = 0; f < NV; ++f) mm |= elen[f] != flen[f] || (flen[f] > 0 && epos[f] != fpos[f]);
        u64* const ctrl = ctrl_words(flags, NV, ntiles);
        if (__ballot(mm) && lane == 0 && !tagged(load_word(&ctrl[kCtrlMismatch]), epoch))
            store_word(&ctrl[kCtrlMismatch], make_word(epoch, kStAgg, 1));
        return;
    }

    // ---- 4. copy (all lanes; fast: waves 1-3) ----
    const int nct = fast ? kThreads - 64 : kThreads;  // copy threads
    const int ctid = fast ? tid - 64 : tid;
    const int T = __builtin_amdgcn_readfirstlane(S.total);
    // per-column values as named scalars: a two-element array indexed by a lane value goes to scratch
    const i64 pre0 = uniform_i64(S.pre[0]), pre1 = uniform_i64(S.pre[NV - 1]);
    const i64 lim0 = uniform_i64(S.lim[0]), lim1 = uniform_i64(S.lim[NV - 1]);
    const uintptr_t stage_end = base + (uintptr_t)nst;
    const bool nt = __builtin_amdgcn_readfirstlane((int)(s1 - s0 <= (u64)kNtSpan)) != 0;  // (st16)
    // LOC: a chunk's record by ballots instead of a binary search over S.cs.  Lane k of every wave
    // holds record k's first chunk (records with no chunks: never); in a wave's 64-chunk window the
    // records starting inside it mark their start with their index, and a chunk's record is the
    // nearest mark at or below it, else the last record starting at or before the window.
    __shared__ uint8_t loc_flg[LOC ? kThreads / 64 : 1][LOC ? UK : 1][64];
    int mk = 0x7fffffff;
    if constexpr (LOC) {
        if (lane < cnt && S.cs[lane + 1] > S.cs[lane]) mk = S.cs[lane];
#pragma unroll
        for (int u = 0; u < UK; ++u) loc_flg[wave][u][lane] = 0xff;
        wave_sync();
    }
    for (int c0 = 0; c0 < T; c0 += nct * UK) {  // uniform loop
        u32x4 v[UK];
        int P_[UK], code[UK];
        uintptr_t X[UK];
        bool glob[UK];
        bool anyg = false;
        int kl[UK];
        if constexpr (LOC) {
#pragma unroll
            for (int u = 0; u < UK; ++u) {
                const int d = mk - (c0 + nct * u + ctid - lane);
                if (d >= 1 && d <= 63) loc_flg[wave][u][d] = (uint8_t)lane;
            }
            wave_sync();
#pragma unroll
            for (int u = 0; u < UK; ++u) {
                const int cw = c0 + nct * u + ctid - lane;
                const u64 bm = __ballot(mk <= cw);
                const int bo = bm ? 63 - __clzll((long long)bm) : 0;
                const int fv = loc_flg[wave][u][lane];
                const u64 m = __ballot(fv != 0xff);
                if (fv != 0xff) loc_flg[wave][u][lane] = 0xff;
                const u64 mm = m & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
                const int pos = mm ? 63 - __clzll((long long)mm) : 0;
                const int vo = __shfl(fv, pos, 64);
                kl[u] = mm ? vo : bo;
            }
        }
#pragma unroll
        for (int u = 0; u < UK; ++u) {
            const int c = c0 + nct * u + ctid;
            const bool has = c < T;
            const int k = !has ? 0 : LOC ? kl[u] : lds_search_64(S.cs, cnt, c);
            int q = c - S.cs[k];
            const int n0 = S.nch0[k];
            const bool second = NV == 2 && q >= n0;
            if (second) q -= n0;
            const int f = second ? 1 : 0;
            const int dk = S.dst[f][k], L = S.dst[f][k + 1] - dk;
            const int off = L >= 16 ? min(16 * q, L - 16) : 0;
            X[u] = in + S.src[f][k] + (uintptr_t)off;
            glob[u] = has && X[u] + 16 > stage_end;
            anyg |= glob[u];
            P_[u] = has ? dk + off : -1;
            code[u] = min(L, 16) | (second ? 1 << 10 : 0);
            v[u] = has && !glob[u] ? lds16u(S.stage, (int)(X[u] - base)) : u32x4{0, 0, 0, 0};
        }
        if (__ballot(anyg)) {  // past the staged span: HBM loads, all issued before any use
            u32x4 g[UK];
#pragma unroll
            for (int u = 0; u < UK; ++u) {
                const uintptr_t Xc = X[u] < in_last ? X[u] : in_last;
                g[u] = ld16u(glob[u] ? Xc : safe);
                code[u] |= glob[u] ? (int)((X[u] - Xc) << 5) : 0;
            }
#pragma unroll
            for (int u = 0; u < UK; ++u) {
                const u32 sh = ((u32)code[u] >> 5) & 31u;
                if (sh) {  // a short field read from the stream's last block: shift down
                    u32 t[4];
                    funnel16(g[u], u32x4{0, 0, 0, 0}, sh, t);
                    g[u] = u32x4{t[0], t[1], t[2], t[3]};
                }
                if (glob[u]) v[u] = g[u];
            }
        }
#pragma unroll
        for (int u = 0; u < UK; ++u) {
            const bool second = (code[u] >> 10) & 1;
            const int nb = code[u] & 31;
            const i64 hi = min((i64)(P_[u] + nb), second ? lim1 : lim0);
            uint8_t* colb = second ? p.bytes[NV - 1] + pre1 : p.bytes[0] + pre0;
            const bool full = P_[u] >= 0 && (i64)P_[u] + 16 <= hi;
            if (full) st16(colb + P_[u], v[u], nt);
            const bool part = P_[u] >= 0 && !full && (i64)P_[u] < hi;
            if (__ballot(part)) {
                const u32 rr[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                if (part) store_chunk(colb, P_[u], 0, hi, rr, nt);
            }
        }
    }
    stamp(4);
    if constexpr (DIAG)
        if (tid == 0) p.dbg[tile * 8 + 5] = blockIdx.x;
}

// ---------------------------------------------------------------- the kernel
// The launch geometry and the measurement modes, one value per decode_pipe_kernel instantiation.
struct PipeCfg {
    int mode = 0;       // 0 the pipeline; 1 copiers only, every prefix taken as 0 (the data movement
                        // alone: a timing bound with WRONG output, tools/kbench.py variant 402)
    int diag = 0;       // 1: per-tile phase timestamps into p.dbg (8 u64 per tile, s_memrealtime at
                        // 100 MHz; tools/fused_timeline.py)
    int sk = kScanPer;  // scanner tiles per thread per step
    int pr = 2;         // parser tiles per wave step
    int stg = kStage;   // staged bytes per tile (LDS: 24.7 KB at kStage -> 6 copiers per CU)
    bool spec = false;  // speculative parsers for kv layouts, the copiers' check and the gate
    int specx = 0;      // timing only: 1 speculation without check or gate, 2 without gate (both
                        // WRONG on misfit records), 3 the gate on one workgroup per CU
    int wpe = 6;        // waves per SIMD the kernel is built for (8 needs <= 64 VGPRs and ~20 KB LDS)
    int uk = kU;        // copy chunks per lane per step
    bool fast = false;  // the copy takes the speculative positions; wave 0 checks them meanwhile
    bool loc = false;   // copy chunks find their record by ballots instead of a binary search
    bool canon = false; // speculative kv decodes: the copier checks the generator's header image, Go's
                        // exact parse only for records that differ from it
    bool tilek = false; // speculative two-field kv decodes: one key length read per tile (spec_tile_held)
};

template <int NF, int NV, bool MIX, PipeCfg C>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(C.wpe, 8))) void decode_pipe_kernel(
    DecodeParams p, u64* flags, u32 epoch) {
    static_assert(NV == 1 || NV == 2, "decode handles one or two string columns");
    static_assert(C.mode == 0 || C.mode == 1, "pipeline or copiers only");
    __shared__ Lds<NV, C.stg> S;
    const u64 ntiles = num_tiles(p.n);
    u64* aw = flags;                        // aggregate words [NV][ntiles]
    u64* pw = flags + (size_t)NV * ntiles;  // prefix words [NV][ntiles]

    const u32 P = p.pipe_parsers;
    const bool forced = p.impl == kImplLookback;  // parsers and scanner idle: look-back only
    constexpr bool kRoles = C.mode == 0;
    if (kRoles && blockIdx.x < P) {
        if (!forced) parser<NF, NV, MIX, C.pr, 32, C.spec, C.tilek>(p, aw, ntiles, epoch, P);
        return;
    }
    if (kRoles && blockIdx.x == P) {
        if (!forced) scanner<NV, C.sk>(aw, pw, ntiles, epoch, S, C.diag ? p.dbg + 1 : nullptr);  // diag: publish times in slot 6
        return;
    }
    const u64 tile = kRoles ? blockIdx.x - P - 1 : blockIdx.x;
    if (tile >= ntiles) return;
    copier<NF, NV, MIX, C.mode, C.diag, C.stg, C.spec && C.mode == 0 && C.specx != 1, C.uk, C.fast, C.loc, C.canon, C.tilek>(
        p, flags, epoch, tile, forced, S);
}

// ---------------------------------------------------------------- the gate
// Runs after every speculative launch (same stream).  When no copier found a speculative length
// wrong -- every batch the generator's layout produced -- each workgroup reads one word and exits,
// and workgroup 0 moves the launch's error bits into p.err.  Otherwise the batch is decoded again
// exactly under tag epoch + 1, rewriting every output of the first launch: the pipeline's roles on
// a persistent grid (exact parsers, the scanner, copiers taking tiles in turn).  Progress never
// depends on which workgroups are resident.
template <int NF, int NV, bool MIX>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(6, 8))) void decode_gate_kernel(
    DecodeParams p, u64* flags, u32 epoch) {
    __shared__ Lds<NV, kStage> S;
    const u64 ntiles = num_tiles(p.n);
    u64* const ctrl = ctrl_words(flags, NV, ntiles);
    const bool miss = tagged((u64)uniform_i64((i64)load_word(&ctrl[kCtrlMismatch])), epoch);
    const bool tmiss = tagged((u64)uniform_i64((i64)load_word(&ctrl[kCtrlTileMiss])), epoch);
    const bool redo = miss || tmiss;
    if (!redo && blockIdx.x == 0 && threadIdx.x == 0) {
        const u64 e = load_word(&ctrl[kCtrlSpecErr]);
        if (tagged(e, epoch)) atomicOr(p.err, (unsigned)(e & kValMask));
    }
    if (!redo) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (miss) *spec_hold_word(p) = p.seq + kSpecHold + 1;        // the next kSpecHold calls parse exactly
        if (tmiss) *spec_tile_hold_word(p) = p.seq + kTileHold + 1;  // the next kTileHold calls read every k0
        *(u64*)(p.err + 6) += 1;  // the ctx's re-decode count (sym_ctx_decode_redos; stream-ordered)
    }
    // the exact pipeline on a persistent grid: a quarter of the workgroups parse every tile exactly,
    // one scans, the rest copy tiles c, c + C, ... (a copier whose prefix is late looks back, so no
    // role waits on residency)
    u64* aw = flags;
    u64* pw = flags + (size_t)NV * ntiles;
    const u32 G = gridDim.x, P = G >= 8 ? G / 4 : 0;
    if (blockIdx.x < P) {
        parser<NF, NV, MIX, 2, 32>(p, aw, ntiles, epoch + 1, P);
        return;
    }
    if (P && blockIdx.x == P) {
        scanner<NV, kScanPer>(aw, pw, ntiles, epoch + 1, S);
        return;
    }
    const u32 c0 = P ? P + 1 : 0;
    for (u64 tile = blockIdx.x - c0; tile < ntiles; tile += G - c0) {
        copier<NF, NV, MIX, 0, 0, kStage, false>(p, flags, epoch + 1, tile, P == 0, S);
        lds_barrier();  // the next tile restages S
    }
}

template <int NF, int NV, bool MIX, PipeCfg C>
hipError_t launch(const DecodeParams& p, u64* flags, u32 epoch, hipStream_t stream, int pnum = 1, int pden = 1) {
    if (C.diag && !p.dbg) return hipErrorInvalidValue;  // timestamps need SYMHIP_DEBUG_PTR (tuning builds)
    static int cus[16] = {0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    int& ncu = cus[dev & 15];
    if (ncu == 0 && (e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    const u64 nt = num_tiles(p.n);
    constexpr bool kRoles = C.mode == 0;
    u64 P = kRoles ? (u64)ncu * pnum / pden : 0;  // parser workgroups: pnum / pden per CU
    if (P > (nt + 3) / 4) P = (nt + 3) / 4;
    DecodeParams q = p;
    q.pipe_parsers = (unsigned)P;
    const u64 grid = kRoles ? P + 1 + nt : nt;
    // speculative parsers: only kv layouts (no int32 fields) under the pipeline with its parsers
    constexpr bool kSpec = C.spec && NF == 0 && C.mode == 0;
    if constexpr (kSpec) {
        if (p.impl != kImplLookback && P > 0) {
            hipLaunchKernelGGL((decode_pipe_kernel<NF, NV, MIX, C>), dim3((unsigned)grid), dim3(kThreads), 0, stream, q, flags,
                               epoch);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            if (C.specx == 1 || C.specx == 2) return hipSuccess;  // timing variants: no gate (WRONG on misfits)
            // one workgroup per CU (the gate's cost is the launch behind the first kernel); a
            // re-decode is the exact pipeline on them
            const u64 g = min(nt + 1 + ncu, (u64)ncu * (C.specx == 3 ? 1 : 4));
            hipLaunchKernelGGL((decode_gate_kernel<NF, NV, MIX>), dim3((unsigned)g), dim3(kThreads), 0, stream, q, flags, epoch);
            return hipGetLastError();
        }
    }
    constexpr PipeCfg X = [] { PipeCfg c = C; c.spec = false; c.specx = 0; return c; }();
    hipLaunchKernelGGL((decode_pipe_kernel<NF, NV, MIX, X>), dim3((unsigned)grid), dim3(kThreads), 0, stream, q, flags, epoch);
    return hipGetLastError();
}

constexpr int kParsersNum = 3;   // parser workgroups = #CUs * 3/4
constexpr int kParsersDen = 4;

template <PipeCfg C>
hipError_t launch_layout(const DecodeParams& p, u64* flags, u32 epoch, hipStream_t stream, int pnum = kParsersNum,
                         int pden = kParsersDen) {
    if (p.type)  // mixed kv batch: GetRequest / SetRequest per record
        return p.lay.nfixed == 0 && p.lay.nvar == 2 ? launch<0, 2, true, C>(p, flags, epoch, stream, pnum, pden)
                                                     : hipErrorInvalidValue;
    if (p.lay.nfixed == 0 && p.lay.nvar == 1) return launch<0, 1, false, C>(p, flags, epoch, stream, pnum, pden);
    if (p.lay.nfixed == 0 && p.lay.nvar == 2) return launch<0, 2, false, C>(p, flags, epoch, stream, pnum, pden);
    if (p.lay.nfixed == 2 && p.lay.nvar == 2) return launch<2, 2, false, C>(p, flags, epoch, stream, pnum, pden);
    return hipErrorInvalidValue;
}

}  // namespace pipe

size_t decode_pipe_flag_bytes(int nvar, uint64_t n) {
    // aggregate + prefix word per column and tile, then 256 bytes: the scanner's store sink
    // (pipe_words.hpp), then 256 bytes of control words (pipe::ctrl_words); the start doubles as the
    // kernels' filler load address
    return ((size_t)nvar * 2 * pipe::num_tiles(n) * sizeof(u64) + 512 + 255) & ~(size_t)255;
}

// The default: speculative kv decodes with parsers on half the CUs and 256-tile scanner steps;
// exact parsers (int32 fields) on 3/4 of the CUs with 512-tile steps (tools/kbench.py sweeps,
// DESIGN.md section 4).  Tuning builds (make tuning) add the measurement variants below; the decode
// experiments of rounds 1-3 that were not adopted (parse geometry sweeps 431-492, the gather copier
// 600-603, copier parse-ahead 620-624, parse-free copiers 700-702, early prefix loads and 20992-byte
// stages 720-728, the persistent ring 500-512) were retired in round 4 with their numbers recorded
// in DESIGN.md; their code is in the history before that commit.
namespace pipe {
// kv layouts: copy chunks located by ballots, the copier's check on the generator's header image
// (round 5, tools/kbench.py: config 2 159 -> 155 us, config 3 393 -> 385 us; variant 730 is the
// round-4 form)
// round 6: one key length read per tile (tilek; tools/kbench.py, one process: config 2 162.6 -> 156.1 us,
// config 3 386.9 -> 369.7 us, the mix 101.7 -> 100.8 us; profiles/r06_*)
constexpr PipeCfg kSpecCfg{.sk = 1, .spec = true, .loc = true, .canon = true, .tilek = true};
constexpr PipeCfg kExactCfg{.spec = true};          // int32 layouts (exact parsers: spec needs NF == 0)
// mixed Get/Set batches: 8 waves per SIMD (<= 64 VGPRs) with a 16 KiB stage, 8 copiers per CU
// (tuning variant 740; r04b: 117.7 -> 102.4 us for the 2^20-record mix, trace mix 551 -> 554 us;
// config 2's 350-byte records run slower so, 159 -> 188 us, and keep kSpecCfg)
constexpr PipeCfg kMixCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .tilek = true};
}  // namespace pipe

hipError_t launch_decode_pipe(const DecodeParams& p, void* flags, unsigned epoch, hipStream_t stream) {
    using pipe::launch_layout;
    using pipe::PipeCfg;
    u64* fl = (u64*)flags;
#ifdef SYMHIP_TUNING
    switch (p.variant) {
        // timing bounds and timelines: copiers only (WRONG output), per-tile timestamps
        case 402: return launch_layout<PipeCfg{.mode = 1}>(p, fl, epoch, stream);
        case 410: return launch_layout<PipeCfg{.diag = 1}>(p, fl, epoch, stream);
        case 412: return launch_layout<PipeCfg{.mode = 1, .diag = 1}>(p, fl, epoch, stream);
        // exact parsers (no speculation, no gate): the round-2 default
        case 710: return launch_layout<PipeCfg{}>(p, fl, epoch, stream);
        // speculation without the copiers' check and the gate / with the check, no gate / gate on one
        // workgroup per CU (711 and 712 are WRONG on batches the speculation misses)
        case 711: return launch_layout<PipeCfg{.spec = true, .specx = 1}>(p, fl, epoch, stream);
        case 712: return launch_layout<PipeCfg{.spec = true, .specx = 2}>(p, fl, epoch, stream);
        case 713: return launch_layout<PipeCfg{.spec = true, .specx = 3}>(p, fl, epoch, stream);
        // speculative parsers on half the CUs: scanner tiles per thread 1 / 4, parser tiles per wave step 4 / 1
        case 730: return launch_layout<PipeCfg{.sk = 1, .spec = true}>(p, fl, epoch, stream, 1, 2);
        case 731: return launch_layout<PipeCfg{.sk = 4, .spec = true}>(p, fl, epoch, stream, 1, 2);
        case 732: return launch_layout<PipeCfg{.sk = 2, .pr = 4, .spec = true}>(p, fl, epoch, stream, 1, 2);
        case 733: return launch_layout<PipeCfg{.sk = 2, .pr = 1, .spec = true}>(p, fl, epoch, stream, 1, 2);
        // round 4: 8 waves per SIMD (<= 64 VGPRs) with a 16 KiB stage (8 copiers per CU by LDS); 742:
        // copiers only at 8 per CU (WRONG output); 743: the 16 KiB stage at 6 waves per SIMD; 747: a
        // 17 KiB stage; 748 / 749: parsers on 3/8, 3/4 of the CUs
        case 740: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8}>(p, fl, epoch, stream, 1, 2);
        case 742: return launch_layout<PipeCfg{.mode = 1, .sk = 1, .stg = 16384, .spec = true, .wpe = 8}>(p, fl, epoch, stream, 1, 2);
        case 743: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true}>(p, fl, epoch, stream, 1, 2);
        case 747: return launch_layout<PipeCfg{.sk = 1, .stg = 17408, .spec = true, .wpe = 8}>(p, fl, epoch, stream, 1, 2);
        case 748: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8}>(p, fl, epoch, stream, 3, 8);
        case 749: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8}>(p, fl, epoch, stream, 3, 4);
        // round 4: copy chunks per lane per step 3 / 4 (default stage), and 3 with the 8-wave 16 KiB stage
        case 744: return launch_layout<PipeCfg{.sk = 1, .spec = true, .uk = 3}>(p, fl, epoch, stream, 1, 2);
        case 745: return launch_layout<PipeCfg{.sk = 1, .spec = true, .uk = 4}>(p, fl, epoch, stream, 1, 2);
        case 746: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .uk = 3}>(p, fl, epoch, stream, 1, 2);
        // round 4: the fast copier (speculative positions, the exact parse as a check beside the copy)
        case 750: return launch_layout<PipeCfg{.sk = 1, .spec = true, .fast = true}>(p, fl, epoch, stream, 1, 2);
        case 751: return launch_layout<PipeCfg{.sk = 1, .spec = true, .uk = 3, .fast = true}>(p, fl, epoch, stream, 1, 2);
        case 752: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .fast = true}>(p, fl, epoch, stream, 1, 2);
        case 753: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .uk = 3, .fast = true}>(p, fl, epoch, stream, 1, 2);
        // round 5: timestamps of the default kv decode; copy chunks located by ballots (LOC), with
        // timestamps, with 3 chunks per lane, and on the mixed batch's 8-wave 16 KiB stage
        case 414: return launch_layout<PipeCfg{.diag = 1, .sk = 1, .spec = true}>(p, fl, epoch, stream, 1, 2);
        case 760: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true}>(p, fl, epoch, stream, 1, 2);
        case 761: return launch_layout<PipeCfg{.diag = 1, .sk = 1, .spec = true, .loc = true}>(p, fl, epoch, stream, 1, 2);
        case 762: return launch_layout<PipeCfg{.sk = 1, .spec = true, .uk = 3, .loc = true}>(p, fl, epoch, stream, 1, 2);
        case 764: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 765: return launch_layout<PipeCfg{.diag = 1, .sk = 1, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 766: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 767: return launch_layout<PipeCfg{.sk = 1, .spec = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        // round 5: parser and scanner geometry around the default (startup: the first prefixes)
        case 770: return launch_layout<PipeCfg{.sk = 1, .pr = 4, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 771: return launch_layout<PipeCfg{.sk = 2, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 772: return launch_layout<PipeCfg{.sk = 2, .pr = 4, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 773: return launch_layout<PipeCfg{.diag = 1, .sk = 1, .pr = 4, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 774: return launch_layout<PipeCfg{.sk = 1, .pr = 4, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 3, 8);
        case 775: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 3, 8);
        // (round 5, measured slower and removed: the prefix word loaded when the tile starts, 156 ->
        // 160 us; loaded right after the stage, ahead of the parse's stores, 158 -> 162 us)
        // (round 5, measured no faster and removed: the record heads' first 32 bytes loaded into
        // registers beside the stage for the header-image check, 156 -> 158 us)
        // round 5: the default with the gate on one workgroup per CU (152.1 vs 152.6 us: the gate's
        // ~4.7 us is its launch behind the pipeline, not its 1024 workgroups)
        case 788: return launch_layout<PipeCfg{.sk = 1, .spec = true, .specx = 3, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        // round 5: parser workgroups at one and two per CU (the mixed batch's config; config 2's):
        // mixed 100.6 -> 105.7 / 113.2 us, config 2 153.4 -> 156.3 us (kbench medians): half a CU's worth kept
        case 789: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8}>(p, fl, epoch, stream, 1, 1);
        case 790: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8}>(p, fl, epoch, stream, 2, 1);
        case 791: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 1);
        case 787: return launch_layout<PipeCfg{.diag = 1, .sk = 1, .stg = 16384, .spec = true, .wpe = 8, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 768: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .canon = true}>(p, fl, epoch, stream, 1, 2);
        case 763: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .loc = true}>(p, fl, epoch, stream, 1, 2);
        // round 6: one key length read per tile (tile-key speculation), kv layouts / the mixed batch
        case 792: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true, .canon = true, .tilek = true}>(p, fl, epoch, stream, 1, 2);
        case 793: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .tilek = true}>(p, fl, epoch, stream, 1, 2);
        case 794: return launch_layout<PipeCfg{.mode = 1, .sk = 1, .loc = true, .canon = true}>(p, fl, epoch, stream, 1, 2);
        // round 6, the mixed batch with tile-key parsers: parsers on 1/4, 3/8 of the CUs; the header-image
        // check; with ballot-located chunks; config 2's geometry (22.5 KB stage, 6 waves)
        case 795: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .tilek = true}>(p, fl, epoch, stream, 1, 4);
        case 796: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .tilek = true}>(p, fl, epoch, stream, 3, 8);
        case 797: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .canon = true, .tilek = true}>(p, fl, epoch, stream, 1, 2);
        case 798: return launch_layout<PipeCfg{.sk = 1, .stg = 16384, .spec = true, .wpe = 8, .loc = true, .canon = true, .tilek = true}>(p, fl, epoch, stream, 1, 2);
        case 799: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true, .canon = true, .tilek = true}>(p, fl, epoch, stream, 1, 2);
        // round 6, kv layouts with tile-key parsers (lighter): parsers on 1/4, 1/8, 3/8 of the CUs; a
        // 2-tile scanner step; parser tiles per step 4 -- config 2 145.8 (default) vs 153.4 / 186.0 /
        // 145.5 / 165.7 / 147.1 us (profiles/r06_kbench_tilek_parsers_c2.txt): the default kept
        case 800: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true, .canon = true, .tilek = true}>(p, fl, epoch, stream, 1, 4);
        case 801: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true, .canon = true, .tilek = true}>(p, fl, epoch, stream, 1, 8);
        case 802: return launch_layout<PipeCfg{.sk = 1, .spec = true, .loc = true, .canon = true, .tilek = true}>(p, fl, epoch, stream, 3, 8);
        case 803: return launch_layout<PipeCfg{.sk = 2, .spec = true, .loc = true, .canon = true, .tilek = true}>(p, fl, epoch, stream, 1, 4);
        case 804: return launch_layout<PipeCfg{.sk = 1, .pr = 4, .spec = true, .loc = true, .canon = true, .tilek = true}>(p, fl, epoch, stream, 1, 4);
        default: break;
    }
#endif
    // speculative parsers are lighter: half the CUs' worth of them keeps ahead of the copiers, and the
    // scanner's 256-tile steps publish sooner (sweeps with configs 2, 3 and the mixed batch,
    // DESIGN.md); exact parsers (int32 fields) keep 3/4 of the CUs and 512-tile steps
    if (p.type)
        return p.lay.nfixed == 0 && p.lay.nvar == 2 ? pipe::launch<0, 2, true, pipe::kMixCfg>(p, fl, epoch, stream, 1, 2)
                                                     : hipErrorInvalidValue;
    if (p.lay.nfixed == 0) return launch_layout<pipe::kSpecCfg>(p, fl, epoch, stream, 1, 2);
    return launch_layout<pipe::kExactCfg>(p, fl, epoch, stream);
}

}  // namespace symhip
