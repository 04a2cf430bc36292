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
//               4-byte load (spec_flen) -- the parsers' header reads were ~10 % of the decode time.
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

// PACE > 0: a parser wave starts a step only once tile t0 - PACE has its prefix (bounded wait), so
// the header lines it reads are still cached when that tile's copier stages them.  XCDP: a parser
// takes only tiles whose copier shares its blockIdx % 8 group (one XCD under round-robin placement),
// so those lines are in that XCD's L2 (speed only; any placement gives the same results).
// R tiles th[] by one wave (lane = record): the records' field lengths with Go's checks, then each
// tile's aggregate word per column.  Every load of the R records is issued before any is used.
template <int NF, int NV, bool MIX, int R, int WB, bool LIGHT = false>
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
        if constexpr (LIGHT) live[h] = win[h] = false;  // timing: offsets only, no header reads
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
                const u64 agg = (u64)__builtin_amdgcn_readlane((u32)inc, 63) |
                                ((u64)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
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

// parse_tiles with speculative lengths: the record offsets (and types), plus one 4-byte load per
// two-field record.
template <int NV, bool MIX, int R>
__device__ __forceinline__ void parse_tiles_spec(const DecodeParams& p, u64* aw, u64 ntiles, u32 epoch, const u64 (&th)[R]) {
    const int lane = threadIdx.x & 63;
    const u64 n = p.n;
    const uintptr_t in = (uintptr_t)p.in;
    bool live[R];
    u64 L[R];
    int nvr[R];
    u32 k0[R];
#pragma unroll
    for (int h = 0; h < R; ++h) {
        const u64 r = th[h] * kRecs + lane;
        live[h] = th[h] < ntiles && r < n;
        const u64 rc = live[h] ? r : n;
        const u64 st = p.rec_off[rc];
        L[h] = p.rec_off[live[h] ? rc + 1 : rc] - st;
        nvr[h] = rec_nvar<NV, MIX>(p, live[h] ? r : 0);
        const bool rd = live[h] && nvr[h] == 2 && L[h] >= 30;
        k0[h] = *(gc_u32*)(rd ? in + st + 22 : (uintptr_t)aw);
    }
#pragma unroll
    for (int h = 0; h < R; ++h) {
        u64 flen[NV];
        spec_flen<NV>(live[h] ? L[h] : 0, nvr[h], k0[h], flen);
        if (th[h] < ntiles) {
#pragma unroll
            for (int f = 0; f < NV; ++f) {
                const u64 inc = wave_incl_scan_u32w_dpp((u32)flen[f]);
                const u64 agg = (u64)__builtin_amdgcn_readlane((u32)inc, 63) |
                                ((u64)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
                if (lane == f) store_word(&aw[(size_t)f * ntiles + th[h]], make_word(epoch, kStAgg, agg));
            }
        }
    }
}

// PACE > 0: a parser wave starts a step only once tile t0 - PACE has its prefix (bounded wait), so
// the header lines it reads are still cached when that tile's copier stages them.  XCDP: a parser
// takes only tiles whose copier shares its blockIdx % 8 group (one XCD under round-robin placement),
// so those lines are in that XCD's L2 (speed only; any placement gives the same results).  tmax:
// only tiles below it (the copiers parse the others ahead, AHEAD in decode_pipe_kernel).
template <int NF, int NV, bool MIX, int R = 2, int WB = 32, bool LIGHT = false, int PACE = 0, bool XCDP = false,
          bool SPEC = false>
__device__ void parser(const DecodeParams& p, u64* aw, u64* pw, u64 ntiles, u32 epoch, u32 P, u64 tmax = ~0ull) {
    const int wave = threadIdx.x >> 6;
    const u64 tlim = min(ntiles, tmax);
    const bool held = SPEC && NF == 0 && spec_held(p);  // exact parsing this call (wave-uniform)
    // tile of (sequence index j, slot h) = tb + ts * (j + h)
    u64 tb = 0, ts = 1, j0 = ((u64)blockIdx.x * 4 + wave) * R, jstep = (u64)P * 4 * R;
    if (XCDP && P % 8 == 0) {
        const u64 g = blockIdx.x & 7, i = blockIdx.x >> 3;
        tb = (g + 8 - ((P + 1) & 7)) & 7;  // copier of tile t is block P + 1 + t
        ts = 8;
        j0 = (i * 4 + wave) * R;
        jstep = (u64)(P / 8) * 4 * R;
    }
    for (u64 j = j0; tb + ts * j < tlim; j += jstep) {
        u64 th[R];
#pragma unroll
        for (int h = 0; h < R; ++h) {
            th[h] = tb + ts * (j + h);
            if (th[h] >= tlim) th[h] = ntiles;  // past the parsers' range: skipped
        }
        const u64 t0 = th[0];
        if constexpr (PACE > 0) {
            if (t0 >= (u64)PACE) {
                u64* w = &pw[t0 - PACE];
                for (const u64 ts0 = now_ticks(); !tagged(load_word(w), epoch) && now_ticks() - ts0 <= kFallbackTicks;)
                    __builtin_amdgcn_s_sleep(8);
            }
        }
        if (SPEC && NF == 0 && !held) parse_tiles_spec<NV, MIX, R>(p, aw, ntiles, epoch, th);
        else parse_tiles<NF, NV, MIX, R, WB, LIGHT>(p, aw, ntiles, epoch, th);
    }
}

// ---------------------------------------------------------------- scanner role: pipe_words.hpp scanner()
constexpr int kScanPerG = 2;  // the gather copier's scanner: tiles per thread per step
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

// ---------------------------------------------------------------- the copier
// Tile `tile`: stage, parse (wave 0), prefix, copy.  forced: no parsers / scanner in this launch, so
// the prefix comes from look-back at once.  SPEC: the parsers published speculative aggregates
// (parse_tiles_spec); wave 0 compares them record by record with Go's exact parse of the staged
// bytes and tags ctrl[kCtrlMismatch] on any difference (the gate then decodes the batch again), and
// a capacity error is tagged in ctrl[kCtrlSpecErr] (it may come from a speculative prefix), merged
// into p.err by the gate when the speculation held.
template <int NF, int NV, bool MIX, int MODE, int DIAG, int STG, bool EARLY, int AHEAD, int NOP, bool SPEC, int UK = kU>
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

    // ---- 1. stage (and wave 0's record offsets, and with EARLY its prefix words) ----
    u64 start = 0, endv = 0, wv_early = 0;
    const bool held = SPEC && spec_held(p);  // loaded beside the stage, used after the parse
    if (wave == 0) {
        start = p.rec_off[r0 + min(lane, cnt)];
        endv = p.rec_off[r0 + min(lane + 1, cnt)];
        if (EARLY && MODE == 0 && lane < NV) wv_early = load_word(&pw[(size_t)lane * ntiles + tile]);
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

    // ---- 2. parse + 3. prefix (wave 0); with AHEAD, wave 1 parses tile + AHEAD meanwhile ----
    if constexpr (AHEAD > 0) {
        if (wave == 1 && !forced && tile + AHEAD < ntiles) {
            const u64 ta[1] = {tile + AHEAD};
            parse_tiles<NF, NV, MIX, 1, 32>(p, aw, ntiles, epoch, ta);
        }
    }
    if (wave == 0) {
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
        u32 st = 0;
        int32_t fx[NF > 0 ? NF : 1] = {};
        u64 flen[NV], fpos[NV];
#pragma unroll
        for (int f = 0; f < NV; ++f) flen[f] = fpos[f] = 0;
        const int nvr = rec_nvar<NV, MIX>(p, live ? r0 + lane : 0);
        if (NOP && live) {  // timing only: the config-2 SetRequest layout assumed, no LDS reads
            flen[0] = 64;
            fpos[0] = 26;
            if constexpr (NV == 2) {
                flen[1] = L - 94;
                fpos[1] = 94;
            }
            p.status[r0 + lane] = 0;
        } else if (live) {
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
            p.status[r0 + lane] = (uint8_t)st;
#pragma unroll
            for (int f = 0; f < NF; ++f) p.fixed[f][r0 + lane] = fx[f];
        }
        u64* const ctrl = ctrl_words(flags, NV, ntiles);
        if (SPEC && !held) {  // the parsers' speculative lengths of these records, from the same bytes
            const u32 k0 = live && nvr == 2 && L >= 30 ? rd32(22) : 0u;
            u64 sf[NV];
            spec_flen<NV>(live ? L : 0, nvr, k0, sf);
            bool mm = false;
#pragma unroll
            for (int f = 0; f < NV; ++f) mm |= sf[f] != flen[f];
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
            agg[f] = (u64)__builtin_amdgcn_readlane((u32)inc, 63) |
                     ((u64)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
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
                wv = EARLY && tagged(wv_early, epoch) ? wv_early : load_word(a);
                if (!forced) {
                    for (const u64 t0 = now_ticks(); !tagged(wv, epoch) && now_ticks() - t0 <= kFallbackTicks;) {
                        __builtin_amdgcn_s_sleep(2);
                        wv = load_word(a);
                    }
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
            if ((MODE == 2 || MODE == 3) && lane < NV)
                store_word(&aw[(size_t)lane * ntiles + tile], make_word(epoch, kStAgg, lane == 0 ? agg[0] : agg[NV - 1]));
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

    // ---- 4. copy (all lanes) ----
    const int T = __builtin_amdgcn_readfirstlane(S.total);
    // per-column values as named scalars: a two-element array indexed by a lane value goes to scratch
    const i64 pre0 = uniform_i64(S.pre[0]), pre1 = uniform_i64(S.pre[NV - 1]);
    const i64 lim0 = uniform_i64(S.lim[0]), lim1 = uniform_i64(S.lim[NV - 1]);
    const uintptr_t stage_end = base + (uintptr_t)nst;
    for (int c0 = 0; c0 < T; c0 += kThreads * UK) {  // uniform loop
        u32x4 v[UK];
        int P_[UK], code[UK];
        uintptr_t X[UK];
        bool glob[UK];
        bool anyg = false;
#pragma unroll
        for (int u = 0; u < UK; ++u) {
            const int c = c0 + kThreads * u + tid;
            const bool has = c < T;
            const int k = has ? lds_search_64(S.cs, cnt, c) : 0;
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
            if (full) *(g_u4*)(colb + P_[u]) = v[u];
            const bool part = P_[u] >= 0 && !full && (i64)P_[u] < hi;
            if (__ballot(part)) {
                const u32 rr[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                if (part) store_chunk(colb, P_[u], 0, hi, rr);
            }
        }
    }
    stamp(4);
    if constexpr (DIAG)
        if (tid == 0) p.dbg[tile * 8 + 5] = blockIdx.x;
}

// ---------------------------------------------------------------- the kernel
// MODE 0: the pipeline.  MODE 1: copiers only, every prefix taken as 0 (timing of the data movement
// alone; wrong output -- tools/kbench.py variant 402).  DIAG: per-tile phase timestamps into p.dbg
// (8 u64 per tile, s_memrealtime at 100 MHz; tools/fused_timeline.py).
// STG: staged bytes per tile (LDS: 24.7 KB at kStage -> 6 copiers per CU; below ~21 KB -> 7).
// EARLY: the prefix word is loaded when the tile starts, so its cross-XCD round trip overlaps the
// stage instead of following the parse.  PACE, XCDP: see parser().
// AHEAD > 0: the parsers take only tiles [0, AHEAD); the copier of tile t parses tile t + AHEAD
// (wave 1, while wave 0 parses its own tile from LDS) -- the same XCD under round-robin placement
// when AHEAD % 8 == 0, so the header lines it reads are still in that XCD's L2 when tile t + AHEAD
// is staged, and the stream is fetched from HBM about once.
template <int NF, int NV, bool MIX, int MODE = 0, int DIAG = 0, int SK = 4, int PR = 2, int STG = kStage,
          bool EARLY = false, int PACE = 0, bool XCDP = false, int AHEAD = 0, int NOP = 0, bool SPEC = false, int SPECX = 0,
          int WPE = 6, int UK = kU>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void decode_pipe_kernel(
    DecodeParams p, u64* flags, u32 epoch) {
    static_assert(NV == 1 || NV == 2, "decode handles one or two string columns");
    __shared__ Lds<NV, STG> S;
    const u64 ntiles = num_tiles(p.n);
    u64* aw = flags;                        // aggregate words [NV][ntiles]
    u64* pw = flags + (size_t)NV * ntiles;  // prefix words [NV][ntiles]

    const u32 P = p.pipe_parsers;
    const bool forced = p.impl == kImplLookback;  // parsers and scanner idle: look-back only
    // MODE 2 / 3 (timing): roles run, copiers never wait; 3: parsers read only the offsets
    constexpr bool kRoles = MODE == 0 || MODE == 2 || MODE == 3;
    if (kRoles && blockIdx.x < P) {
        if (!forced)
            parser<NF, NV, MIX, PR, 32, MODE == 3, PACE, XCDP, SPEC>(p, aw, pw, ntiles, epoch, P, AHEAD > 0 ? (u64)AHEAD : ~0ull);
        return;
    }
    if (kRoles && blockIdx.x == P) {
        if (!forced) scanner<NV, SK>(aw, pw, ntiles, epoch, S);
        return;
    }
    const u64 tile = kRoles ? blockIdx.x - P - 1 : blockIdx.x;
    if (tile >= ntiles) return;
    copier<NF, NV, MIX, MODE, DIAG, STG, EARLY, AHEAD, NOP, SPEC && MODE == 0 && SPECX != 1, UK>(p, flags, epoch, tile, forced, S);
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
    const bool redo = tagged((u64)uniform_i64((i64)load_word(&ctrl[kCtrlMismatch])), epoch);
    if (!redo && blockIdx.x == 0 && threadIdx.x == 0) {
        const u64 e = load_word(&ctrl[kCtrlSpecErr]);
        if (tagged(e, epoch)) atomicOr(p.err, (unsigned)(e & kValMask));
    }
    if (!redo) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) *spec_hold_word(p) = p.seq + kSpecHold + 1;  // the next kSpecHold calls parse exactly
    // the exact pipeline on a persistent grid: a quarter of the workgroups parse every tile exactly,
    // one scans, the rest copy tiles c, c + C, ... (a copier whose prefix is late looks back, so no
    // role waits on residency)
    u64* aw = flags;
    u64* pw = flags + (size_t)NV * ntiles;
    const u32 G = gridDim.x, P = G >= 8 ? G / 4 : 0;
    if (blockIdx.x < P) {
        parser<NF, NV, MIX, 2, 32>(p, aw, pw, ntiles, epoch + 1, P);
        return;
    }
    if (P && blockIdx.x == P) {
        scanner<NV, kScanPer>(aw, pw, ntiles, epoch + 1, S);
        return;
    }
    const u32 c0 = P ? P + 1 : 0;
    for (u64 tile = blockIdx.x - c0; tile < ntiles; tile += G - c0) {
        copier<NF, NV, MIX, 0, 0, kStage, false, 0, 0, false>(p, flags, epoch + 1, tile, P == 0, S);
        lds_barrier();  // the next tile restages S
    }
}

// ---------------------------------------------------------------- the gather copier
// A copier without the LDS stage.  Wave 0 parses its 64 records straight from HBM through a 96-byte
// register window per record -- the lines the copy reads next, so they are fetched once -- runs Go's
// checks, publishes the tile's aggregate and takes its prefix as the staged copier does.  Then all
// four waves write the tile's column ranges output-stationary, as encode_kernel writes records: lane
// = aligned 16-byte output chunk, assembled from byte-unaligned 16-byte loads of the one or two
// fields it covers (more only under fields shorter than 16 bytes) under byte masks, one
// global_store_dwordx4 per chunk (byte stores only at a range's two edges).  kGU chunks per lane per
// step, every load of the step issued before its stores.  LDS holds only the field tables (~2 KB),
// so a CU keeps up to 8 copiers resident instead of 6.
constexpr int kGWin = 96;  // parse window bytes per record
constexpr int kGU = 4;     // output chunks per lane per step


template <int NV>
struct GatherLds {
    u64 addr[NV][kRecs];   // the tile's non-empty fields, compacted: source address
    int o[NV][kRecs + 1];  // output start inside the tile's column range; [nl] = the range length
    i64 pre[NV];           // the range's start in the column
    int hi[NV];            // bytes of the range to write (the capacity may cut it)
    int nl[NV];
    int nch[NV];           // output chunks of the range
    int first[NV];         // the first chunk's start relative to the range, in (-16, 0]
    int safe;              // every 16-byte window of the tile lies inside the stream's readable extent
    int skip;              // a range of 2 GiB or more (reported): nothing is written
};

template <int NF, int NV, bool MIX, int MODE = 0>
__global__ __launch_bounds__(kThreads) void decode_gather_kernel(DecodeParams p, u64* flags, u32 epoch) {
    static_assert(NV == 1 || NV == 2, "decode handles one or two string columns");
    constexpr int NW = kGWin / 4;
    __shared__ GatherLds<NV> S;
    __shared__ ScanLds SL;
    __shared__ MaskTable masks;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u64 n = p.n, ntiles = num_tiles(n);
    const uintptr_t in = (uintptr_t)p.in;
    const uintptr_t in_lo = in + p.rec_off[0];
    const uintptr_t in_end16 = (in + p.rec_off[n] + 15) & ~(uintptr_t)15;  // readable limit (ABI rule)
    u64* aw = flags;
    u64* pw = flags + (size_t)NV * ntiles;
    const u32 P = p.pipe_parsers;
    const bool forced = p.impl == kImplLookback;
    if (blockIdx.x < P) {
        if (!forced) parser<NF, NV, MIX, 2, 32>(p, aw, pw, ntiles, epoch, P);
        return;
    }
    if (blockIdx.x == P) {
        if (!forced) scanner<NV, kScanPerG>(aw, pw, ntiles, epoch, SL);
        return;
    }
    const u64 tile = blockIdx.x - P - 1;
    if (tile >= ntiles) return;
    mask_table_init(masks, tid);
    const u64 r0 = tile * kRecs;
    const int cnt = (int)min((u64)kRecs, n - r0);

    // ---- 1. parse from HBM (wave 0, lane = record), prefix, tables ----
    if (wave == 0) {
        const bool live = lane < cnt;
        const u64 start = p.rec_off[r0 + min(lane, cnt)];
        const u64 L = p.rec_off[r0 + min(lane + 1, cnt)] - start;
        const uintptr_t A = in + start;
        // the window: every 16-byte block that lies inside the readable extent (zero past it)
        u32 w[NW];
        const u64 room = in_end16 > A ? (u64)(in_end16 - A) : 0;
        const int wv = live ? (int)min((u64)kGWin, room) & ~15 : 0;  // window bytes loaded
#pragma unroll
        for (int k = 0; k < kGWin / 16; ++k) {
            const u32x4 a = ld16u(16 * k < wv ? A + 16 * k : (uintptr_t)flags);
            w[4 * k] = a.x;
            w[4 * k + 1] = a.y;
            w[4 * k + 2] = a.z;
            w[4 * k + 3] = a.w;
        }
        auto rd8 = [&](u64 q) -> u32 {
            constexpr u64 M = kGWin - 4;
            return q < (u64)wv ? (win_u32<NW>(w, (u32)min(q, M)) >> (8 * (q > M ? q - M : 0))) & 0xffu : ld_u8(A + q);
        };
        auto rd32 = [&](u64 q) -> u32 {
            return q + 4 <= (u64)wv ? win_u32<NW>(w, (u32)q) : *(gc_u32*)(A + q);  // unaligned OK
        };
        u32 st = 0;
        int32_t fx[NF > 0 ? NF : 1] = {};
        u64 flen[NV], fpos[NV];
#pragma unroll
        for (int f = 0; f < NV; ++f) flen[f] = fpos[f] = 0;
        const int nvr = rec_nvar<NV, MIX>(p, live ? r0 + lane : 0);
        if (live) {  // kv.syn.go:681-745, echo.syn.go:186-263
            if (L < 13) {
                st = SYM_STATUS_TOO_SHORT;
            } else if (rd8(0) != 0x01) {
                st = SYM_STATUS_BAD_VERSION;
            } else {
                const u64 off2p = rd32(1);
                if (off2p >= L || rd8(off2p) != 0x01) {
                    st = SYM_STATUS_NO_PRIVATE;
                } else {
                    const u64 pts = off2p + 1;
                    u64 toff = 0;
#pragma unroll
                    for (int f = 0; f < NF; ++f, toff += 4) {
                        if (st == 0) {
                            if (L < pts + toff + 4) st = SYM_STATUS_FIELD_TOO_SHORT;
                            else fx[f] = (int32_t)rd32(pts + toff);
                        }
                    }
                    if (st == 0) {
#pragma unroll
                        for (int f = 0; f < NV; ++f, toff += 4) {
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
            p.status[r0 + lane] = (uint8_t)st;
#pragma unroll
            for (int f = 0; f < NF; ++f) p.fixed[f][r0 + lane] = fx[f];
        }
        u64 agg[NV], excl[NV];
        bool too_large = false;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const u64 inc = wave_incl_scan_u32w_dpp((u32)flen[f]);
            agg[f] = (u64)__builtin_amdgcn_readlane((u32)inc, 63) |
                     ((u64)__builtin_amdgcn_readlane((u32)(inc >> 32), 63) << 32);
            excl[f] = inc - flen[f];
            too_large |= agg[f] >= ((u64)1 << 31);  // positions inside a tile's range are 32-bit
        }
        // the prefix: from the scanner, else (after kFallbackTicks, or forced) by look-back
        i64 pre[NV];
        if constexpr (MODE == 0) {
            u64 wvv = 0;
            bool got = true;
            if (lane < NV) {
                store_word(&aw[(size_t)lane * ntiles + tile], make_word(epoch, kStAgg, lane == 0 ? agg[0] : agg[NV - 1]));
                u64* a = &pw[(size_t)lane * ntiles + tile];
                wvv = load_word(a);
                if (!forced) {
                    for (const u64 t0 = now_ticks(); !tagged(wvv, epoch) && now_ticks() - t0 <= kFallbackTicks;) {
                        __builtin_amdgcn_s_sleep(2);
                        wvv = load_word(a);
                    }
                }
                got = tagged(wvv, epoch);
            }
            if (__ballot(!got)) {
                lookback<NF, NV, MIX>(p, aw, pw, ntiles, tile, epoch, pre);
#pragma unroll
                for (int f = 0; f < NV; ++f)
                    if (lane == 0) store_word(&pw[(size_t)f * ntiles + tile], make_word(epoch, kStPre, (u64)pre[f]));
            } else {
                pre[0] = (i64)((u64)__shfl((long long)wvv, 0, 64) & kValMask);
                if constexpr (NV == 2) pre[1] = (i64)((u64)__shfl((long long)wvv, 1, 64) & kValMask);
            }
        } else {  // timing only (wrong output): every prefix in proportion to the stream offset
            const double frac = (double)(start - p.rec_off[0]) / (double)(p.rec_off[n] - p.rec_off[0] + 1);
#pragma unroll
            for (int f = 0; f < NV; ++f) pre[f] = uniform_i64((i64)(__shfl(frac, 0, 64) * (double)p.cap[f]));
        }
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            if (live) p.offs[f][r0 + lane] = (u64)pre[f] + excl[f];
            if (lane == 0 && r0 + cnt == n) p.offs[f][n] = (u64)pre[f] + agg[f];
        }
        // the tables: non-empty fields compacted, each with its source and its output start
        bool safe = true;
#pragma unroll
        for (int f = 0; f < NV; ++f) {
            const bool ne = live && flen[f] > 0;
            const u64 m = __ballot(ne);
            const int slot = (int)__builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
            const uintptr_t src = A + fpos[f];
            if (ne) {
                S.addr[f][slot] = (u64)src;
                S.o[f][slot] = (int)excl[f];
                safe = safe && src >= in_lo + 16 && src + flen[f] + 16 <= in_end16 - 16;
            }
            if (lane == 0) {
                const int nl = (int)__popcll(m);
                S.o[f][nl] = (int)agg[f];
                S.nl[f] = nl;
                S.pre[f] = pre[f];
                const i64 cap = (i64)p.cap[f];
                if (MODE == 0 && agg[f] > 0 && pre[f] + (i64)agg[f] > cap) atomicOr(p.err, kErrCapacity);
                S.hi[f] = (int)max((i64)0, min((i64)agg[f], cap - pre[f]));
                const int first = -(int)(((uintptr_t)p.bytes[f] + (uintptr_t)pre[f]) & 15);
                S.first[f] = first;
                S.nch[f] = agg[f] > 0 ? (int)(((i64)agg[f] - first + 15) >> 4) : 0;
            }
        }
        const bool all_safe = __all(safe);
        if (lane == 0) {
            S.safe = all_safe;
            S.skip = __ballot(too_large) != 0;
            if (too_large) atomicOr(p.err, kErrTooLarge);
        }
    }
    __syncthreads();
    if (S.skip) return;

    // ---- 2. the column ranges, output-stationary (all lanes) ----
    const int n0 = S.nch[0];
    const int ntot = n0 + (NV == 2 ? S.nch[NV - 1] : 0);
    const bool safe = S.safe != 0;
    const uintptr_t dummy = (uintptr_t)flags;  // readable; its bytes are masked off
    for (int c0 = 0; c0 < ntot; c0 += kThreads * kGU) {  // uniform loop
        u32x4 r[kGU];
        int Pq[kGU], fq[kGU];
#pragma unroll
        for (int u = 0; u < kGU; ++u) {
            const int c = c0 + kThreads * u + tid;
            const int f = NV == 2 && c >= n0 ? 1 : 0;
            fq[u] = c < ntot ? f : -1;
            const int Pc = S.first[f] + 16 * (c - (f ? n0 : 0));
            Pq[u] = Pc;
            r[u] = u32x4{0, 0, 0, 0};
            if (c >= ntot) continue;
            const int nl = S.nl[f];
            const int k0 = lds_search_64(S.o[f], nl, max(Pc, 0));
            const int o0 = S.o[f][k0], o1 = S.o[f][k0 + 1];
            const bool two = k0 + 1 < nl && o1 < Pc + 16;  // the next field starts inside this chunk
            if (safe) {
                const int o2 = two ? S.o[f][k0 + 2] : o1;
                const uintptr_t X0 = (uintptr_t)(S.addr[f][k0] + (u64)(i64)(Pc - o0));
                const uintptr_t X1 = two ? (uintptr_t)(S.addr[f][k0 + 1] + (u64)(i64)(Pc - o1)) : dummy;
                r[u] = (ld16u(X0) & range_mask(masks, o0 - Pc, o1 - Pc)) |
                       (ld16u(X1) & range_mask(masks, two ? o1 - Pc : 16, o2 - Pc));
                for (int k = k0 + 2; two && k < nl && S.o[f][k] < Pc + 16; ++k)  // fields under 16 bytes
                    r[u] |= ld16u((uintptr_t)(S.addr[f][k] + (u64)(i64)(Pc - S.o[f][k]))) &
                            range_mask(masks, S.o[f][k] - Pc, S.o[f][k + 1] - Pc);
            } else {  // batch edges: aligned blocks holding valid bytes only
                u32 t[4] = {0, 0, 0, 0};
                for (int k = k0; k < nl && S.o[f][k] < Pc + 16; ++k) {
                    const int lo = S.o[f][k] - Pc, hi = S.o[f][k + 1] - Pc;
                    if (hi <= 0) continue;
                    or_window_global((uintptr_t)(S.addr[f][k] + (u64)(i64)(Pc - S.o[f][k])), max(lo, 0), min(hi, 16), t);
                }
                r[u] = u32x4{t[0], t[1], t[2], t[3]};
            }
        }
#pragma unroll
        for (int u = 0; u < kGU; ++u) {
            if (fq[u] < 0) continue;
            const int f = fq[u];
            const u32 rr[4] = {r[u].x, r[u].y, r[u].z, r[u].w};
            store_chunk(p.bytes[f] + S.pre[f], Pq[u], 0, S.hi[f], rr);
        }
    }
}

template <int NF, int NV, bool MIX, int MODE>
hipError_t launch_gather(const DecodeParams& p, u64* flags, u32 epoch, hipStream_t stream, int pnum, int pden) {
    static int cus[16] = {0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    int& ncu = cus[dev & 15];
    if (ncu == 0 && (e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    const u64 nt = num_tiles(p.n);
    u64 P = (u64)ncu * pnum / pden;
    if (P > (nt + 3) / 4) P = (nt + 3) / 4;
    DecodeParams q = p;
    q.pipe_parsers = (unsigned)P;
    hipLaunchKernelGGL((decode_gather_kernel<NF, NV, MIX, MODE>), dim3((unsigned)(P + 1 + nt)), dim3(kThreads), 0,
                       stream, q, flags, epoch);
    return hipGetLastError();
}

template <int MODE>
hipError_t launch_gather_layout(const DecodeParams& p, u64* flags, u32 epoch, hipStream_t stream, int pnum = 3,
                                int pden = 4) {
    if (p.type)
        return p.lay.nfixed == 0 && p.lay.nvar == 2 ? launch_gather<0, 2, true, MODE>(p, flags, epoch, stream, pnum, pden)
                                                     : hipErrorInvalidValue;
    if (p.lay.nfixed == 0 && p.lay.nvar == 1) return launch_gather<0, 1, false, MODE>(p, flags, epoch, stream, pnum, pden);
    if (p.lay.nfixed == 0 && p.lay.nvar == 2) return launch_gather<0, 2, false, MODE>(p, flags, epoch, stream, pnum, pden);
    if (p.lay.nfixed == 2 && p.lay.nvar == 2) return launch_gather<2, 2, false, MODE>(p, flags, epoch, stream, pnum, pden);
    return hipErrorInvalidValue;
}

template <int NF, int NV, bool MIX, int MODE, int DIAG, int SK = 4, int PR = 2, int STG = kStage, bool EARLY = false,
          int PACE = 0, bool XCDP = false, int AHEAD = 0, int NOP = 0, bool SPEC = false, int SPECX = 0, int WPE = 6,
          int UK = kU>
hipError_t launch(const DecodeParams& p, u64* flags, u32 epoch, hipStream_t stream, int pnum = 1, int pden = 1) {
    if (DIAG && !p.dbg) return hipErrorInvalidValue;  // timestamps need SYMHIP_DEBUG_PTR (tuning builds)
    static int cus[16] = {0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    int& ncu = cus[dev & 15];
    if (ncu == 0 && (e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    const u64 nt = num_tiles(p.n);
    constexpr bool kRoles = MODE == 0 || MODE == 2 || MODE == 3;
    u64 P = kRoles ? (u64)ncu * pnum / pden : 0;  // parser workgroups: pnum / pden per CU
    if (P > (nt + 3) / 4) P = (nt + 3) / 4;
    if (AHEAD > 0 && P > (u64)(AHEAD + 4 * PR - 1) / (4 * PR)) P = (AHEAD + 4 * PR - 1) / (4 * PR);  // tiles [0, AHEAD)
    DecodeParams q = p;
    q.pipe_parsers = (unsigned)P;
    const u64 grid = kRoles ? P + 1 + nt : nt;
    // speculative parsers: only kv layouts (no int32 fields) under the pipeline with its parsers
    constexpr bool kSpec = SPEC && NF == 0 && MODE == 0;
    if constexpr (kSpec) {
        if (p.impl != kImplLookback && P > 0) {
            hipLaunchKernelGGL((decode_pipe_kernel<NF, NV, MIX, MODE, DIAG, SK, PR, STG, EARLY, PACE, XCDP, AHEAD, NOP, true, SPECX, WPE, UK>),
                               dim3((unsigned)grid), dim3(kThreads), 0, stream, q, flags, epoch);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            if (SPECX == 1 || SPECX == 2) return hipSuccess;  // timing variants: no gate (WRONG on misfits)
            // four workgroups per CU (the gate's cost is the launch behind the first kernel, the same
            // for 1 or 4 per CU); a re-decode is the exact pipeline on them
            const u64 g = min(nt + 1 + ncu, (u64)ncu * (SPECX == 3 ? 1 : 4));
            hipLaunchKernelGGL((decode_gate_kernel<NF, NV, MIX>), dim3((unsigned)g), dim3(kThreads), 0, stream, q, flags, epoch);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((decode_pipe_kernel<NF, NV, MIX, MODE, DIAG, SK, PR, STG, EARLY, PACE, XCDP, AHEAD, NOP, false, 0, WPE, UK>), dim3((unsigned)grid),
                       dim3(kThreads), 0, stream, q, flags, epoch);
    return hipGetLastError();
}

constexpr int kParsersNum = 3;   // parser workgroups = #CUs * 3/4
constexpr int kParsersDen = 4;

template <int MODE, int DIAG, int SK = kScanPer, int PR = 2, int STG = kStage, bool EARLY = false, int PACE = 0,
          bool XCDP = false, int AHEAD = 0, int NOP = 0, bool SPEC = false, int SPECX = 0, int WPE = 6, int UK = kU>
hipError_t launch_layout(const DecodeParams& p, u64* flags, u32 epoch, hipStream_t stream, int pnum = kParsersNum,
                         int pden = kParsersDen) {
#define SYMHIP_PIPE_LAUNCH(NF, NV, MIX) \
    launch<NF, NV, MIX, MODE, DIAG, SK, PR, STG, EARLY, PACE, XCDP, AHEAD, NOP, SPEC, SPECX, WPE, UK>(p, flags, epoch, stream, pnum, pden)
    if (p.type)  // mixed kv batch: GetRequest / SetRequest per record
        return p.lay.nfixed == 0 && p.lay.nvar == 2 ? SYMHIP_PIPE_LAUNCH(0, 2, true) : hipErrorInvalidValue;
    if (p.lay.nfixed == 0 && p.lay.nvar == 1) return SYMHIP_PIPE_LAUNCH(0, 1, false);
    if (p.lay.nfixed == 0 && p.lay.nvar == 2) return SYMHIP_PIPE_LAUNCH(0, 2, false);
    if (p.lay.nfixed == 2 && p.lay.nvar == 2) return SYMHIP_PIPE_LAUNCH(2, 2, false);
#undef SYMHIP_PIPE_LAUNCH
    return hipErrorInvalidValue;
}

#ifdef SYMHIP_TUNING
// The persistent "ring" decode (tuning variants 500-512): an experiment measured against the pipeline
// above (decode section).
#include "decode_ring.inc"
#endif

}  // namespace pipe

size_t decode_pipe_flag_bytes(int nvar, uint64_t n) {
    // aggregate + prefix word per column and tile, then 256 bytes: the scanner's store sink
    // (pipe_words.hpp), then 256 bytes of control words (pipe::ctrl_words); the start doubles as the
    // kernels' filler load address
    return ((size_t)nvar * 2 * pipe::num_tiles(n) * sizeof(u64) + 512 + 255) & ~(size_t)255;
}

// The pipeline: 512-tile scanner steps, parsers on 3/4 of the CUs (tools/kbench.py sweep).
// Tuning builds (make tuning) add the measurement variants: 402 data movement only (copiers without
// the scan: WRONG output, a timing bound), 410 / 412 per-tile timestamps, 43x-46x geometry sweeps.
hipError_t launch_decode_pipe(const DecodeParams& p, void* flags, unsigned epoch, hipStream_t stream) {
    u64* fl = (u64*)flags;
#ifdef SYMHIP_TUNING
    switch (p.variant) {
        case 402: return pipe::launch_layout<1, 0>(p, fl, epoch, stream);
        case 410: return pipe::launch_layout<0, 1>(p, fl, epoch, stream);
        case 412: return pipe::launch_layout<1, 1>(p, fl, epoch, stream);
        case 431: return pipe::launch_layout<0, 0>(p, fl, epoch, stream, 1, 2);
        case 432: return pipe::launch_layout<0, 0>(p, fl, epoch, stream, 2, 1);
        case 433: return pipe::launch_layout<0, 0>(p, fl, epoch, stream, 1, 4);
        case 434: return pipe::launch_layout<0, 0>(p, fl, epoch, stream, 3, 2);
        case 440: return pipe::launch_layout<0, 0, 8>(p, fl, epoch, stream);
        case 443: return pipe::launch_layout<0, 0, 1>(p, fl, epoch, stream);
        case 446: return pipe::launch_layout<0, 0, 3>(p, fl, epoch, stream);
        case 447: return pipe::launch_layout<0, 0, 2>(p, fl, epoch, stream, 5, 8);
        case 449: return pipe::launch_layout<0, 0, 2>(p, fl, epoch, stream, 11, 16);
        case 460: return pipe::launch_layout<0, 0, 2, 1>(p, fl, epoch, stream);
        case 461: return pipe::launch_layout<0, 0, 2, 4>(p, fl, epoch, stream);
        // round 2: early prefix load, 7 copiers per CU (20992-byte stage), both
        case 470: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, true>(p, fl, epoch, stream);
        case 471: return pipe::launch_layout<0, 0, 2, 2, 20992, false>(p, fl, epoch, stream);
        case 472: return pipe::launch_layout<0, 0, 2, 2, 20992, true>(p, fl, epoch, stream);
        case 473: return pipe::launch_layout<0, 0, 2, 2, 20992, true>(p, fl, epoch, stream, 1, 2);
        case 474: return pipe::launch_layout<0, 0, 2, 2, 20992, true>(p, fl, epoch, stream, 1, 1);
        case 475: return pipe::launch_layout<1, 0, 2, 2, 20992, false>(p, fl, epoch, stream);
        case 476: return pipe::launch_layout<2, 0>(p, fl, epoch, stream);  // roles run, no waits (WRONG output)
        case 477: return pipe::launch_layout<0, 0>(p, fl, epoch, stream, 0, 1);  // no parsers
        case 478: return pipe::launch_layout<0, 0>(p, fl, epoch, stream, 1, 8);
        case 479: return pipe::launch_layout<0, 0>(p, fl, epoch, stream, 1, 4);
        case 480: return pipe::launch_layout<0, 0>(p, fl, epoch, stream, 1, 2);
        case 481: return pipe::launch_layout<0, 0, 2, 1>(p, fl, epoch, stream);
        case 482: return pipe::launch_layout<2, 0>(p, fl, epoch, stream, 0, 1);  // scanner only, no waits
        case 483: return pipe::launch_layout<3, 0>(p, fl, epoch, stream);  // parsers read offsets only, no waits
        case 484: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 2048>(p, fl, epoch, stream);
        case 485: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 4096>(p, fl, epoch, stream);
        case 486: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 8192>(p, fl, epoch, stream);
        case 487: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 4096>(p, fl, epoch, stream, 1, 2);
        case 488: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 0, true>(p, fl, epoch, stream);
        case 489: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 512, true>(p, fl, epoch, stream);
        case 490: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 1024, true>(p, fl, epoch, stream);
        case 491: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 2048, true>(p, fl, epoch, stream);
        case 492: return pipe::launch_layout<2, 0, 2, 2, pipe::kStage, false, 0, true>(p, fl, epoch, stream);
        // copiers parse ahead (AHEAD tiles; the parsers take only the first AHEAD tiles)
        case 620: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 0, false, 256>(p, fl, epoch, stream);
        case 621: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 0, false, 512>(p, fl, epoch, stream);
        case 622: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 0, false, 1024>(p, fl, epoch, stream);
        case 623: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 0, false, 2048>(p, fl, epoch, stream);
        case 624: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 0, false, 4096>(p, fl, epoch, stream);
        // round 3: the copier's parse replaced by the config-2 layout (timing bound of a parse-free copier)
        case 700: return pipe::launch_layout<0, 0, 2, 2, pipe::kStage, false, 0, false, 0, 1>(p, fl, epoch, stream);
        case 701: return pipe::launch_layout<1, 0, 2, 2, pipe::kStage, false, 0, false, 0, 1>(p, fl, epoch, stream);
        case 702: return pipe::launch_layout<2, 0, 2, 2, pipe::kStage, false, 0, false, 0, 1>(p, fl, epoch, stream);
        // round 3: exact parsers (no speculation, no gate): the round-2 default
        case 710: return pipe::launch_layout<0, 0>(p, fl, epoch, stream);
        // speculation without the copiers' check and the gate / with the check, no gate / gate on one
        // workgroup per CU (711 and 712 are WRONG on batches the speculation misses)
        case 711: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true, 1>(p, fl, epoch, stream);
        case 712: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true, 2>(p, fl, epoch, stream);
        case 713: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true, 3>(p, fl, epoch, stream);
        // round 3: the speculative default with an early prefix load and / or a 20992-byte stage
        case 720: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, true, 0, false, 0, 0, true>(p, fl, epoch, stream);
        case 721: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, 20992, true, 0, false, 0, 0, true>(p, fl, epoch, stream);
        case 722: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, 20992, false, 0, false, 0, 0, true>(p, fl, epoch, stream);
        case 723: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 2);
        case 724: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 1);
        case 725: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 4);
        case 726: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 3, 8);
        case 727: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 5, 8);
        case 728: return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 8);
        // speculative parsers on half the CUs: scanner tiles per thread 1 / 4, parser tiles per wave step 4 / 1
        case 730: return pipe::launch_layout<0, 0, 1, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 2);
        case 731: return pipe::launch_layout<0, 0, 4, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 2);
        case 732: return pipe::launch_layout<0, 0, pipe::kScanPer, 4, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 2);
        case 733: return pipe::launch_layout<0, 0, pipe::kScanPer, 1, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 2);
        // round 4: 8 waves per SIMD (<= 64 VGPRs) with a 16 KiB stage (8 copiers per CU by LDS), with the
        // speculative default's geometry; 742: copiers only at 8 per CU (WRONG output); 743: the 16 KiB
        // stage at 6 waves per SIMD
        case 740: return pipe::launch_layout<0, 0, 1, 2, 16384, false, 0, false, 0, 0, true, 0, 8>(p, fl, epoch, stream, 1, 2);
        case 742: return pipe::launch_layout<1, 0, 1, 2, 16384, false, 0, false, 0, 0, true, 0, 8>(p, fl, epoch, stream, 1, 2);
        case 743: return pipe::launch_layout<0, 0, 1, 2, 16384, false, 0, false, 0, 0, true, 0, 6>(p, fl, epoch, stream, 1, 2);
        // round 4: copy chunks per lane per step 3 / 4 (default stage), and with the 8-wave 16 KiB stage
        case 744: return pipe::launch_layout<0, 0, 1, 2, pipe::kStage, false, 0, false, 0, 0, true, 0, 6, 3>(p, fl, epoch, stream, 1, 2);
        case 745: return pipe::launch_layout<0, 0, 1, 2, pipe::kStage, false, 0, false, 0, 0, true, 0, 6, 4>(p, fl, epoch, stream, 1, 2);
        case 746: return pipe::launch_layout<0, 0, 1, 2, 16384, false, 0, false, 0, 0, true, 0, 8, 3>(p, fl, epoch, stream, 1, 2);
        // the gather copier (no LDS stage, output-stationary copy); 601: its timing mode (WRONG output)
        case 600: return pipe::launch_gather_layout<0>(p, fl, epoch, stream);
        case 601: return pipe::launch_gather_layout<1>(p, fl, epoch, stream);
        case 602: return pipe::launch_gather_layout<0>(p, fl, epoch, stream, 1, 2);
        case 603: return pipe::launch_gather_layout<0>(p, fl, epoch, stream, 1, 1);
        // the ring decode: lead 3 / 4, barrier / one-wave scanner; 51x: with timestamps
        case 500: return pipe::launch_ring_layout<0, 3, 0>(p, fl, epoch, stream);
        case 501: return pipe::launch_ring_layout<0, 3, 1>(p, fl, epoch, stream);
        case 502: return pipe::launch_ring_layout<0, 4, 0>(p, fl, epoch, stream);
        case 503: return pipe::launch_ring_layout<0, 4, 1>(p, fl, epoch, stream);
        case 504: return pipe::launch_ring_layout<0, 3, 2>(p, fl, epoch, stream);  // no scan (WRONG output)
        case 510: return pipe::launch_ring_layout<1, 3, 0>(p, fl, epoch, stream);
        case 512: return pipe::launch_ring_layout<1, 4, 0>(p, fl, epoch, stream);
        default: break;
    }
#endif
    // speculative parsers are lighter: half the CUs' worth of them keeps ahead of the copiers, and the
    // scanner's 256-tile steps publish sooner (sweeps with configs 2, 3 and the mixed batch,
    // DESIGN.md); exact parsers (int32 fields) keep 3/4 of the CUs and 512-tile steps
    if (p.lay.nfixed == 0)
        return pipe::launch_layout<0, 0, 1, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream, 1, 2);
    return pipe::launch_layout<0, 0, pipe::kScanPer, 2, pipe::kStage, false, 0, false, 0, 0, true>(p, fl, epoch, stream);
}

}  // namespace symhip
