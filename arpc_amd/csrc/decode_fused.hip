// decode_fused.hip -- EXPERIMENTAL single-pass Symphony UnmarshalSymphony on gfx950 (decode variants
// >= 400; the default decode is the three-kernel path in decode.hip -- DESIGN.md section 4 has the
// measurements that decided it).
//
// Same semantics as decode.hip (the per-record unmarshaller into a fresh struct,
// benchmark/kv-store-symphony/symphony/kv.syn.go:680-745; echo.syn.go:186-263 for int32 fields;
// generator cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:622-694, :734-793), in ONE pass over
// the stream: every stream byte is fetched from HBM once.
//
// Design (persistent workgroups, one 64-record tile at a time, tiles round-robin over the grid):
//  1. stage: the tile's byte span is loaded into LDS with aligned, coalesced 16-byte loads (up to
//     kStage bytes; a longer span's tail stays in HBM and is read from there).
//  2. parse (wave 0, lane = record): Go's header checks and per-field bounds checks (64-bit
//     arithmetic, as Go's int) read the staged bytes; writes the status byte and int32 fields.
//     A DPP scan of the field lengths gives each record's position inside the tile's column range.
//  3. look-back (wave 0): the tile's column aggregates are published as 8-byte {epoch, status,
//     value} words (the word is the flag: agent-scope relaxed atomics, MI355X_MICROARCH.md
//     visibility "R2"), then predecessors' words are summed back to the nearest inclusive prefix,
//     64 words per lane-group step.  Writes the output offsets.
//  4. copy (all 256 lanes): every field is a run of 16-byte chunks (the last one moved back to end
//     at the field end), each one byte-unaligned LDS read (or HBM load past the staged span) and
//     one 16-byte store.
// The grid is sized to the co-resident capacity, so a tile only ever waits on tiles already held
// by running workgroups (launched cooperatively where the runtime allows, which guarantees it).
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

namespace fused {

constexpr int kRecs = 64;       // records per tile
constexpr int kThreads = 256;   // 4 waves
constexpr int kStage = 22528;   // staged bytes per tile: a whole 64-record tile of 350-B records
constexpr int kStageLoads = (kStage / 16 + kThreads - 1) / kThreads;
constexpr int kLW = 8;          // look-back words per lane per step

// Look-back word: [63:44] epoch, [43:42] status (1 = aggregate, 2 = inclusive prefix), [41:0] value.
constexpr int kEpochShift = 44;
constexpr u64 kStAgg = 1ull << 42;
constexpr u64 kStInc = 2ull << 42;
constexpr u64 kValMask = (1ull << 42) - 1;
constexpr unsigned kSpinLimit = 1u << 21;

__host__ __device__ inline u64 num_tiles(u64 n) { return (n + kRecs - 1) / kRecs; }

template <int NV>
struct alignas(16) Lds {
    uint8_t stage[kStage + 16];
    u64 src[NV][kRecs];        // field payload position (stream offset)
    int dst[NV][kRecs + 1];    // field start in the tile's column range; [cnt..] = aggregate
    int cs[kRecs + 1];         // record's first copy chunk (record-major chunk sequence)
    int nch0[kRecs];           // chunks of the record's first string field
    i64 pre[NV];               // tile prefix per column
    i64 lim[NV];               // bytes of the tile's column range that fit the output capacity
    int total;                 // chunks in the tile (-1: tile skipped, error reported)
    u64 agg[NV];               // tile aggregate per column (workgroup look-back input)
    u64 red[4];                // per-wave partial sums (workgroup look-back)
    int first[4];              // per-wave first inclusive lane (workgroup look-back)
};

__device__ __forceinline__ int word_status(u64 w, u32 epoch) {
    return (u32)(w >> kEpochShift) == epoch ? (int)((w >> 42) & 3) : 0;
}
__device__ __forceinline__ u64 make_word(u32 epoch, u64 st, u64 v) { return ((u64)epoch << kEpochShift) | st | v; }
__device__ __forceinline__ void store_word(u64* w, u64 v) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 load_word(u64* w) {
    return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Decoupled look-back for NV columns, run by one full wave: lanes [h*HL, (h+1)*HL) serve column h,
// each lane checking kLW predecessors, so one step covers HL*kLW tiles per column.  Publishes the
// tile's aggregate first and its inclusive prefix last; returns column `lane / HL`'s exclusive
// prefix in every lane of that column's group.
// Workgroup barrier that orders LDS only: outstanding global stores keep flying (__syncthreads()
// would wait for them).  Global loads whose data is used were waited on at their use.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NV>
__device__ u64 lookback(u64* flags, u64 ntiles, u64 tile, u64 agg, u32 epoch, unsigned* err, int lane) {
    constexpr int HL = 64 / NV;
    const int h = lane / HL, hl = lane % HL;
    u64* words = flags + (size_t)h * ntiles;
    if (tile == 0) {
        if (hl == 0) store_word(&words[0], make_word(epoch, kStInc, agg));
        return 0;
    }
    if (hl == 0) store_word(&words[tile], make_word(epoch, kStAgg, agg));
    u64 excl = 0;
    bool done = false;
    i64 base = (i64)tile - 1 - (i64)hl * kLW;
    for (;;) {
        u64 part = 0;
        bool inc = false;
        if (!done) {
            u64 w[kLW];
#pragma unroll
            for (int k = 0; k < kLW; ++k)
                w[k] = base - k >= 0 ? load_word(&words[base - k]) : make_word(epoch, kStInc, 0);
            unsigned spins = 0;
            for (;;) {
                bool pending = false;
#pragma unroll
                for (int k = 0; k < kLW; ++k) pending |= word_status(w[k], epoch) == 0;
                if (!pending) break;
                if (++spins >= kSpinLimit) {  // report and stop waiting so the grid drains
                    atomicOr(err, kErrTimeout);
#pragma unroll
                    for (int k = 0; k < kLW; ++k)
                        if (word_status(w[k], epoch) == 0) w[k] = make_word(epoch, kStInc, 0);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
#pragma unroll
                for (int k = 0; k < kLW; ++k)
                    if (word_status(w[k], epoch) == 0) w[k] = load_word(&words[base - k]);
            }
#pragma unroll
            for (int k = 0; k < kLW; ++k) {
                if (!inc) part += w[k] & kValMask;
                inc |= word_status(w[k], epoch) == 2;
            }
        }
        const u64 incs = __ballot(inc);
        const u64 mine = NV == 2 ? (h ? incs >> 32 : incs & 0xffffffffull) : incs;
        const int pl = mine ? __ffsll((long long)mine) - 1 : HL - 1;
        const u64 s = wave_incl_scan_u64(!done && hl <= pl ? part : 0, lane);
        const u64 s_lo = (u64)__shfl((long long)s, HL - 1, 64);
        if (!done) excl += (NV == 2 && h) ? (u64)__shfl((long long)s, 63, 64) - s_lo : s_lo;
        else (void)__shfl((long long)s, 63, 64);  // keep the shuffle wave-uniform
        done = done || mine != 0;
        if (__ballot(!done) == 0) break;
        base -= (i64)HL * kLW;
    }
    if (hl == 0) store_word(&words[tile], make_word(epoch, kStInc, (excl + agg) & kValMask));
    return excl;
}

// In-round hierarchical scan (the default).  The grid is persistent: round i is tiles [iG, iG+G),
// tile iG+w belongs to workgroup w.  Tiles form groups of 64 consecutive tiles.  Every tile
//   1. publishes its aggregate, then loads its group's 64 aggregates (one word per lane):
//      its in-group prefix and the group total; the group's first tile publishes that total;
//   2. loads the round's group totals (<= 64 groups, G <= 4096): its groups' prefix and the
//      round total.
// The round totals advance a carry that every workgroup keeps for itself, so no tile ever waits
// on another round and no chain runs through the round: two dependent round trips per tile.
template <int NV>
__device__ __forceinline__ void wait_tagged(u64 (&v)[NV], u64* const (&addr)[NV], bool ex, u64 fill, u32 epoch,
                                            unsigned* err, int lane) {
    for (unsigned spins = 0;;) {
        bool pend = false;
#pragma unroll
        for (int f = 0; f < NV; ++f) pend |= ex && word_status(v[f], epoch) == 0;
        if (!__ballot(pend)) break;
        if (++spins >= kSpinLimit) {  // report and stop waiting so the grid drains
            if (lane == 0) atomicOr(err, kErrTimeout);
#pragma unroll
            for (int f = 0; f < NV; ++f)
                if (word_status(v[f], epoch) == 0) v[f] = fill;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int f = 0; f < NV; ++f)
            if (ex && word_status(v[f], epoch) == 0) v[f] = load_word(addr[f]);
    }
}

template <int NV>
__device__ void round_scan(u64* aw, u64* gw, u64 ntiles, u64 tile, u32 G, const u64 (&agg)[NV], u32 epoch,
                           unsigned* err, int lane, u64 (&carry)[NV], u64 (&pre)[NV]) {
    const u64 round = tile / G;
    const u32 w = (u32)(tile - round * G);
    const u64 rbase = round * G;
    const u64 rend = min(rbase + G, ntiles);
    const u32 NG = (G + 63) / 64;
    const u64 ngt = ((ntiles + G - 1) / G) * NG;  // group-total words per column
    const u32 g = w / 64, wi = w % 64;
    const u32 ngv = (u32)((rend - rbase + 63) / 64);
    if (lane < NV) {
        const u64 a = lane == 0 ? agg[0] : agg[NV - 1];
        store_word(&aw[(size_t)lane * ntiles + tile], make_word(epoch, kStAgg, a));
    }
    // ---- step 1: the group's aggregates ----
    const u64 t = rbase + 64 * (u64)g + lane;
    const bool ex = t < rend;
    u64 v[NV];
    u64* addr[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        addr[f] = &aw[(size_t)f * ntiles + (ex ? t : 0)];
        v[f] = ex ? load_word(addr[f]) : make_word(epoch, kStAgg, 0);
    }
    wait_tagged<NV>(v, addr, ex, make_word(epoch, kStAgg, 0), epoch, err, lane);
    u64 mine[NV];
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u64 x = v[f] & kValMask;
        const u64 s = wave_incl_scan_u64(x, lane);
        const u64 tot = (u64)__shfl((long long)s, 63, 64);
        mine[f] = (u64)__shfl((long long)(s - x), (int)wi, 64);
        if (wi == 0 && lane == 0) store_word(&gw[(size_t)f * ngt + round * NG + g], make_word(epoch, kStInc, tot));
    }
    // ---- step 2: the round's group totals ----
    const bool exg = (u32)lane < ngv;
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        addr[f] = &gw[(size_t)f * ngt + round * NG + (exg ? lane : 0)];
        v[f] = exg ? load_word(addr[f]) : make_word(epoch, kStInc, 0);
    }
    wait_tagged<NV>(v, addr, exg, make_word(epoch, kStInc, 0), epoch, err, lane);
#pragma unroll
    for (int f = 0; f < NV; ++f) {
        const u64 x = v[f] & kValMask;
        const u64 s = wave_incl_scan_u64(x, lane);
        const u64 tot = (u64)__shfl((long long)s, 63, 64);
        const u64 before = g ? (u64)__shfl((long long)s, (int)g - 1, 64) : 0;
        pre[f] = carry[f] + before + mine[f];
        carry[f] += tot;
    }
}

// Decoupled look-back run by the whole workgroup (the waves are otherwise idle here): column h
// is served by threads [h*HL, (h+1)*HL), each checking kWL predecessors, so one step covers
// HL*kWL = 1024 tiles per column -- wide enough that a tile finds an inclusive prefix in one step
// even when ~1500 tiles are in flight.  Reads S.agg, writes S.pre (the tile's exclusive prefixes).
template <int NV, typename LdsT>
__device__ void wg_lookback(u64* flags, u64 ntiles, u64 tile, LdsT& S, u32 epoch, unsigned* err, int tid) {
    constexpr int HL = kThreads / NV;
    constexpr int kWL = 1024 / HL;
    constexpr int WPC = HL / 64;  // waves per column
    const int h = tid / HL, hl = tid % HL, lane = tid & 63, wave = tid >> 6;
    u64* words = flags + (size_t)h * ntiles;
    const u64 agg = S.agg[h];
    if (tile == 0) {
        if (hl == 0) {
            store_word(&words[0], make_word(epoch, kStInc, agg));
            S.pre[h] = 0;
        }
        return;
    }
    if (hl == 0) store_word(&words[tile], make_word(epoch, kStAgg, agg));
    u64 excl = 0;
    bool done = false;  // uniform per column
    i64 base = (i64)tile - 1 - (i64)hl * kWL;
    for (;;) {
        u64 part = 0;
        bool inc = false;
        if (!done) {
            u64 w[kWL];
#pragma unroll
            for (int k = 0; k < kWL; ++k)
                w[k] = base - k >= 0 ? load_word(&words[base - k]) : make_word(epoch, kStInc, 0);
            // wait for this lane's words up to (and including) its nearest inclusive one
            for (unsigned spins = 0;;) {
                bool pending = false, seen_inc = false;
#pragma unroll
                for (int k = 0; k < kWL; ++k) {
                    const int st = word_status(w[k], epoch);
                    pending |= !seen_inc && st == 0;
                    seen_inc |= st == 2;
                }
                if (!pending) break;
                if (++spins >= kSpinLimit) {  // report and stop waiting so the grid drains
                    atomicOr(err, kErrTimeout);
#pragma unroll
                    for (int k = 0; k < kWL; ++k)
                        if (word_status(w[k], epoch) == 0) w[k] = make_word(epoch, kStInc, 0);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int k = 0; k < kWL; ++k)
                    if (word_status(w[k], epoch) == 0) w[k] = load_word(&words[base - k]);
            }
#pragma unroll
            for (int k = 0; k < kWL; ++k) {
                if (!inc) part += w[k] & kValMask;
                inc |= word_status(w[k], epoch) == 2;
            }
        }
        // first lane of the column holding an inclusive word, then the sum of parts up to it
        const u64 b = __ballot(inc);
        if (lane == 0) S.first[wave] = b ? (wave % WPC) * 64 + __ffsll((long long)b) - 1 : HL;
        lds_barrier();
        int pl = HL;
#pragma unroll
        for (int q = 0; q < WPC; ++q) pl = min(pl, S.first[h * WPC + q]);
        const u64 ws = wave_sum_u64(!done && hl <= pl ? part : 0);
        if (lane == 0) S.red[wave] = ws;
        lds_barrier();
        u64 colsum = 0;
#pragma unroll
        for (int q = 0; q < WPC; ++q) colsum += S.red[h * WPC + q];
        if (!done) excl += colsum;
        done = done || pl < HL;
        bool all_done = done;
        // every thread must agree on when to stop: publish per-column done flags
        if (hl == 0) S.first[h * WPC] = done ? -1 : 0;  // reuse: -1 = column done
        lds_barrier();
#pragma unroll
        for (int c = 0; c < NV; ++c) all_done = all_done && S.first[c * WPC] == -1;
        lds_barrier();  // S.first is rewritten by the next step
        if (all_done) break;
        base -= (i64)HL * kWL;
    }
    if (hl == 0) {
        store_word(&words[tile], make_word(epoch, kStInc, (excl + agg) & kValMask));
        S.pre[h] = (i64)excl;
    }
}

// SCAN: 0 = round_scan, 1 = decoupled look-back, 2 = none (timing only, wrong output).
// DIAG (timing diagnostics only, tools/fused_timeline.py): per-tile phase timestamps into p.dbg
// (8 u64 per tile, s_memrealtime at 100 MHz).
template <int NF, int NV, int kU, int SCAN = 0, int DIAG = 0>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(6, 8))) void decode_fused_kernel(DecodeParams p, u64* flags, u32 epoch) {
    static_assert(NV == 1 || NV == 2, "decode handles one or two string columns");
    __shared__ Lds<NV> S;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u64 n = p.n, ntiles = num_tiles(n);
    const uintptr_t in = (uintptr_t)p.in;
    // readable limit of the stream: the 16-byte boundary past its last byte (ABI memory rule)
    const uintptr_t in_end16 = (in + p.rec_off[n] + 15) & ~(uintptr_t)15;
    const uintptr_t in_last = in_end16 - 16;
    const uintptr_t safe = (uintptr_t)flags;  // readable filler address for lanes with nothing to load

    u64 carry[NV];  // wave 0: column totals of all earlier rounds (round_scan)
#pragma unroll
    for (int f = 0; f < NV; ++f) carry[f] = 0;
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
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
        const int nst = (int)min((u64)kStage, (u64)(stop > base ? stop - base : 0));  // multiple of 16

        // ---- 1. stage (and wave 0's record offsets) ----
        u64 start = 0, endv = 0;
        if (wave == 0) {
            start = p.rec_off[r0 + min(lane, cnt)];
            endv = p.rec_off[r0 + min(lane + 1, cnt)];
        }
        {
            u32x4 sv[kStageLoads];
#pragma unroll
            for (int k = 0; k < kStageLoads; ++k) {
                const int c = tid + kThreads * k;
                sv[k] = ld16u(16 * c < nst ? base + 16 * (uintptr_t)c : safe);
            }
#pragma unroll
            for (int k = 0; k < kStageLoads; ++k) {
                const int c = tid + kThreads * k;
                if (16 * c < nst) *(u32x4*)&S.stage[16 * c] = sv[k];
            }
        }
        lds_barrier();
        stamp(1);

        // ---- 2. parse + 3. look-back (wave 0) ----
        // wave 0's per-record parse results (live across the workgroup look-back's barriers)
        u64 agg[NV], excl[NV];
        u32 nch[NV];
        bool too_large = false;
        i64 pre[NV];
        const bool live = lane < cnt;
        if (wave == 0) {
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
            if (live) {
                if (L < 13) {
                    st = 1;  // "invalid data: too short"
                } else if (rd8(0) != 0x01) {
                    st = 2;  // "invalid data: wrong public version"
                } else {
                    const u64 off2p = rd32(1);
                    if (off2p >= L || rd8(off2p) != 0x01) {
                        st = 3;  // "missing private segment"
                    } else {
                        const u64 pts = off2p + 1;
                        u64 toff = 0;
#pragma unroll
                        for (int f = 0; f < NF; ++f, toff += 4) {
                            if (st == 0) {
                                if (L < pts + toff + 4) st = 4;  // "invalid data: too short for field"
                                else fx[f] = (int32_t)rd32(pts + toff);
                            }
                        }
                        if (st == 0) {
#pragma unroll
                            for (int f = 0; f < NV; ++f, toff += 4) {
                                if (L >= pts + toff + 4) {
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
            // tile scan of the field lengths (each < 2^32)
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
            // look-back: the lane group of column h carries column h's aggregate
            stamp(2);
            if constexpr (SCAN == 3) {  // workgroup look-back below
                if (lane == 0)
#pragma unroll
                    for (int f = 0; f < NV; ++f) S.agg[f] = agg[f];
            } else if constexpr (SCAN == 1) {  // decoupled look-back (comparison variant)
                u64 my_agg = agg[0];
                if constexpr (NV == 2) my_agg = lane >= 32 ? agg[1] : agg[0];
                const u64 ex = lookback<NV>(flags, ntiles, tile, my_agg, epoch, p.err, lane);
                pre[0] = (i64)__shfl((long long)ex, 0, 64);
                if constexpr (NV == 2) pre[1] = (i64)__shfl((long long)ex, 32, 64);
            } else if constexpr (SCAN == 0) {
                u64 pr[NV];
                round_scan<NV>(flags, flags + (size_t)NV * ntiles, ntiles, tile, gridDim.x, agg, epoch, p.err, lane,
                               carry, pr);
#pragma unroll
                for (int f = 0; f < NV; ++f) pre[f] = (i64)pr[f];
            } else if constexpr (SCAN == 4) {  // tile prefixes from the measure + scan kernels
#pragma unroll
                for (int f = 0; f < NV; ++f) pre[f] = (i64)p.tile_pre[(size_t)f * ntiles + tile];
            } else {  // timing only: no scan (wrong output)
#pragma unroll
                for (int f = 0; f < NV; ++f) pre[f] = 0;
            }
        }
        if constexpr (SCAN == 3) {
            lds_barrier();
            wg_lookback<NV>(flags, ntiles, tile, S, epoch, p.err, tid);
            lds_barrier();
        }
        if (wave == 0) {
            if constexpr (SCAN == 3)
#pragma unroll
                for (int f = 0; f < NV; ++f) pre[f] = S.pre[f];
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
                    if (agg[f] > 0 && pre[f] + (i64)agg[f] > cap) atomicOr(p.err, kErrCapacity);
                    S.lim[f] = max((i64)0, min((i64)agg[f], cap - pre[f]));
                }
                S.total = too_large ? -1 : T;
            }
            if (__ballot(too_large) && lane == 0) atomicOr(p.err, kErrTooLarge);
        }
        lds_barrier();

        // ---- 4. copy (all lanes) ----
        const int T = __builtin_amdgcn_readfirstlane(S.total);
        // per-column values as named scalars: a two-element array indexed by a lane value is
        // lowered to scratch
        const i64 pre0 = uniform_i64(S.pre[0]), pre1 = uniform_i64(S.pre[NV - 1]);
        const i64 lim0 = uniform_i64(S.lim[0]), lim1 = uniform_i64(S.lim[NV - 1]);
        const uintptr_t stage_end = base + (uintptr_t)nst;
        for (int c0 = 0; c0 < T; c0 += kThreads * kU) {  // uniform loop
            u32x4 v[kU];
            int P[kU], code[kU];
            uintptr_t X[kU];
            bool glob[kU];
            bool anyg = false;
#pragma unroll
            for (int u = 0; u < kU; ++u) {
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
                P[u] = has ? dk + off : -1;
                code[u] = min(L, 16) | (second ? 1 << 10 : 0);
                v[u] = has && !glob[u] ? lds16u(S.stage, (int)(X[u] - base)) : u32x4{0, 0, 0, 0};
            }
            if (__ballot(anyg)) {  // past the staged span: HBM loads, all issued before any use
                u32x4 g[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const uintptr_t Xc = X[u] < in_last ? X[u] : in_last;
                    g[u] = ld16u(glob[u] ? Xc : safe);
                    code[u] |= glob[u] ? (int)((X[u] - Xc) << 5) : 0;
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
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
            for (int u = 0; u < kU; ++u) {
                const bool second = (code[u] >> 10) & 1;
                const int nb = code[u] & 31;
                const i64 hi = min((i64)(P[u] + nb), second ? lim1 : lim0);
                uint8_t* colb = second ? p.bytes[NV - 1] + pre1 : p.bytes[0] + pre0;
                const bool full = P[u] >= 0 && (i64)P[u] + 16 <= hi;
                if (full) *(g_u4*)(colb + P[u]) = v[u];
                const bool part = P[u] >= 0 && !full && (i64)P[u] < hi;
                if (__ballot(part)) {
                    const u32 rr[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                    if (part) store_chunk(colb, P[u], 0, hi, rr);
                }
            }
        }
        lds_barrier();  // LDS is restaged by the next tile (the copy's stores need not drain)
        stamp(4);
        if constexpr (DIAG)
            if (tid == 0) p.dbg[tile * 8 + 5] = blockIdx.x;
    }
}

template <int NF, int NV, int kU, int SCAN = 0, int DIAG = 0>
hipError_t launch(const DecodeParams& p, u64* flags, u32 epoch, hipStream_t stream, bool coop, bool persistent = true) {
    if (!persistent) {  // one workgroup per tile, in tile order
        if (SCAN == 0) return hipErrorInvalidValue;  // round_scan needs the persistent grid
        hipLaunchKernelGGL((decode_fused_kernel<NF, NV, kU, SCAN, DIAG>), dim3((unsigned)num_tiles(p.n)),
                           dim3(kThreads), 0, stream, p, flags, epoch);
        return hipGetLastError();
    }
    static int max_blocks[8] = {0};  // co-resident workgroups per device (occupancy x CUs)
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const int slot = dev & 7;
    // one cache per template instance: the query is per kernel
    if (max_blocks[slot] == 0) {
        int per_cu = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_fused_kernel<NF, NV, kU, SCAN, DIAG>, kThreads, 0);
        if (e != hipSuccess) return e;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        max_blocks[slot] = per_cu * cus > 0 ? per_cu * cus : 1;
    }
    const u64 ntiles = num_tiles(p.n);
    u64 grid64 = ntiles < (u64)max_blocks[slot] ? ntiles : (u64)max_blocks[slot];
    if (grid64 > 4096) grid64 = 4096;  // round_scan: at most 64 groups of 64 tiles per round
    const unsigned grid = (unsigned)grid64;
    if (coop) {
        DecodeParams pp = p;
        void* args[] = {&pp, &flags, &epoch};
        return hipLaunchCooperativeKernel((const void*)decode_fused_kernel<NF, NV, kU, SCAN, DIAG>, dim3(grid), dim3(kThreads),
                                          args, 0, stream);
    }
    hipLaunchKernelGGL((decode_fused_kernel<NF, NV, kU, SCAN, DIAG>), dim3(grid), dim3(kThreads), 0, stream, p, flags, epoch);
    return hipGetLastError();
}

}  // namespace fused

size_t decode_fused_flag_bytes(int nvar, uint64_t n) {
    // per column: ntiles aggregate words + at most ntiles/64 + rounds + 64 group-total words (G <= 4096)
    const size_t t = fused::num_tiles(n);
    return ((size_t)nvar * (2 * t + 130) * sizeof(u64) + 256 + 255) & ~(size_t)255;  // >= 256: the filler address
}

hipError_t launch_decode_fused(const DecodeParams& p, void* flags, unsigned epoch, hipStream_t stream) {
    u64* fl = (u64*)flags;
    // variants: 0/400 round_scan; 401 decoupled look-back; 402 no scan (timing only);
    // +10 per-tile timestamps; +100 non-cooperative launch; 404 four chunks per lane per step
    int v = p.variant;
    if (v >= 600) {  // one workgroup per tile (not persistent): decoupled look-back in tile order
        switch (v) {
            case 610:
#define SYM_NP(NF, NV) return fused::launch<NF, NV, 2, 1, 1>(p, fl, epoch, stream, false, false)
                if (p.lay.nfixed == 0 && p.lay.nvar == 1) SYM_NP(0, 1);
                if (p.lay.nfixed == 0 && p.lay.nvar == 2) SYM_NP(0, 2);
                if (p.lay.nfixed == 2 && p.lay.nvar == 2) SYM_NP(2, 2);
                return hipErrorInvalidValue;
#undef SYM_NP
            case 620:
#define SYM_NP(NF, NV) return fused::launch<NF, NV, 2, 3, 0>(p, fl, epoch, stream, false, false)
                if (p.lay.nfixed == 0 && p.lay.nvar == 1) SYM_NP(0, 1);
                if (p.lay.nfixed == 0 && p.lay.nvar == 2) SYM_NP(0, 2);
                if (p.lay.nfixed == 2 && p.lay.nvar == 2) SYM_NP(2, 2);
                return hipErrorInvalidValue;
#undef SYM_NP
            case 630:
#define SYM_NP(NF, NV) return fused::launch<NF, NV, 2, 3, 1>(p, fl, epoch, stream, false, false)
                if (p.lay.nfixed == 0 && p.lay.nvar == 1) SYM_NP(0, 1);
                if (p.lay.nfixed == 0 && p.lay.nvar == 2) SYM_NP(0, 2);
                if (p.lay.nfixed == 2 && p.lay.nvar == 2) SYM_NP(2, 2);
                return hipErrorInvalidValue;
#undef SYM_NP
            default:
#define SYM_NP(NF, NV) return fused::launch<NF, NV, 2, 1, 0>(p, fl, epoch, stream, false, false)
                if (p.lay.nfixed == 0 && p.lay.nvar == 1) SYM_NP(0, 1);
                if (p.lay.nfixed == 0 && p.lay.nvar == 2) SYM_NP(0, 2);
                if (p.lay.nfixed == 2 && p.lay.nvar == 2) SYM_NP(2, 2);
                return hipErrorInvalidValue;
#undef SYM_NP
        }
    }
    const bool coop = v < 500;
    if (!coop) v -= 100;
#define SYM_FUSED(NF, NV)                                                                          \
    switch (v) {                                                                                   \
        case 401: return fused::launch<NF, NV, 2, 1>(p, fl, epoch, stream, coop);                 \
        case 402: return fused::launch<NF, NV, 2, 2>(p, fl, epoch, stream, coop);                 \
        case 404: return fused::launch<NF, NV, 4, 0>(p, fl, epoch, stream, coop);                 \
        case 407: return fused::launch<NF, NV, 2, 4>(p, fl, epoch, stream, coop);                 \
        case 417: return fused::launch<NF, NV, 2, 4, 1>(p, fl, epoch, stream, coop);              \
        case 410: return fused::launch<NF, NV, 2, 0, 1>(p, fl, epoch, stream, coop);              \
        case 411: return fused::launch<NF, NV, 2, 1, 1>(p, fl, epoch, stream, coop);              \
        case 412: return fused::launch<NF, NV, 2, 2, 1>(p, fl, epoch, stream, coop);              \
        default: return fused::launch<NF, NV, 2, 0>(p, fl, epoch, stream, coop);                  \
    }
    if (p.lay.nfixed == 0 && p.lay.nvar == 1) SYM_FUSED(0, 1);
    if (p.lay.nfixed == 0 && p.lay.nvar == 2) SYM_FUSED(0, 2);
    if (p.lay.nfixed == 2 && p.lay.nvar == 2) SYM_FUSED(2, 2);
#undef SYM_FUSED
    return hipErrorInvalidValue;
}

}  // namespace symhip
