// flat.hip -- batched Symphony codec for any flat schema on gfx950 (flat part).
//
// The generated MarshalSymphony / UnmarshalSymphony of a message whose fields are fixed-width
// (bool 1 byte; int32 / uint32 / float / enum 4; int64 / uint64 / double 8) or string / bytes,
// each public or private (cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:196-368, 439-620,
// 622-800), driven by a field descriptor at run time instead of per-schema kernels:
//  * encode: per-record size (thread = record), tile totals, tile scan, output offsets; then a
//    thread per record writes header, tables and payloads, string payloads as byte-unaligned
//    16-byte chunks;
//  * decode: a thread per record checks the header, copies the fixed fields into their columns
//    and resolves each string field (source, length) with the generator's checks and the per-tile
//    totals; then per string field the tile scan and the shared segment gather (raw_fields.hip)
//    write the packed column and its offsets.
// The all-private two-column schemas also have the specialised pipelines of encode.hip /
// decode_pipe.hip; this is the general path.
#include <algorithm>
#include <cstring>

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

namespace flat {

using raw::Pair;

constexpr int kMax = SYM_MAX_FLAT_FIELDS;

struct Schema {
    int nf;
    uint8_t seg[kMax], width[kMax];
    u32 table[2];  // public / private table bytes
};

inline Schema make_schema(const sym_field* f, int nf) {
    Schema s{};
    s.nf = nf;
    for (int k = 0; k < nf; ++k) {
        s.seg[k] = f[k].segment;
        s.width[k] = f[k].width;
        s.table[f[k].segment] += f[k].width ? f[k].width : 4;
    }
    return s;
}

// ---- encode (main.go:196-330, 334-368, 439-620), output-stationary like encode.hip.
// A record is  G_0 P_0 G_1 P_1 ... P_{nv-1} G_nv : payload bytes P_v (public strings in field
// order, then private strings) and generated pieces G_q (header, tables, length prefixes, the
// private marker) whose lengths depend on the schema only, so their concatenation -- the "image",
// G = 14 + tables + 4 nv bytes -- is built per record in LDS, and out_off is affine:
//   out_off[r] = r G + sum_v (offs_v[r] - offs_v[0]).
struct EncArgs {
    Schema sc;
    u64 n;
    const uint8_t* col[kMax];  // by field: fixed n values of width bytes; string packed bytes
    const u64* offs[kMax];     // by field: string n+1 offsets
    u32 sid, mid;
    uint8_t* out;
    u64* out_off;
    unsigned* err;
    // payload order: public strings then private strings, each in field order
    int nv, np;
    uint8_t vfield[kMax];
    u32 G;
    u32 g0, gnp, glast;  // lengths of G_0, G_np (0 < np < nv), G_nv; every other G_q is 4
};

// the generated piece lengths as register arithmetic: a lane's piece index diverges, so a table
// in kernel-argument memory would cost a vector load per piece
__device__ __forceinline__ int gen_len(const EncArgs& a, int q) {
    return q == 0 ? (int)a.g0 : q == a.nv ? (int)a.glast : q == a.np ? (int)a.gnp : 4;
}

constexpr int kEncRecs = 64;  // records per wave tile
constexpr int kEncWaves = 4;

// per-wave LDS: o[65] int | len[nv][64] u32 | src[nv][64] u64 | column lo / hi [nv] u64 | pad 16 |
// image 64 G | pad 16
struct EncLds {
    size_t len, src, clo, chi, img, total;
};
__host__ __device__ inline EncLds enc_lds(int nv, u32 G) {
    EncLds l;
    l.len = (kEncRecs + 1) * 4;
    l.src = (l.len + (size_t)nv * kEncRecs * 4 + 7) & ~(size_t)7;
    l.clo = l.src + (size_t)nv * kEncRecs * 8;
    l.chi = l.clo + (size_t)nv * 8;
    l.img = l.chi + (size_t)nv * 8 + 16;
    l.total = (l.img + (size_t)kEncRecs * G + 16 + 15) & ~(size_t)15;
    return l;
}

__global__ __launch_bounds__(256) void enc_tile_kernel(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    __shared__ MaskTable masks;
    mask_table_init(masks, threadIdx.x);
    __syncthreads();  // the only workgroup barrier

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const Schema& sc = a.sc;
    const int nv = a.nv;
    const u32 G = a.G;
    const EncLds ly = enc_lds(nv, G);
    char* const W = dyn + (size_t)wave * ly.total;
    int* const So = (int*)W;
    u32* const Slen = (u32*)(W + ly.len);
    u64* const Ssrc = (u64*)(W + ly.src);
    u64* const Sclo = (u64*)(W + ly.clo);  // string column q's 16-byte-rounded extent
    u64* const Schi = (u64*)(W + ly.chi);
    uint8_t* const img = (uint8_t*)(W + ly.img);

    const u64 r0 = ((u64)blockIdx.x * (blockDim.x >> 6) + wave) * kEncRecs;
    if (r0 >= a.n) return;  // wave-uniform
    const int cnt = (int)min((u64)kEncRecs, a.n - r0);

    // ---------------- phase 1 (lane = record): offsets and the generated image ----------------
    i64 o = 0, size = 0;
    if (lane < cnt) {
        const u64 r = r0 + lane;
        o = (i64)(r * G);
        size = G;
        u64 pub = 0;
        for (int v = 0; v < nv; ++v) {
            const int k = a.vfield[v];
            const u64 lo = a.offs[k][r], L = a.offs[k][r + 1] - lo;
            o += (i64)(lo - a.offs[k][0]);
            size += (i64)L;
            if (v < a.np) pub += 4 + L;
            Slen[v * kEncRecs + lane] = (u32)L;
            Ssrc[v * kEncRecs + lane] = (u64)(uintptr_t)(a.col[k] + lo);
        }
        a.out_off[r] = (u64)o;
        if (r == a.n - 1) a.out_off[a.n] = (u64)(o + size);
        // image: header | public table | public length prefixes | marker | private table |
        // private length prefixes
        uint8_t* im = img + (size_t)lane * G;
        auto put = [&](u64 v, int w) {
            for (int b = 0; b < w; ++b) *im++ = (uint8_t)(v >> (8 * b));
        };
        const u64 off2p = 13 + sc.table[0] + pub;
        put(1, 1);
        put(off2p, 4);
        put(a.sid, 4);  // the client's ID patch, pkg/rpc/client.go:267-271
        put(a.mid, 4);
        for (int seg = 0; seg < 2; ++seg) {
            u64 pos = seg ? 1 + sc.table[1] : 13 + sc.table[0];  // next length prefix (private: relative)
            if (seg) put(1, 1);
            int v = seg ? a.np : 0;
            for (int k = 0; k < sc.nf; ++k) {
                if (sc.seg[k] != seg) continue;
                const int w = sc.width[k];
                if (w == 1) put(a.col[k][r], 1);
                else if (w == 4) put(((const u32*)a.col[k])[r], 4);
                else if (w == 8) put(((const u64*)a.col[k])[r], 8);
                else {
                    put(pos, 4);
                    pos += 4 + Slen[v * kEncRecs + lane];
                    ++v;
                }
            }
            for (int u = seg ? a.np : 0; u < (seg ? nv : a.np); ++u) put(Slen[u * kEncRecs + lane], 4);
        }
    }
    const i64 T0 = uniform_i64((i64)__shfl((long long)o, 0, 64));
    const i64 T1 = uniform_i64((i64)__shfl((long long)(o + size), cnt - 1, 64));
    if (T1 - T0 >= (i64)1 << 31) {  // positions are 32-bit inside a tile
        if (lane == 0) atomicOr(a.err, kErrTooLarge);
        return;
    }
    if (lane < cnt) So[lane] = (int)(o - T0);
    if (lane == cnt - 1) So[cnt] = (int)(T1 - T0);
    if (lane < nv) {
        const int k = a.vfield[lane];
        Sclo[lane] = (u64)(uintptr_t)(a.col[k] + a.offs[k][0]) & ~(u64)15;
        Schi[lane] = ((u64)(uintptr_t)(a.col[k] + a.offs[k][a.n]) + 15) & ~(u64)15;
    }
    wave_sync();

    // ---------------- phase 2 (lane = aligned 16-byte output chunk) ----------------
    const int span = (int)(T1 - T0);
    const i64 mis = (i64)((uintptr_t)a.out & 15);
    const int first = (int)(((T0 + mis) & ~(i64)15) - mis - T0);  // in (-16, 0]
    uint8_t* const out_t = a.out + T0;
    const uintptr_t dummy = (uintptr_t)a.out & ~(uintptr_t)15;  // readable; its bytes get masked off

    // Every byte of chunk P: generated bytes straight from LDS, payload windows as byte-unaligned
    // 16-byte loads.  `fast` collects at most two payload windows per chunk (loads issued after
    // the walk, all chunks of a step together); a chunk with more, or with a window at a column's
    // end, is redone by `slow` with in-place loads.
    auto locate = [&](int P) {  // largest j with So[j] <= P (0 for the chunk straddling the start)
        int j = 0;
        for (int step = 32; step; step >>= 1)
            if (j + step < cnt && So[j + step] <= P) j += step;
        return j;
    };
    auto slow = [&](int P) -> u32x4 {
        u32x4 acc = {0, 0, 0, 0};
        for (int j = locate(P); j < cnt; ++j) {
            const int b = P - So[j];  // chunk start relative to record j
            if (b <= -16) break;
            int rs = 0, gi = 0;
            const uint8_t* im = img + (size_t)j * G;
            for (int q = 0; q <= nv; ++q) {
                const int gl = gen_len(a, q);
                if (gl && rs + gl > b) acc |= lds16u(im, gi + b - rs) & range_mask(masks, rs - b, rs + gl - b);
                rs += gl;
                gi += gl;
                if (rs >= b + 16 || q == nv) break;
                const int L = (int)Slen[q * kEncRecs + j];
                if (L && rs + L > b) {
                    const uintptr_t X = (uintptr_t)(Ssrc[q * kEncRecs + j] + (u64)(i64)(b - rs));
                    u32 t[4] = {0, 0, 0, 0};
                    or_window_global(X, max(rs - b, 0), min(rs + L - b, 16), t);
                    acc |= u32x4{t[0], t[1], t[2], t[3]};
                }
                rs += L;
                if (rs >= b + 16) break;
            }
        }
        return acc;
    };
    constexpr int kU = 4;  // chunks per lane per step
    for (int B0 = first; B0 < span; B0 += 16 * 64 * kU) {  // wave-uniform loop
        u32x4 acc[kU];
        uintptr_t X0[kU], X1[kU];
        int lo0[kU], hi0[kU], lo1[kU], hi1[kU], nw[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int P = B0 + 16 * 64 * u + 16 * lane;
            acc[u] = u32x4{0, 0, 0, 0};
            X0[u] = X1[u] = dummy;
            lo0[u] = hi0[u] = lo1[u] = hi1[u] = 0;
            nw[u] = 0;
            if (P >= span) continue;
            for (int j = locate(P); j < cnt; ++j) {
                const int b = P - So[j];
                if (b <= -16) break;
                int rs = 0, gi = 0;
                const uint8_t* im = img + (size_t)j * G;
                for (int q = 0; q <= nv; ++q) {
                    const int gl = gen_len(a, q);
                    if (gl && rs + gl > b)
                        acc[u] |= lds16u(im, gi + b - rs) & range_mask(masks, rs - b, rs + gl - b);
                    rs += gl;
                    gi += gl;
                    if (rs >= b + 16 || q == nv) break;
                    const int L = (int)Slen[q * kEncRecs + j];
                    if (L && rs + L > b) {
                        const u64 X = Ssrc[q * kEncRecs + j] + (u64)(i64)(b - rs);
                        const bool inside = X >= Sclo[q] && X + 16 <= Schi[q];
                        if (!inside || nw[u] >= 2) {
                            nw[u] = 3;  // slow chunk
                        } else if (nw[u] == 0) {
                            X0[u] = (uintptr_t)X, lo0[u] = rs - b, hi0[u] = rs + L - b, nw[u] = 1;
                        } else {
                            X1[u] = (uintptr_t)X, lo1[u] = rs - b, hi1[u] = rs + L - b, nw[u] = 2;
                        }
                    }
                    rs += L;
                    if (rs >= b + 16) break;
                }
            }
            if (nw[u] == 3) X0[u] = X1[u] = dummy;
        }
        u32x4 w0[kU], w1[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {  // unconditional loads: all issue before the first wait
            w0[u] = ld16u(X0[u]);
            w1[u] = ld16u(X1[u]);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int P = B0 + 16 * 64 * u + 16 * lane;
            if (P >= span) continue;
            u32x4 r = acc[u];
            if (nw[u] == 3) {
                r |= slow(P);
            } else {
                r |= (w0[u] & range_mask(masks, lo0[u], hi0[u])) | (w1[u] & range_mask(masks, lo1[u], hi1[u]));
            }
            const u32 rr[4] = {r.x, r.y, r.z, r.w};
            store_chunk(out_t, P, 0, span, rr);
        }
    }
}

// ---- decode parse (main.go:622-800): status, fixed fields, string (source, length) + tile totals
struct DecArgs {
    Schema sc;
    u64 n;
    const uint8_t* in;
    const u64* rec_off;
    uint8_t* col[kMax];  // fixed: n values of width bytes
    uint8_t* status;
    u64* seg_src;        // [nvar][n]
    u64* seg_len;        // [nvar][n]
    Pair* agg;           // [nvar][tiles]
    u64 tiles;
};

__global__ __launch_bounds__(256) void dec_parse_kernel(DecArgs a) {
    __shared__ u64 red[kMax][4];
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    const Schema& sc = a.sc;
    u64 vlen[kMax];
    for (int k = 0; k < kMax; ++k) vlen[k] = 0;
    if (i < a.n) {
        const u64 s = a.rec_off[i], L = a.rec_off[i + 1] - s;
        const uintptr_t d = (uintptr_t)(a.in + s);
        for (int k = 0; k < sc.nf; ++k)  // fresh struct: zero values
            if (sc.width[k])
                for (int t = 0; t < sc.width[k]; ++t) a.col[k][(u64)sc.width[k] * i + t] = 0;
        int vi = 0;
        for (int k = 0; k < sc.nf; ++k)
            if (!sc.width[k]) {
                a.seg_src[(u64)vi * a.n + i] = s;
                ++vi;
            }
        uint8_t st = SYM_STATUS_OK;
        if (L < (sc.nf ? 13u : 14u)) st = SYM_STATUS_TOO_SHORT;
        else if (ld_u8(d) != 1) st = SYM_STATUS_BAD_VERSION;
        else {
            const u64 o = ld_u32(d + 1);
            if (o >= L || ld_u8(d + o) != 1) st = SYM_STATUS_NO_PRIVATE;
            for (int seg = 0; seg < 2 && st == SYM_STATUS_OK; ++seg) {
                const u64 ts = seg ? o + 1 : 13;
                u64 t = 0;
                int v = 0;
                for (int k = 0; k < sc.nf; ++k) {
                    if (!sc.width[k] && sc.seg[k] != seg) {
                        ++v;
                        continue;
                    }
                    if (sc.seg[k] != seg) continue;
                    const int w = sc.width[k];
                    if (w) {
                        if (L < ts + t + w) {
                            st = SYM_STATUS_FIELD_TOO_SHORT;  // "invalid data: too short for field"
                            break;
                        }
                        for (int b = 0; b < w; ++b) a.col[k][(u64)w * i + b] = (uint8_t)ld_u8(d + ts + t + b);
                        t += w;
                    } else {
                        if (L >= ts + t + 4) {
                            u64 po = ld_u32(d + ts + t);
                            if (seg && po > 0) po += o;  // private offsets are relative
                            if (po > 0 && L >= po + 4) {
                                const u64 dl = ld_u32(d + po);
                                if (L >= po + 4 + dl) {
                                    a.seg_src[(u64)v * a.n + i] = s + po + 4;
                                    vlen[v] = dl;
                                }
                            }
                        }
                        t += 4;
                        ++v;
                    }
                }
            }
        }
        a.status[i] = st;
        // a decode error leaves every string field of the record empty only past the failing
        // field; fields resolved before it keep their values (the struct is filled in order)
        vi = 0;
        for (int k = 0; k < sc.nf; ++k)
            if (!sc.width[k]) {
                a.seg_len[(u64)vi * a.n + i] = vlen[vi];
                ++vi;
            }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int nv = 0;
    for (int k = 0; k < sc.nf; ++k) nv += sc.width[k] == 0;
    for (int v = 0; v < nv; ++v) {
        const u64 w = wave_sum_u64(vlen[v]);
        if (lane == 0) red[v][wave] = w;
    }
    __syncthreads();
    if (threadIdx.x < nv)
        a.agg[(u64)threadIdx.x * a.tiles + blockIdx.x] =
            Pair{red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3], 0};
}

inline u64 tiles(u64 m) { return (m + 255) / 256; }
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace flat

// decode workspace: [seg_src (nv x n) | seg_len (nv x n) | tile totals (nv x tiles) | tile
// prefixes (nv x (tiles + 1))]; encode needs none
static size_t dec_ws(int nv, u64 n) {
    const u64 nt = flat::tiles(n);
    return 2 * flat::al256((size_t)nv * n * 8) + flat::al256((size_t)nv * nt * sizeof(raw::Pair)) +
           flat::al256((size_t)nv * (nt + 1) * sizeof(raw::Pair));
}

size_t flat_ws_bytes(const sym_field* f, int nf, u64 n) {
    int nv = 0;
    for (int k = 0; k < nf; ++k) nv += f[k].width == 0;
    return dec_ws(nv, n);
}

hipError_t launch_flat_encode(const sym_field* f, int nf, u64 n, const void* const* cols, const u64* const* offs,
                              u32 sid, u32 mid, uint8_t* out, u64* out_off, unsigned* err, hipStream_t stream) {
    flat::EncArgs a{};
    a.sc = flat::make_schema(f, nf);
    a.n = n;
    for (int k = 0; k < nf; ++k) {
        a.col[k] = (const uint8_t*)cols[k];
        a.offs[k] = f[k].width ? nullptr : offs[k];
    }
    for (int seg = 0; seg < 2; ++seg)
        for (int k = 0; k < nf; ++k)
            if (!f[k].width && f[k].segment == seg) a.vfield[a.nv++] = (uint8_t)k;
    for (int k = 0; k < nf; ++k) a.np += !f[k].width && f[k].segment == 0;
    a.sid = sid;
    a.mid = mid;
    a.out = out;
    a.out_off = out_off;
    a.err = err;
    // generated piece lengths: G_0 = header + public table + (first length prefix, or, without
    // public strings, marker + private table + first length prefix); G_np = marker + private
    // table + its length prefix; other inner pieces one length prefix; G_nv = marker + private
    // table when every string is public
    const u32 t0 = a.sc.table[0], t1 = a.sc.table[1];
    a.G = 14 + t0 + t1 + 4 * (u32)a.nv;
    if (a.nv == 0) {
        a.g0 = a.G;  // q == 0 == nv: gen_len returns g0
    } else {
        a.g0 = 13 + t0 + (a.np > 0 ? 4 : 1 + t1 + 4);
        a.gnp = 1 + t1 + 4;
        a.glast = a.np == a.nv ? 1 + t1 : 0;
    }
    // up to 4 waves per workgroup within 64 KiB of dynamic LDS (a wave needs 5-22 KiB)
    const size_t wl = flat::enc_lds(a.nv, a.G).total;
    const int waves = (int)std::min<size_t>(flat::kEncWaves, 65536 / wl);
    const u64 per = (u64)flat::kEncRecs * waves;
    hipLaunchKernelGGL(flat::enc_tile_kernel, dim3((unsigned)((n + per - 1) / per)), dim3(64 * waves), waves * wl,
                       stream, a);
    return hipGetLastError();
}

hipError_t launch_flat_decode(const sym_field* f, int nf, u64 n, const uint8_t* in, const u64* rec_off,
                              void* const* cols, const u64* caps, u64* const* offs, uint8_t* status, void* ws,
                              unsigned* err, hipStream_t stream) {
    using raw::Pair;
    flat::DecArgs a{};
    a.sc = flat::make_schema(f, nf);
    a.n = n;
    a.in = in;
    a.rec_off = rec_off;
    for (int k = 0; k < nf; ++k) a.col[k] = f[k].width ? (uint8_t*)cols[k] : nullptr;
    a.status = status;
    const u64 nt = flat::tiles(n);
    a.tiles = nt;
    int nv = 0;
    for (int k = 0; k < nf; ++k) nv += f[k].width == 0;
    char* w = (char*)ws;
    a.seg_src = (u64*)w;
    a.seg_len = (u64*)(w + flat::al256((size_t)nv * n * 8));
    a.agg = (Pair*)(w + 2 * flat::al256((size_t)nv * n * 8));
    Pair* pre = (Pair*)((char*)a.agg + flat::al256((size_t)nv * nt * sizeof(Pair)));
    const dim3 g((unsigned)nt), b(256);
    hipLaunchKernelGGL(flat::dec_parse_kernel, g, b, 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // every string field: tile scan of its lengths, then the gather into its column
    int v = 0;
    for (int k = 0; k < nf; ++k) {
        if (f[k].width) continue;
        const Pair* agg = a.agg + (size_t)v * nt;  // row v: written at v * tiles + tile
        Pair* pv = pre + (size_t)v * (nt + 1);
        if ((e = launch_tile_scan(agg, pv, nt, stream)) != hipSuccess) return e;
        raw::GatherArgs ga{};
        ga.in = in;
        ga.n = n;
        ga.lo_ptr = rec_off;
        ga.hi_ptr = rec_off + n;
        ga.pre = pv;
        ga.seg_src = a.seg_src + (size_t)v * n;
        ga.seg_len = a.seg_len + (size_t)v * n;
        ga.out = (uint8_t*)cols[k];
        ga.cap = caps[k];
        ga.out_off = offs[k];
        ga.err = err;
        if ((e = launch_segment_gather(ga, stream)) != hipSuccess) return e;
        ++v;
    }
    return hipSuccess;
}

}  // namespace symhip
