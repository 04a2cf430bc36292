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

struct EncArgs {
    Schema sc;
    u64 n;
    const uint8_t* col[kMax];  // fixed: n values of width bytes; string: packed bytes
    const u64* offs[kMax];     // string: n+1 offsets
    u32 sid, mid;
    uint8_t* out;
    u64* out_off;
    u64* size;
    Pair* agg;
};

__device__ inline void put_u32(uint8_t* p, u32 v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

__device__ inline void block_total(u64 v, Pair* agg) {
    __shared__ u64 red[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 w = wave_sum_u64(v);
    if (lane == 0) red[wave] = w;
    __syncthreads();
    if (threadIdx.x == 0) agg[blockIdx.x] = Pair{red[0] + red[1] + red[2] + red[3], 0};
}

// ---- encode size (main.go:214-285): 13 + public table + public payloads + 1 + private table + payloads
__global__ __launch_bounds__(256) void enc_size_kernel(EncArgs a) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    u64 sz = 0;
    if (i < a.n) {
        if (a.sc.nf == 0) {
            sz = 14;  // empty message, main.go:201-212
        } else {
            sz = 13 + (u64)a.sc.table[0] + 1 + (u64)a.sc.table[1];
            for (int k = 0; k < a.sc.nf; ++k)
                if (!a.sc.width[k]) sz += 4 + (a.offs[k][i + 1] - a.offs[k][i]);
        }
        a.size[i] = sz;
    }
    block_total(sz, a.agg);
}

__global__ __launch_bounds__(256) void apply_kernel(const u64* size, u64 n, const Pair* tpre, u64* out_off) {
    __shared__ u64 wb[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    const u64 v = i < n ? size[i] : 0;
    const u64 inc = wave_incl_scan_u64(v, lane);
    if (lane == 63) wb[wave] = inc;
    __syncthreads();
    u64 p = tpre[blockIdx.x].bytes;
    for (int q = 0; q < wave; ++q) p += wb[q];
    if (i < n) out_off[i] = p + inc - v;
    if (i == n - 1) out_off[n] = p + inc;
}

// copy L bytes src -> dst (both arbitrary byte addresses): 16-byte chunks, byte tail
__device__ inline void copy_bytes(uint8_t* dst, uintptr_t src, u64 L) {
    u64 o = 0;
    for (; o + 16 <= L; o += 16) *(g_u4*)(dst + o) = ld16u(src + o);
    for (; o < L; ++o) *(g_u8*)(dst + o) = (uint8_t)ld_u8(src + o);
}

// ---- encode write (main.go:286-330 and the segment emitters :334-368, 439-620)
__global__ __launch_bounds__(256) void enc_write_kernel(EncArgs a) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    uint8_t* const b = a.out + a.out_off[i];
    const Schema& sc = a.sc;
    if (sc.nf == 0) {
        for (int t = 0; t < 14; ++t) b[t] = 0;
        b[0] = 1;
        put_u32(b + 1, 13);
        put_u32(b + 5, a.sid);
        put_u32(b + 9, a.mid);
        b[13] = 1;
        return;
    }
    u64 off2p = 13 + sc.table[0];
    for (int k = 0; k < sc.nf; ++k)
        if (!sc.seg[k] && !sc.width[k]) off2p += 4 + (a.offs[k][i + 1] - a.offs[k][i]);
    b[0] = 1;
    put_u32(b + 1, (u32)off2p);
    put_u32(b + 5, a.sid);  // the client's ID patch, pkg/rpc/client.go:267-271
    put_u32(b + 9, a.mid);
    b[off2p] = 1;
    u64 tab[2] = {13, off2p + 1};
    u64 pos[2] = {13 + (u64)sc.table[0], off2p + 1 + (u64)sc.table[1]};
    for (int k = 0; k < sc.nf; ++k) {
        const int s = sc.seg[k];
        const int w = sc.width[k];
        if (w) {
            const uint8_t* v = a.col[k] + (u64)w * i;
            for (int t = 0; t < w; ++t) b[tab[s] + t] = v[t];
            tab[s] += w;
        } else {
            const u64 s0 = a.offs[k][i], L = a.offs[k][i + 1] - s0;
            put_u32(b + tab[s], (u32)(s ? pos[s] - off2p : pos[s]));  // private offsets are relative
            put_u32(b + pos[s], (u32)L);
            copy_bytes(b + pos[s] + 4, (uintptr_t)(a.col[k] + s0), L);
            pos[s] += 4 + L;
            tab[s] += 4;
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

// workspace: encode [size (n) | tile totals | tile prefixes]; decode [seg_src (nv x n) | seg_len
// (nv x n) | tile totals (nv x tiles) | tile prefixes (nv x (tiles + 1))]
static size_t enc_ws(u64 n) { return flat::al256(n * 8) + 2 * flat::al256((flat::tiles(n) + 1) * sizeof(raw::Pair)); }
static size_t dec_ws(int nv, u64 n) {
    const u64 nt = flat::tiles(n);
    return 2 * flat::al256((size_t)nv * n * 8) + flat::al256((size_t)nv * nt * sizeof(raw::Pair)) +
           flat::al256((size_t)nv * (nt + 1) * sizeof(raw::Pair));
}

size_t flat_ws_bytes(const sym_field* f, int nf, u64 n) {
    int nv = 0;
    for (int k = 0; k < nf; ++k) nv += f[k].width == 0;
    const size_t e = enc_ws(n), d = dec_ws(nv, n);
    return e > d ? e : d;
}

hipError_t launch_flat_encode(const sym_field* f, int nf, u64 n, const void* const* cols, const u64* const* offs,
                              u32 sid, u32 mid, uint8_t* out, u64* out_off, void* ws, hipStream_t stream) {
    using raw::Pair;
    flat::EncArgs a{};
    a.sc = flat::make_schema(f, nf);
    a.n = n;
    for (int k = 0; k < nf; ++k) {
        a.col[k] = (const uint8_t*)cols[k];
        a.offs[k] = f[k].width ? nullptr : offs[k];
    }
    a.sid = sid;
    a.mid = mid;
    a.out = out;
    a.out_off = out_off;
    const u64 nt = flat::tiles(n);
    a.size = (u64*)ws;
    a.agg = (Pair*)((char*)ws + flat::al256(n * 8));
    Pair* tpre = (Pair*)((char*)a.agg + flat::al256((nt + 1) * sizeof(Pair)));
    const dim3 g((unsigned)nt), b(256);
    hipLaunchKernelGGL(flat::enc_size_kernel, g, b, 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = launch_tile_scan(a.agg, tpre, nt, stream)) != hipSuccess) return e;
    hipLaunchKernelGGL(flat::apply_kernel, g, b, 0, stream, (const u64*)a.size, n, (const Pair*)tpre, out_off);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(flat::enc_write_kernel, g, b, 0, stream, a);
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
