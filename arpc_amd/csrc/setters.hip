// setters.hip -- batched Raw setters: XxxRaw.SetF(v_i) on n buffers, gfx950.
//
// Restates the generated setters (cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:1038-1093
// assertions, :1296-1336 fixed fields, :1567-1620 strings / bytes, :1685-1740 repeated fixed
// fields, :371-437 the remarshal path; e.g. GetRequestRaw.SetScore / SetUsername / SetKey,
// benchmark/kv-store-symphony-element/symphony/kv.syn.go:340-412) for any flat schema:
//   public field : a complete buffer (data[offsetToPrivate] == 1) panics;
//   private field: a buffer under 5 bytes or without its private marker panics;
//   a table entry past the end is an error ("buffer too short [for table entry]");
//   fixed fields are written in place; a payload field (string / bytes / repeated fixed) in place
//   when its old payload offset is set and the new length / count is not larger (u32 length or
//   count, then the new bytes; the old tail stays as slack), else the message is remarshalled:
//   public -- unmarshal data + [0x01] + a zeroed private table, set, marshal, restore bytes [5:13],
//   keep the public part; private -- unmarshal, set, marshal (bytes [5:13] come back 0).
// Every buffer is written to a new stream (its size may change), a panicking or failing one
// unchanged, with its status.  Two launches around the shared tile scan:
//   plan  (thread = buffer): status, what happens (copy / patch / remarshal) and the output size;
//         the buffer's offset inside its 256-buffer tile, tile totals;
//   write (wave = buffer):   the output bytes, lanes striding over each piece; final offsets.
// This is the correctness-first form of a control-path operation (a proxy rewriting fields): byte
// loads and stores, every remarshal read through the generator's rules.
#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"
#include "flat_schema.hpp"

namespace symhip {
namespace setter {

using flat::kMax;
using flat::Schema;
using raw::Pair;

constexpr int kTile = 256;
constexpr u64 kCopy = 0, kPatch = 1, kRemarshal = 2;

struct SetArgs {
    Schema sc;
    int k;
    u64 n;
    const uint8_t* in;
    const u64* rec_off;
    const uint8_t* val;  // fixed: n values of width bytes; payload: bytes with val_off
    const u64* val_off;
    uint8_t* out;
    u64 cap;
    u64* out_off;
    uint8_t* status;
    Pair* agg;  // [tiles]
    Pair* pre;  // [tiles + 1]
    u64 tiles;
    unsigned* err;
};

SYMHIP_KERNARG_ARRAY(SetArgs, sc.seg);
SYMHIP_KERNARG_ARRAY(SetArgs, sc.shift);

// The buffer as Go sees it.  fake: the public remarshal's data + [0x01] + zeroed private table,
// whose [1:5] holds len(data) (written before the marker, main.go:397-400).
struct View {
    const uint8_t* m;
    u64 L, Lv;
    bool fake;
    __device__ u32 byte(u64 q) const {
        if (!fake) return m[q];
        if (q == L) return 1u;
        if (q >= 1 && q < 5) return (u32)(L >> (8 * (q - 1))) & 0xffu;
        return q < L ? m[q] : 0u;
    }
    __device__ u64 u32at(u64 q) const {
        return (u64)byte(q) | ((u64)byte(q + 1) << 8) | ((u64)byte(q + 2) << 16) | ((u64)byte(q + 3) << 24);
    }
};

struct Plan {
    u32 st, mode;
    u64 size;
    u64 toff;        // the field's table entry / fixed value (absolute)
    u64 po, newn;    // patch: payload offset (absolute) and new length / count
    u64 vstart, vn;  // the new value in the value column
    bool pub;
    u64 off2p_new;   // remarshal: the new offsetToPrivate
};

__device__ __forceinline__ int scalar_w(const Schema& sc, int j) { return sc.width[j]; }
__device__ __forceinline__ u64 entry_w(const Schema& sc, int j) { return sc.width[j] ? sc.width[j] : 4u; }

// Unmarshal v into a fresh struct (main.go:622-800): fixed values in fx, payloads as (source, bytes).
__device__ u32 unmarshal(const Schema& sc, const View& v, u64 (&fx)[kMax], u64 (&src)[kMax], u64 (&len)[kMax]) {
    for (int j = 0; j < kMax; ++j) fx[j] = src[j] = len[j] = 0;
    const u64 L = v.Lv;
    if (L < (sc.nf ? 13u : 14u)) return SYM_STATUS_TOO_SHORT;
    if (v.byte(0) != 1) return SYM_STATUS_BAD_VERSION;
    const u64 o = v.u32at(1);
    if (o >= L || v.byte(o) != 1) return SYM_STATUS_NO_PRIVATE;
    for (int s = 0; s < 2; ++s) {
        const u64 ts = s ? o + 1 : 13;
        u64 t = 0;
        for (int j = 0; j < sc.nf; ++j) {
            if (sc.seg[j] != s) continue;
            const int w = scalar_w(sc, j);
            if (w) {
                if (L < ts + t + w) return SYM_STATUS_FIELD_TOO_SHORT;
                u64 x = 0;
                for (int b = 0; b < w; ++b) x |= (u64)v.byte(ts + t + b) << (8 * b);
                fx[j] = x;
                t += w;
            } else {
                if (L >= ts + t + 4) {
                    u64 po = v.u32at(ts + t);
                    if (s && po > 0) po += o;
                    if (po > 0 && L >= po + 4) {
                        const u64 dl = v.u32at(po) << sc.shift[j];
                        if (L >= po + 4 + dl) {
                            src[j] = po + 4;
                            len[j] = dl;
                        }
                    }
                }
                t += 4;
            }
        }
    }
    return SYM_STATUS_OK;
}

__device__ u64 table_offset(const Schema& sc, int k) {
    u64 t = sc.seg[k] ? 1 : 13;
    for (int j = 0; j < k; ++j)
        if (sc.seg[j] == sc.seg[k]) t += entry_w(sc, j);
    return t;
}

// What SetF does to buffer i (and, for a remarshal, the unmarshalled fields).
__device__ Plan plan_one(const SetArgs& a, u64 i, View& v, u64 (&fx)[kMax], u64 (&src)[kMax], u64 (&len)[kMax]) {
    const Schema& sc = a.sc;
    const int k = a.k;
    Plan p{};
    const u64 s0 = a.rec_off[i];
    v.m = a.in + s0;
    v.L = v.Lv = a.rec_off[i + 1] - s0;
    v.fake = false;
    const u64 L = v.L;
    p.pub = sc.seg[k] == 0;
    const int w = scalar_w(sc, k);
    p.vstart = w ? (u64)w * i : a.val_off[i];
    p.vn = w ? (u64)w : a.val_off[i + 1] - a.val_off[i];
    p.size = L;
    p.mode = kCopy;
    u64 o2p = 0;
    p.toff = table_offset(sc, k);
    if (p.pub) {
        if (L >= 5) {
            o2p = v.u32at(1);
            if (o2p < L && v.byte(o2p) == 1) p.st = SYM_SET_COMPLETE_BUFFER;
        }
    } else if (L < 5) {
        p.st = SYM_SET_INVALID_BUFFER;
    } else {
        o2p = v.u32at(1);
        if (o2p >= L || v.byte(o2p) != 1) p.st = SYM_SET_PUBLIC_ONLY;
        p.toff += o2p;
    }
    if (p.st) return p;
    if (L < p.toff + (w ? (u64)w : 4u)) {
        p.st = SYM_SET_TOO_SHORT;
        return p;
    }
    if (w) {  // fixed: in place
        p.mode = kPatch;
        return p;
    }
    if (p.vn & ((1ull << sc.shift[k]) - 1)) {  // a repeated field's value is not whole elements
        p.st = SYM_SET_BAD_LENGTH;
        return p;
    }
    u64 po = v.u32at(p.toff);
    if (!p.pub && po > 0) po += o2p;
    const u64 oldn = po > 0 && L >= po + 4 ? v.u32at(po) : 0;
    p.newn = p.vn >> sc.shift[k];
    if (po > 0 && p.newn <= oldn) {  // in place; an out-of-range length / element write panics in Go
        if (L < po + 4 || (sc.shift[k] && L < po + 4 + p.vn)) {
            p.st = SYM_SET_BOUNDS;
            return p;
        }
        p.po = po;
        p.mode = kPatch;
        return p;
    }
    // remarshal
    if (p.pub) {
        if (L + 1 + sc.table[1] < 5) {  // fakeComplete[1:5] out of range: Go panics
            p.st = SYM_SET_BOUNDS;
            return p;
        }
        v.fake = true;
        v.Lv = L + 1 + sc.table[1];
    }
    if (unmarshal(sc, v, fx, src, len) != SYM_STATUS_OK) {
        p.st = SYM_SET_UNMARSHAL;
        v.fake = false;
        v.Lv = L;
        return p;
    }
    len[k] = p.vn;
    u64 pubpay = 0, privpay = 0;
    for (int j = 0; j < sc.nf; ++j)
        if (!scalar_w(sc, j)) (sc.seg[j] ? privpay : pubpay) += 4 + len[j];
    p.off2p_new = 13 + sc.table[0] + pubpay;
    p.size = p.pub ? p.off2p_new : p.off2p_new + 1 + sc.table[1] + privpay;
    p.mode = kRemarshal;
    return p;
}

__global__ __launch_bounds__(kTile) void plan_kernel(SetArgs a) {
    __shared__ u64 wsum[4];
    const u64 i = (u64)blockIdx.x * kTile + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 size = 0;
    if (i < a.n) {
        View v;
        u64 fx[kMax], src[kMax], len[kMax];
        const Plan p = plan_one(a, i, v, fx, src, len);
        size = p.st ? v.L : p.size;
        a.status[i] = (uint8_t)p.st;
    }
    const u64 inc = wave_incl_scan_u64(size, lane);
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    u64 before = 0, tot = 0;
    for (int q = 0; q < 4; ++q) {
        if (q < wave) before += wsum[q];
        tot += wsum[q];
    }
    if (i < a.n) a.out_off[i] = before + inc - size;  // inside the tile; the write kernel adds the tile prefix
    if (threadIdx.x == 0) a.agg[blockIdx.x] = Pair{tot, 0};
}

// Lanes write bytes [0, len) of one piece at dst: byte b = f(b).
template <typename F>
__device__ __forceinline__ void put_piece(uint8_t* dst, u64 len, F f) {
    const int lane = threadIdx.x & 63;
    for (u64 b = lane; b < len; b += 64) dst[b] = (uint8_t)f(b);
}

__global__ __launch_bounds__(256) void write_kernel(SetArgs a) {
    const int lane = threadIdx.x & 63;
    const u64 nw = (u64)gridDim.x * 4;
    const Schema& sc = a.sc;
    for (u64 i = (u64)blockIdx.x * 4 + (threadIdx.x >> 6); i < a.n; i += nw) {  // wave = buffer
        View v;
        u64 fx[kMax], src[kMax], len[kMax];
        const Plan p = plan_one(a, i, v, fx, src, len);  // every lane: the same (wave-uniform) plan
        const u64 size = p.st ? v.L : p.size;
        const u64 at = a.pre[i / kTile].bytes + a.out_off[i];
        wave_sync_global();  // every lane has read its tile-relative offset
        if (lane == 0) {
            a.out_off[i] = at;
            if (i == a.n - 1) a.out_off[a.n] = at + size;
        }
        if (at + size > a.cap) {
            if (lane == 0) atomicOr(a.err, kErrCapacity);
            continue;
        }
        uint8_t* o = a.out + at;
        const uint8_t* nv = a.val + p.vstart;
        if (p.st || p.mode != kRemarshal) {
            const u64 L = v.L;
            const int w = scalar_w(sc, a.k);
            const bool patch = p.st == 0 && p.mode == kPatch;
            const u64 c = !w && patch ? min(p.vn, L - p.po - 4) : 0;  // copy() stops at the end
            put_piece(o, L, [&](u64 b) -> u32 {
                if (patch && w) {
                    if (b >= p.toff && b < p.toff + w) return nv[b - p.toff];
                } else if (patch) {
                    if (b >= p.po && b < p.po + 4) return (u32)(p.newn >> (8 * (b - p.po))) & 0xffu;
                    if (b >= p.po + 4 && b < p.po + 4 + c) return nv[b - p.po - 4];
                }
                return v.m[b];
            });
            continue;
        }
        // remarshal: marshal (main.go:196-368) with field k replaced; public: IDs restored, public part only
        u64 ids = 0;
        if (p.pub && v.L >= 13)
            for (int b = 0; b < 8; ++b) ids |= (u64)v.m[5 + b] << (8 * b);
        const u64 o2p = p.off2p_new;
        put_piece(o, 13, [&](u64 b) -> u32 {
            if (b == 0) return 1u;
            if (b < 5) return (u32)(o2p >> (8 * (b - 1))) & 0xffu;
            return (u32)(ids >> (8 * (b - 5))) & 0xffu;
        });
        const int segs = p.pub ? 1 : 2;
        for (int s = 0; s < segs; ++s) {
            u64 tab = s ? o2p + 1 : 13;
            u64 pay = tab + sc.table[s];
            if (s) put_piece(o + o2p, 1, [](u64) -> u32 { return 1u; });
            for (int j = 0; j < sc.nf; ++j) {
                if (sc.seg[j] != s) continue;
                const int w = scalar_w(sc, j);
                if (w) {
                    const u64 x = fx[j];
                    put_piece(o + tab, w, [&](u64 b) -> u32 { return (u32)(x >> (8 * b)) & 0xffu; });
                    tab += w;
                    continue;
                }
                const u64 rel = s ? pay - o2p : pay, cnt = len[j] >> sc.shift[j];
                put_piece(o + tab, 4, [&](u64 b) -> u32 { return (u32)(rel >> (8 * b)) & 0xffu; });
                put_piece(o + pay, 4, [&](u64 b) -> u32 { return (u32)(cnt >> (8 * b)) & 0xffu; });
                if (j == a.k)
                    put_piece(o + pay + 4, len[j], [&](u64 b) -> u32 { return nv[b]; });
                else
                    put_piece(o + pay + 4, len[j], [&](u64 b) -> u32 { return v.byte(src[j] + b); });
                tab += 4;
                pay += 4 + len[j];
            }
        }
    }
}

}  // namespace setter

size_t raw_set_ws_bytes(uint64_t n) {
    const u64 t = (n + setter::kTile - 1) / setter::kTile;
    return (size_t)(2 * t + 1) * sizeof(raw::Pair) + 256;
}

hipError_t launch_raw_set(const sym_field* f, int nf, int k, uint64_t n, const uint8_t* in, const uint64_t* rec_off,
                          const uint8_t* val, const uint64_t* val_off, uint8_t* out, uint64_t cap, uint64_t* out_off,
                          uint8_t* status, void* ws, unsigned* err, hipStream_t stream) {
    if (n == 0) return hipMemsetAsync(out_off, 0, sizeof(uint64_t), stream);
    setter::SetArgs a{};
    a.sc = flat::make_schema(f, nf);
    a.k = k;
    a.n = n;
    a.in = in;
    a.rec_off = rec_off;
    a.val = val;
    a.val_off = val_off;
    a.out = out;
    a.cap = cap;
    a.out_off = out_off;
    a.status = status;
    a.tiles = (n + setter::kTile - 1) / setter::kTile;
    a.agg = (raw::Pair*)ws;
    a.pre = a.agg + a.tiles;
    a.err = err;
    hipLaunchKernelGGL(setter::plan_kernel, dim3((unsigned)a.tiles), dim3(setter::kTile), 0, stream, a);
    hipError_t e = launch_tile_scan(a.agg, a.pre, a.tiles, stream);
    if (e != hipSuccess) return e;
    const u64 waves = (n + 3) / 4;
    const unsigned grid = (unsigned)(waves < 8192 ? waves : 8192);
    hipLaunchKernelGGL(setter::write_kernel, dim3(grid), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace symhip
