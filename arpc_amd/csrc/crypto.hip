// crypto.hip -- batched per-segment AES-256-GCM of Symphony records on gfx950.
//
// Restates EncryptSymphonyData / DecryptSymphonyData (pkg/transport/encryption.go:82-256) for n
// records per call: the public segment data[13:off2p] under the public key and the private
// segment data[off2p:] under the private key, each sealed as nonce(12) || ciphertext || tag(16)
// with Go's crypto/cipher GCM (12-byte nonce, 16-byte tag, no additional data).  Nonces are an
// input (24 bytes per record), the parity hook SURVEY.md 8f N4 asks for; production fills them
// from a CSPRNG as encryption.go:115-121 does.
//
//  * plan (thread = record): the header checks, the output size (a closed form of the input
//    header), per-tile totals; tile scan; apply -> output offsets.
//  * cipher (wave = record, grid-stride over a persistent grid; lane = 16-byte block): AES-256
//    with a 1 KiB T-table in LDS (the other three tables are byte rotations), CTR from
//    inc32(J0), and GHASH computed in parallel: lane b multiplies its ciphertext block by
//    H^(e-b) for its 64-block window [s, e) with Shoup 4-bit tables of H^1..H^64 in LDS, a wave
//    XOR-reduction sums the window, and windows chain by Horner (Y := Y * H^len xor window).
//    Decrypt authenticates both segments (and the private version byte) before any plaintext is
//    written; a record that fails gets zeros.  A record within one GHASH window decrypts in the
//    hashing pass (plaintext held in registers until the tags check); longer ones take a second
//    pass.
#include <cstring>

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"

namespace symhip {

namespace crypt {

using raw::Pair;

constexpr int kWaves = 8;  // 512-thread workgroups: one LDS copy of the tables serves 8 waves

// Device tables for one (public, private) key pair; built on the host (build_tables below).
struct Tables {
    u32 te0[256];           // T0[x] = 2S(x) | S(x) << 8 | S(x) << 16 | 3S(x) << 24
    u32 rk[2][60];          // AES-256 round keys (public, private): little-endian column words
    u32 red[16];            // GHASH: reduction of the 4 bits a right shift by 4 drops (top word)
    u32 pad[8];
    u32x4 ghash[2][64][16]; // [key][power - 1][nibble]: poly(nibble) * H^power, big-endian words
};
static_assert(sizeof(Tables) % 16 == 0, "Tables is copied to LDS in 16-byte pieces");

// The tables as the cipher reads them, in LDS, laid out against bank conflicts (round 6; round 5's
// counters: 52 % of the LDS-active cycles were bank conflicts, profiles/r05_counters_summary.txt):
//  * the T-table in 32 copies interleaved by word, te[x][c]: lane l reads copy l % 32, whose words all
//    sit in bank l % 32 (ds_read_b32 serves 32 lanes per cycle from banks (a/4) mod 32), so a wave's
//    random lookups never collide;
//  * the Shoup tables transposed, gh[key][nibble][power - 1]: the 16 entries of one power share one
//    group of 4 banks (ds_read_b128: 16 lanes per cycle over 64 banks), and the lanes of a window hash
//    consecutive powers, so their random nibbles hit different bank groups.
struct LdsTables {
    u32 te[256 * 32];
    u32 rk[2][60];
    u32 red[16];
    u32 pad[8];
    u32x4 gh[2][16][64];
};
static_assert(offsetof(LdsTables, gh) % 16 == 0, "16-byte GHASH entries");

__device__ __forceinline__ u32 rotl(u32 x, int s) { return (x << s) | (x >> (32 - s)); }
__device__ __forceinline__ u32 bswap(u32 x) { return __builtin_bswap32(x); }

// AES-256 encryption of one block (little-endian column words), T-table rounds.  T: this lane's copy
// of the interleaved table (LdsTables::te + lane % 32); entry x is T[32 x].
__device__ inline u32x4 aes_block(const u32* Tc, const u32* rk, u32x4 in) {
    auto T = [&](u32 x) { return Tc[x << 5]; };
    u32 w0 = in.x ^ rk[0], w1 = in.y ^ rk[1], w2 = in.z ^ rk[2], w3 = in.w ^ rk[3];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        const u32 t0 = T(w0 & 0xff) ^ rotl(T((w1 >> 8) & 0xff), 8) ^ rotl(T((w2 >> 16) & 0xff), 16) ^
                       rotl(T(w3 >> 24), 24) ^ rk[4 * r];
        const u32 t1 = T(w1 & 0xff) ^ rotl(T((w2 >> 8) & 0xff), 8) ^ rotl(T((w3 >> 16) & 0xff), 16) ^
                       rotl(T(w0 >> 24), 24) ^ rk[4 * r + 1];
        const u32 t2 = T(w2 & 0xff) ^ rotl(T((w3 >> 8) & 0xff), 8) ^ rotl(T((w0 >> 16) & 0xff), 16) ^
                       rotl(T(w1 >> 24), 24) ^ rk[4 * r + 2];
        const u32 t3 = T(w3 & 0xff) ^ rotl(T((w0 >> 8) & 0xff), 8) ^ rotl(T((w1 >> 16) & 0xff), 16) ^
                       rotl(T(w2 >> 24), 24) ^ rk[4 * r + 3];
        w0 = t0;
        w1 = t1;
        w2 = t2;
        w3 = t3;
    }
    auto S = [&](u32 x) { return (T(x) >> 8) & 0xffu; };
    const u32 o0 = S(w0 & 0xff) | (S((w1 >> 8) & 0xff) << 8) | (S((w2 >> 16) & 0xff) << 16) | (S(w3 >> 24) << 24);
    const u32 o1 = S(w1 & 0xff) | (S((w2 >> 8) & 0xff) << 8) | (S((w3 >> 16) & 0xff) << 16) | (S(w0 >> 24) << 24);
    const u32 o2 = S(w2 & 0xff) | (S((w3 >> 8) & 0xff) << 8) | (S((w0 >> 16) & 0xff) << 16) | (S(w1 >> 24) << 24);
    const u32 o3 = S(w3 & 0xff) | (S((w0 >> 8) & 0xff) << 8) | (S((w1 >> 16) & 0xff) << 16) | (S(w2 >> 24) << 24);
    return u32x4{o0 ^ rk[56], o1 ^ rk[57], o2 ^ rk[58], o3 ^ rk[59]};
}

// x * P in GF(2^128) (GCM bit order; big-endian words), M = the 4-bit table of P: entry v at M[64 v]
// (LdsTables::gh[key][.][power - 1]).
__device__ inline u32x4 gf_mul(u32x4 x, const u32x4* M, const u32* red) {
    u32x4 z = {0, 0, 0, 0};
    const u32 xw[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 31; k >= 0; --k) {  // nibble k = degrees 4k..4k+3, highest first (Horner)
        const u32 nib = (xw[k >> 3] >> (28 - 4 * (k & 7))) & 0xfu;
        const u32 t = z.w & 0xfu;
        z.w = (z.w >> 4) | (z.z << 28);
        z.z = (z.z >> 4) | (z.y << 28);
        z.y = (z.y >> 4) | (z.x << 28);
        z.x = (z.x >> 4) ^ red[t];
        z ^= M[nib << 6];
    }
    return z;
}

__device__ inline u32x4 wave_xor_u32x4(u32x4 v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        v.x ^= (u32)__shfl_xor((int)v.x, d, 64);
        v.y ^= (u32)__shfl_xor((int)v.y, d, 64);
        v.z ^= (u32)__shfl_xor((int)v.z, d, 64);
        v.w ^= (u32)__shfl_xor((int)v.w, d, 64);
    }
    return v;
}

__device__ inline u32 ld_le32(uintptr_t p) { return ld_u32(p); }
__device__ __forceinline__ u64 lane_u64c(u64 v, int l) {
    return (u64)(u32)__builtin_amdgcn_readlane((u32)v, l) | ((u64)(u32)__builtin_amdgcn_readlane((u32)(v >> 32), l) << 32);
}

// bytes [0, m) at p (m <= 16) as little-endian words, zero above m; reads only aligned blocks that
// hold wanted bytes
__device__ inline u32x4 load_partial(uintptr_t p, int m) {
    u32 r[4] = {0, 0, 0, 0};
    if (m > 0) or_window_global(p, 0, m, r);
    return u32x4{r[0], r[1], r[2], r[3]};
}

// bytes [0, m) of v to p: a full block is one byte-unaligned 16-byte store, a tail is byte stores
__device__ inline void store_bytes(uint8_t* p, u32x4 v, int m) {
    const u32 r[4] = {v.x, v.y, v.z, v.w};
    if (m == 16) {
        st16((uint8_t*)p, v, true);  // nontemporal: the cipher's records are written once
        return;
    }
    for (int t = 0; t < m; ++t) *(g_u8*)(p + t) = chunk_byte(r, t);
}

__device__ inline u32x4 counter_block(u32x4 nonce_le, u32 ctr) { return u32x4{nonce_le.x, nonce_le.y, nonce_le.z, bswap(ctr)}; }

// Per-record descriptor the plan leaves for the cipher, so that a record's geometry is one 16-byte
// load instead of a chain of dependent loads (offsets, then the header).
struct RecDesc {
    u64 s;  // stream offset
    u32 L;  // record bytes
    u32 o;  // offsetToPrivate; kNoWork: nothing to seal/open (bad header); kSlow: L >= 2^32, read it all
};
constexpr u32 kNoWork = 0xFFFFFFFFu, kSlow = 0xFFFFFFFEu;

// ---- plan: header checks and output sizes (encryption.go:84-95, 184-202, 313-318)
template <bool ENC>
__global__ __launch_bounds__(256) void plan_kernel(const uint8_t* in, const u64* rec_off, u64 n, u64* size,
                                                   uint8_t* status, Pair* agg, RecDesc* desc) {
    __shared__ u64 red_b[4];
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    u64 sz = 0;
    if (i < n) {
        const u64 s = rec_off[i], L = rec_off[i + 1] - s;
        uint8_t st = SYM_CRYPT_OK;
        if (L < 13) {
            st = SYM_CRYPT_TOO_SHORT;
        } else {
            const u64 o = ld_u32((uintptr_t)(in + s) + 1);
            if (ENC) {
                if (o < 13 || o > L) st = SYM_CRYPT_BAD_OFFSET;
                else sz = L + 28 + (o < L ? 28 : 0);
            } else {
                if (o < 41 || o > L) st = SYM_CRYPT_BAD_OFFSET;
                else if (o < L && L - o < 28) st = SYM_CRYPT_AUTH_PRIVATE;  // "encrypted data too short"
                else sz = 13 + (o - 41) + (o < L ? L - o - 28 : 0);
            }
        }
        status[i] = st;
        size[i] = sz;
        const u64 o = L >= 13 ? ld_u32((uintptr_t)(in + s) + 1) : 0;
        desc[i] = RecDesc{s, (u32)L, st != SYM_CRYPT_OK ? kNoWork : L >> 32 ? kSlow : (u32)o};
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 w = wave_sum_u64(sz);
    if (lane == 0) red_b[wave] = w;
    __syncthreads();
    if (threadIdx.x == 0) agg[blockIdx.x] = Pair{red_b[0] + red_b[1] + red_b[2] + red_b[3], 0};
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

struct Args {
    const uint8_t* in;
    const u64* rec_off;
    u64 n;
    const uint8_t* nonces;  // ENC: 24 bytes per record
    const u64* out_off;
    uint8_t* status;
    uint8_t* out;
    const Tables* tables;
    const RecDesc* desc;
};

__device__ inline u32x4 to_be(u32x4 v) { return u32x4{bswap(v.x), bswap(v.y), bswap(v.z), bswap(v.w)}; }

// One 64-slot window of a segment's GHASH.  A segment of nb data blocks has nb + 1 slots: block i
// (ciphertext) and, last, the length block [0]64 || [8 len]64.  Slot i of a window contributes
// X_i * H^(e - i), e = one past the segment's last slot in the window, and the length slot adds
// E(K, J0); the window's terms are XOR-reduced and chained by Horner (Y := Y * H^cnt xor window).
// A segment that fits one window (63 data blocks) is therefore one parallel multiply per lane and
// one reduction: no serial GF multiplications.
template <int W>
__device__ inline u32x4 subwave_xor_u32x4(u32x4 v) {
#pragma unroll
    for (int d = W / 2; d > 0; d >>= 1) {
        v.x ^= (u32)__shfl_xor((int)v.x, d, 64);
        v.y ^= (u32)__shfl_xor((int)v.y, d, 64);
        v.z ^= (u32)__shfl_xor((int)v.z, d, 64);
        v.w ^= (u32)__shfl_xor((int)v.w, d, 64);
    }
    return v;
}

template <int W>
__device__ inline u32x4 ghash_fold(u32x4 y, bool first, bool mine, u32x4 term, u32 cnt, const LdsTables& T, int key) {
    u32x4 c = mine ? term : u32x4{0, 0, 0, 0};
    c = subwave_xor_u32x4<W>(c);
    if (cnt == 0) return y;
    return first ? c : (gf_mul(y, &T.gh[key][0][cnt - 1], T.red) ^ c);
}

// A record's geometry (the lane's own record, loaded one pair ahead).
struct Geo {
    u64 s, L, o, oo;  // stream offset, bytes, offsetToPrivate, output offset
    bool work;
};
__device__ inline Geo load_geo(const Args& a, u64 r) {
    Geo g{0, 0, 0, 0, false};
    if (r >= a.n) return g;
    const RecDesc d = a.desc[r];
    g.oo = a.out_off[r];
    g.work = d.o != kNoWork;
    g.s = d.s;
    g.L = d.L;
    g.o = d.o;
    if (d.o == kSlow) {  // a record of 4 GiB or more: the full-width values
        g.L = a.rec_off[r + 1] - d.s;
        g.o = ld_u32((uintptr_t)(a.in + d.s) + 1);
    }
    return g;
}

// GHASH slots of a record (data blocks + one length block per segment), 0 when it has no work
__device__ inline u32 record_slots(const Geo& g, bool enc) {
    if (!g.work) return 0;
    const u64 np = enc ? g.o - 13 : g.o - 41, nv = g.o < g.L ? (enc ? g.L - g.o : g.L - g.o - 28) : 0;
    return (u32)((np + 15) / 16 + 1 + (g.o < g.L ? (nv + 15) / 16 + 1 : 0));
}
__device__ inline Geo lane_geo(const Geo& g, int l) {  // lane l's geometry, wave-uniform
    Geo u;
    u.s = lane_u64c(g.s, l);
    u.L = lane_u64c(g.L, l);
    u.o = lane_u64c(g.o, l);
    u.oo = lane_u64c(g.oo, l);
    u.work = __builtin_amdgcn_readlane((int)g.work, l) != 0;
    return u;
}

// One record on a sub-wave of W lanes (sl = lane within it).  W = 32 packs two records per wave.
template <bool ENC, int W>
__device__ void seal_or_open(const Args& a, const LdsTables& T, const u32* ts, u64 r, const Geo& G, int sl) {
    const u64 L = G.L, o = G.o;
    const uintptr_t d = (uintptr_t)(a.in + G.s);
    uint8_t* const q = a.out + G.oo;
    const bool priv = o < L;
    // segment geometry: plaintext/ciphertext source, length, destination, nonce
    u64 np, nv;
    uintptr_t src_pub, src_priv, non_pub, non_priv;
    uint8_t *dst_pub, *dst_priv;
    if (ENC) {
        np = o - 13;
        nv = priv ? L - o : 0;
        src_pub = d + 13;
        src_priv = d + o;
        non_pub = (uintptr_t)(a.nonces + 24 * r);
        non_priv = non_pub + 12;
        dst_pub = q + 25;
        dst_priv = q + 13 + 28 + np + 12;
    } else {
        np = o - 41;
        nv = priv ? L - o - 28 : 0;
        src_pub = d + 25;
        src_priv = d + o + 12;
        non_pub = d + 13;
        non_priv = d + o;
        dst_pub = q + 13;
        dst_priv = q + 13 + np;
    }
    const u32x4 nonce_pub = {ld_le32(non_pub), ld_le32(non_pub + 4), ld_le32(non_pub + 8), 0};
    const u32x4 nonce_priv = priv ? u32x4{ld_le32(non_priv), ld_le32(non_priv + 4), ld_le32(non_priv + 8), 0}
                                  : u32x4{0, 0, 0, 0};
    const u32 nbp = (u32)((np + 15) / 16), nbv = (u32)((nv + 15) / 16);
    const u32 nsp = nbp + 1, nsv = priv ? nbv + 1 : 0, ns = nsp + nsv;  // GHASH slots
    u32x4 y_pub = {0, 0, 0, 0}, y_priv = {0, 0, 0, 0};
    u32 version = 1;  // DEC: first private plaintext byte
    // DEC of a record whose GHASH slots fit one window (config 2's 350-byte records: 24 slots): pass 1
    // also runs CTR and keeps the lane's plaintext block in registers until the tags are checked,
    // so AES overlaps GHASH as in ENC and no second pass re-reads the ciphertext
    const bool one = !ENC && ns <= (u32)W;
    u32x4 held = {0, 0, 0, 0};
    int held_m = 0;
    uint8_t* held_dst = nullptr;
    // ---- pass 1: ENC encrypts, writes and hashes; DEC hashes the ciphertext (+ private byte 0)
    for (u32 w0 = 0; w0 < ns; w0 += W) {
        const u32 g = w0 + sl;
        const bool act = g < ns, is_priv = g >= nsp;
        const u32 i = is_priv ? g - nsp : g;  // slot within the segment
        const u32 nbs = is_priv ? nbv : nbp;
        const bool is_len = act && i == nbs, is_data = act && i < nbs;
        const u64 seg_len = is_priv ? nv : np;
        const int m = is_data ? (int)min((u64)16, seg_len - 16 * (u64)i) : 0;
        const u32x4 x = load_partial((is_priv ? src_priv : src_pub) + 16 * (u64)i, m);
        const bool ver = !ENC && is_priv && is_data && i == 0;
        u32x4 ks = {0, 0, 0, 0};
        if (is_len || ((ENC || one) && is_data) || ver)  // J0 for the tag, J0 + 1 + i for block i
            ks = aes_block(ts, T.rk[is_priv ? 1 : 0],
                           counter_block(is_priv ? nonce_priv : nonce_pub, is_len ? 1u : i + 2));
        u32x4 c = x;
        if (ENC && is_data) {
            c = (x ^ ks) & u32x4{dword_mask(0, m, 0), dword_mask(0, m, 1), dword_mask(0, m, 2), dword_mask(0, m, 3)};
            store_bytes((is_priv ? dst_priv : dst_pub) + 16 * (u64)i, c, m);
        }
        if (ver) version = (x.x ^ ks.x) & 0xffu;
        if (one && is_data) {
            held = x ^ ks;
            held_m = m;
            held_dst = (is_priv ? dst_priv : dst_pub) + 16 * (u64)i;
        }
        const u64 bits = seg_len * 8;
        const u32x4 X = is_len ? u32x4{0, 0, (u32)(bits >> 32), (u32)bits} : to_be(c);
        const u32 e = min(is_priv ? ns : nsp, w0 + W);
        u32x4 term = {0, 0, 0, 0};
        if (act) term = gf_mul(X, &T.gh[is_priv ? 1 : 0][0][e - g - 1], T.red);
        if (is_len) term ^= to_be(ks);
        const u32 cnt_pub = w0 < nsp ? min(nsp, w0 + W) - w0 : 0;
        y_pub = ghash_fold<W>(y_pub, w0 == 0, act && !is_priv, term, cnt_pub, T, 0);
        if (nsv) {
            const u32 lo = w0 > nsp ? w0 : nsp, hi = min(ns, w0 + W);
            y_priv = ghash_fold<W>(y_priv, lo == nsp, act && is_priv, term, hi > lo ? hi - lo : 0, T, 1);
        }
    }
    if (!ENC) version = (u32)__shfl((int)version, (int)(nsp & (W - 1)), W);  // the lane of private slot 0
    const u32x4 tag_pub = to_be(y_pub), tag_priv = to_be(y_priv);  // little-endian words
    if (ENC) {
        // header (offsetToPrivate patched) and nonces: 37 bytes, one per lane of the sub-wave (lanes
        // 0..4 take a second when W = 32), every load issued before any store -- byte copies by one
        // lane are a chain of round trips (a store may alias the next load), and were most of the
        // cipher's time (round 6: 2.1 -> see DESIGN.md section 4)
        const u32 no = (u32)(13 + 28 + np);
        auto src = [&](int t) -> uintptr_t {  // 0: a patched byte (no load)
            return t < 13 ? (t >= 1 && t <= 4 ? 0 : d + t) : t < 25 ? non_pub + (t - 13) : non_priv + (t - 25);
        };
        auto dst = [&](int t) -> uint8_t* { return t < 25 ? q + t : q + 41 + np + (t - 25); };
        const int t0 = sl, t1 = sl + W, nt = priv ? 37 : 25;
        const uintptr_t a0 = t0 < nt ? src(t0) : 0, a1 = t1 < nt ? src(t1) : 0;
        auto patched = [&](int t) { return t >= 1 && t <= 4 ? (no >> (8 * (t - 1))) & 0xffu : 0u; };
        const u32 b0 = a0 ? ld_u8(a0) : patched(t0);
        const u32 b1 = a1 ? ld_u8(a1) : patched(t1);
        if (t0 < nt) *dst(t0) = (uint8_t)b0;
        if (t1 < nt) *dst(t1) = (uint8_t)b1;
        if (sl == 0) {  // tags
            store_bytes(q + 25 + np, tag_pub, 16);
            if (priv) store_bytes(q + 41 + np + 12 + nv, tag_priv, 16);
        }
        return;
    }
    // ---- DEC: authenticate, then decrypt (or zero the record's output)
    auto tag_at = [&](uintptr_t p) { return u32x4{ld_le32(p), ld_le32(p + 4), ld_le32(p + 8), ld_le32(p + 12)}; };
    const u32x4 want_pub = tag_at(d + o - 16);
    const u32x4 want_priv = priv ? tag_at(d + L - 16) : u32x4{0, 0, 0, 0};
    uint8_t st = SYM_CRYPT_OK;
    const u32x4 dp = want_pub ^ tag_pub, dv = want_priv ^ tag_priv;
    if (dp.x | dp.y | dp.z | dp.w) st = SYM_CRYPT_AUTH_PUBLIC;
    else if (priv && (dv.x | dv.y | dv.z | dv.w)) st = SYM_CRYPT_AUTH_PRIVATE;
    else if (priv && (nv < 1 || version != 1)) st = SYM_CRYPT_BAD_VERSION;
    const u64 size = 13 + np + nv;
    if (st != SYM_CRYPT_OK) {
        if (sl == 0) a.status[r] = st;
        for (u64 t = (u64)sl; t < size; t += W) q[t] = 0;
        return;
    }
    if (one && held_m) store_bytes(held_dst, held, held_m);
    const u32 nb = one ? 0u : nbp + nbv;
    for (u32 g0 = 0; g0 < nb; g0 += W) {
        const u32 g = g0 + sl;
        if (g >= nb) continue;
        const bool is_priv = g >= nbp;
        const u32 b = is_priv ? g - nbp : g;
        const u64 seg_len = is_priv ? nv : np;
        const int m = (int)min((u64)16, seg_len - 16 * (u64)b);
        const u32x4 x = load_partial((is_priv ? src_priv : src_pub) + 16 * (u64)b, m);
        const u32x4 ks = aes_block(ts, T.rk[is_priv ? 1 : 0], counter_block(is_priv ? nonce_priv : nonce_pub, b + 2));
        store_bytes((is_priv ? dst_priv : dst_pub) + 16 * (u64)b, x ^ ks, m);
    }
    if (sl < 13) {  // the header, offsetToPrivate patched: one byte per lane (see ENC above)
        const u32 no = (u32)(13 + np);
        q[sl] = sl >= 1 && sl <= 4 ? (uint8_t)(no >> (8 * (sl - 1))) : (uint8_t)ld_u8(d + sl);
    }
}

// A wave takes records in pairs: when both fit 32 GHASH slots (records under ~450 bytes) each half
// of the wave seals one of them; otherwise the whole wave takes them one after the other.
template <bool ENC>
__global__ __launch_bounds__(kWaves * 64) void cipher_kernel(Args a) {
    __shared__ LdsTables T;
    {  // stage the tables (65 KiB in LdsTables' layout) once per workgroup; the grid is persistent
        // (every thread's loads issued before its LDS stores: one round trip, not one per entry)
        const Tables& g = *a.tables;
        const int tid = threadIdx.x;
        static_assert(kWaves * 64 == 512, "staging assumes 512 threads");
        if (tid < 256) {  // T-table entry tid -> its 32 copies
            const u32 v = g.te0[tid];
#pragma unroll
            for (int c = 0; c < 32; ++c) T.te[32 * tid + c] = v;
        } else {  // GHASH entries 8 (tid - 256) .. +7, transposed
            u32x4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 8 * (tid - 256) + j;
                v[j] = g.ghash[k >> 10][k & 63][(k >> 6) & 15];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 8 * (tid - 256) + j;
                T.gh[k >> 10][(k >> 6) & 15][k & 63] = v[j];
            }
        }
        if (tid < 2 * 60) T.rk[tid / 60][tid % 60] = g.rk[tid / 60][tid % 60];
        if (tid >= 128 && tid < 144) T.red[tid - 128] = g.red[tid - 128];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const u32* ts = T.te + (lane & 31);  // this lane's copy of the T-table
    const u64 nw = (u64)gridDim.x * kWaves;
    const u64 npairs = (a.n + 1) / 2;
    // lanes 0..31 hold the pair's first record's geometry, 32..63 the second's; the next pair's is
    // loaded while this one is sealed
    u64 p = (u64)blockIdx.x * kWaves + (threadIdx.x >> 6);
    Geo cur = load_geo(a, 2 * p + (lane >> 5));
    for (; p < npairs; p += nw) {  // wave-uniform
        const Geo nxt = load_geo(a, 2 * (p + nw) + (lane >> 5));
        const u64 r0 = 2 * p, r1 = 2 * p + 1;
        const u32 sl_mine = record_slots(cur, ENC);
        const u32 s0 = __builtin_amdgcn_readlane(sl_mine, 0), s1 = __builtin_amdgcn_readlane(sl_mine, 32);  // uniform
        if (s0 <= 32 && s1 <= 32) {
            const u64 r = lane < 32 ? r0 : r1;
            if (sl_mine != 0) seal_or_open<ENC, 32>(a, T, ts, r, cur, lane & 31);
        } else {
            if (s0) seal_or_open<ENC, 64>(a, T, ts, r0, lane_geo(cur, 0), lane);
            if (s1) seal_or_open<ENC, 64>(a, T, ts, r1, lane_geo(cur, 32), lane);
        }
        cur = nxt;
    }
}

inline u64 tiles(u64 m) { return (m + 255) / 256; }
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// ---------------------------------------------------------------- host: key schedule and GHASH tables
namespace host {

const uint8_t kSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82, 0xc9,
    0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f,
    0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, 0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07,
    0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3,
    0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58,
    0xcf, 0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3,
    0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec, 0x5f,
    0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73, 0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88,
    0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac,
    0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a,
    0xae, 0x08, 0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, 0x70,
    0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11,
    0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, 0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42,
    0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x >> 7) * 0x1b)); }

// FIPS 197 5.2 (Nk = 8): 60 words, word i = bytes 4i..4i+3 little-endian (a state column)
void expand(const uint8_t key[32], u32 rk[60]) {
    uint8_t w[60][4];
    memcpy(w, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint8_t t[4] = {w[i - 1][0], w[i - 1][1], w[i - 1][2], w[i - 1][3]};
        if (i % 8 == 0) {
            const uint8_t r0 = t[0];
            t[0] = (uint8_t)(kSbox[t[1]] ^ rcon);
            t[1] = kSbox[t[2]];
            t[2] = kSbox[t[3]];
            t[3] = kSbox[r0];
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            for (int b = 0; b < 4; ++b) t[b] = kSbox[t[b]];
        }
        for (int b = 0; b < 4; ++b) w[i][b] = (uint8_t)(w[i - 8][b] ^ t[b]);
    }
    for (int i = 0; i < 60; ++i) rk[i] = (u32)w[i][0] | ((u32)w[i][1] << 8) | ((u32)w[i][2] << 16) | ((u32)w[i][3] << 24);
}

void encrypt(const u32 rk[60], const uint8_t in[16], uint8_t out[16]) {  // byte-wise, for H only
    uint8_t s[16];
    for (int b = 0; b < 16; ++b) s[b] = in[b] ^ (uint8_t)(rk[b / 4] >> (8 * (b % 4)));
    for (int round = 1; round <= 14; ++round) {
        uint8_t t[16];
        for (int b = 0; b < 16; ++b) t[b] = kSbox[s[b]];
        for (int c = 0; c < 4; ++c)
            for (int r = 0; r < 4; ++r) s[c * 4 + r] = t[((c + r) % 4) * 4 + r];
        if (round < 14)
            for (int c = 0; c < 4; ++c) {
                uint8_t* col = s + 4 * c;
                const uint8_t a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3], x = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
                col[0] = (uint8_t)(a0 ^ x ^ xtime((uint8_t)(a0 ^ a1)));
                col[1] = (uint8_t)(a1 ^ x ^ xtime((uint8_t)(a1 ^ a2)));
                col[2] = (uint8_t)(a2 ^ x ^ xtime((uint8_t)(a2 ^ a3)));
                col[3] = (uint8_t)(a3 ^ x ^ xtime((uint8_t)(a3 ^ a0)));
            }
        for (int b = 0; b < 16; ++b) s[b] ^= (uint8_t)(rk[4 * round + b / 4] >> (8 * (b % 4)));
    }
    memcpy(out, s, 16);
}

struct V128 {
    u32 w[4];  // big-endian words: w[0] = bytes 0..3
};

V128 gf_mul(V128 x, V128 y) {  // SP 800-38D Algorithm 1
    V128 z = {{0, 0, 0, 0}}, v = y;
    for (int i = 0; i < 128; ++i) {
        if ((x.w[i >> 5] >> (31 - (i & 31))) & 1)
            for (int k = 0; k < 4; ++k) z.w[k] ^= v.w[k];
        const u32 lsb = v.w[3] & 1;
        v.w[3] = (v.w[3] >> 1) | (v.w[2] << 31);
        v.w[2] = (v.w[2] >> 1) | (v.w[1] << 31);
        v.w[1] = (v.w[1] >> 1) | (v.w[0] << 31);
        v.w[0] >>= 1;
        if (lsb) v.w[0] ^= 0xe1000000u;
    }
    return z;
}

}  // namespace host

void build_tables(const uint8_t pub_key[32], const uint8_t priv_key[32], Tables& t) {
    memset(&t, 0, sizeof(t));
    for (int x = 0; x < 256; ++x) {
        const u32 s = host::kSbox[x], s2 = host::xtime((uint8_t)s), s3 = s2 ^ s;
        t.te0[x] = s2 | (s << 8) | (s << 16) | (s3 << 24);
    }
    const uint8_t* keys[2] = {pub_key, priv_key};
    for (int k = 0; k < 2; ++k) {
        host::expand(keys[k], t.rk[k]);
        uint8_t zero[16] = {0}, h[16];
        host::encrypt(t.rk[k], zero, h);
        host::V128 H, P;
        for (int w = 0; w < 4; ++w)
            H.w[w] = ((u32)h[4 * w] << 24) | ((u32)h[4 * w + 1] << 16) | ((u32)h[4 * w + 2] << 8) | h[4 * w + 3];
        P = H;
        for (int j = 0; j < 64; ++j) {  // table of H^(j+1)
            for (int v = 0; v < 16; ++v) {
                host::V128 nv = {{(u32)v << 28, 0, 0, 0}};
                const host::V128 m = host::gf_mul(nv, P);
                t.ghash[k][j][v] = u32x4{m.w[0], m.w[1], m.w[2], m.w[3]};
            }
            P = host::gf_mul(P, H);
        }
    }
    for (int v = 0; v < 16; ++v) {  // the 4 dropped bits, shifted out one at a time with reduction
        u32 w[4] = {0, 0, 0, (u32)v};
        for (int s = 0; s < 4; ++s) {
            const u32 lsb = w[3] & 1;
            w[3] = (w[3] >> 1) | (w[2] << 31);
            w[2] = (w[2] >> 1) | (w[1] << 31);
            w[1] = (w[1] >> 1) | (w[0] << 31);
            w[0] >>= 1;
            if (lsb) w[0] ^= 0xe1000000u;
        }
        t.red[v] = w[0];
    }
}

}  // namespace crypt

size_t crypt_tables_bytes() { return sizeof(crypt::Tables); }
void crypt_build_tables(const uint8_t pub_key[32], const uint8_t priv_key[32], void* host_tables) {
    crypt::build_tables(pub_key, priv_key, *(crypt::Tables*)host_tables);
}

size_t crypt_ws_bytes(u64 n) {
    return crypt::al256(n * 8) + 2 * crypt::al256((crypt::tiles(n) + 1) * sizeof(raw::Pair)) +
           crypt::al256(n * sizeof(crypt::RecDesc));
}

hipError_t launch_crypt(bool enc, const uint8_t* in, const u64* rec_off, u64 n, const uint8_t* nonces,
                        const void* d_tables, uint8_t* out, u64* out_off, uint8_t* status, void* ws, int num_cus,
                        hipStream_t stream) {
    using raw::Pair;
    u64* size = (u64*)ws;
    Pair* agg = (Pair*)((char*)ws + crypt::al256(n * 8));
    Pair* tpre = (Pair*)((char*)agg + crypt::al256((crypt::tiles(n) + 1) * sizeof(Pair)));
    crypt::RecDesc* desc = (crypt::RecDesc*)((char*)tpre + crypt::al256((crypt::tiles(n) + 1) * sizeof(Pair)));
    const dim3 g((unsigned)crypt::tiles(n)), b(256);
    if (enc) hipLaunchKernelGGL(crypt::plan_kernel<true>, g, b, 0, stream, in, rec_off, n, size, status, agg, desc);
    else hipLaunchKernelGGL(crypt::plan_kernel<false>, g, b, 0, stream, in, rec_off, n, size, status, agg, desc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = launch_tile_scan(agg, tpre, crypt::tiles(n), stream)) != hipSuccess) return e;
    hipLaunchKernelGGL(crypt::apply_kernel, g, b, 0, stream, (const u64*)size, n, (const Pair*)tpre, out_off);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    crypt::Args a{in, rec_off, n, nonces, out_off, status, out, (const crypt::Tables*)d_tables, desc};
    const u64 want = (n + crypt::kWaves - 1) / crypt::kWaves;
    const u64 cap = (u64)num_cus * 2;  // resident: 66 KB of LDS tables per workgroup, two per CU
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    if (enc) hipLaunchKernelGGL(crypt::cipher_kernel<true>, dim3(grid), dim3(crypt::kWaves * 64), 0, stream, a);
    else hipLaunchKernelGGL(crypt::cipher_kernel<false>, dim3(grid), dim3(crypt::kWaves * 64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace symhip
