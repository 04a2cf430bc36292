/*
 * crypto_oracle.c -- CPU restatement of aRPC's per-segment AES-256-GCM of Symphony data.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the HIP segment cipher (arpc_amd/csrc/crypto.hip).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * The cipher itself lives in Go's standard library (crypto/aes, crypto/cipher.NewGCM: 12-byte
 * nonce, 16-byte tag, no additional data), which this image cannot run.  It is restated from its
 * published specifications: AES-256 (FIPS 197: key expansion with Nk = 8, 14 rounds) and GCM
 * (NIST SP 800-38D: H = E(K, 0^128), J0 = IV || 0^31 || 1, CTR from inc32(J0), GHASH over the
 * ciphertext and the 64-bit bit lengths, tag = E(K, J0) xor S).
 * Parity status: pinned by the published GCM test vectors (McGrew-Viega test cases 13-15, the
 * AES-256 ones) and by OpenSSL's EVP_aes_256_gcm (the system libcrypto, loaded by the tests only)
 * on random inputs -- tests/test_crypto.py.
 *
 * What it restates around the cipher (paths relative to the reference root):
 *   EncryptSymphonyData: len >= 13; 13 <= offsetToPrivate <= len; public = data[13:off2p] sealed
 *     with the public key, private = data[off2p:] (with its version byte) sealed with the private
 *     key when off2p < len; a sealed segment = nonce(12) || ciphertext || tag(16); output =
 *     header(13, offsetToPrivate := 13 + len(sealed public)) || sealed public || sealed private
 *                                        pkg/transport/encryption.go:82-171, 262-298
 *   DecryptSymphonyData: len >= 13; 41 <= offsetToPrivate <= len; open both segments (a sealed
 *     private segment < 28 bytes or a failed tag is an error); the private plaintext must start
 *     with 0x01; output = header with offsetToPrivate := 13 + len(public plaintext) || plaintexts
 *                                        pkg/transport/encryption.go:183-256, 300-335
 * Batch conventions (where Go panics on one message): a record's output size follows from its
 * header alone (0 for TOO_SHORT / BAD_OFFSET and for a private segment shorter than nonce + tag);
 * a record that fails authentication or the version check gets a status and zero bytes of that
 * size.  Nonces: production draws 24 random bytes per message (encryption.go:115-121); here they
 * are an input (public nonce = bytes [0, 12), private = [12, 24) of the record's 24) -- the test
 * hook SURVEY.md 8f N4 asks for.
 */
#include <stdint.h>
#include <string.h>

#define CRYPT_OK 0
#define CRYPT_TOO_SHORT 1   /* "too short for header" */
#define CRYPT_BAD_OFFSET 2  /* "invalid offsetToPrivate" / "invalid encrypted offsetToPrivate" */
#define CRYPT_AUTH_PUBLIC 3 /* public segment: "message authentication failed" */
#define CRYPT_AUTH_PRIVATE 4 /* private segment: too short, or "message authentication failed" */
#define CRYPT_BAD_VERSION 5 /* "invalid decrypted private segment: missing or incorrect version byte" */

static const uint8_t SBOX[256] = {
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

typedef struct {
    uint8_t rk[15][16]; /* 15 round keys (AES-256) */
} Aes;

static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x >> 7) * 0x1b)); }

/* FIPS 197 5.2, Nk = 8. */
static void aes_expand(Aes* a, const uint8_t key[32]) {
    uint8_t w[60][4];
    memcpy(w, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint8_t t[4] = {w[i - 1][0], w[i - 1][1], w[i - 1][2], w[i - 1][3]};
        if (i % 8 == 0) {
            const uint8_t r0 = t[0];
            t[0] = (uint8_t)(SBOX[t[1]] ^ rcon);
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[r0];
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            for (int b = 0; b < 4; ++b) t[b] = SBOX[t[b]];
        }
        for (int b = 0; b < 4; ++b) w[i][b] = (uint8_t)(w[i - 8][b] ^ t[b]);
    }
    memcpy(a->rk, w, sizeof(a->rk));
}

/* FIPS 197 5.1: state column-major, s[c*4 + r]. */
static void aes_encrypt(const Aes* a, const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int b = 0; b < 16; ++b) s[b] = in[b] ^ a->rk[0][b];
    for (int round = 1; round <= 14; ++round) {
        uint8_t t[16];
        for (int b = 0; b < 16; ++b) t[b] = SBOX[s[b]];
        for (int c = 0; c < 4; ++c) /* ShiftRows: row r rotates left by r */
            for (int r = 0; r < 4; ++r) s[c * 4 + r] = t[((c + r) % 4) * 4 + r];
        if (round < 14)
            for (int c = 0; c < 4; ++c) { /* MixColumns */
                uint8_t* col = s + 4 * c;
                const uint8_t a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3], x = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
                col[0] = (uint8_t)(a0 ^ x ^ xtime((uint8_t)(a0 ^ a1)));
                col[1] = (uint8_t)(a1 ^ x ^ xtime((uint8_t)(a1 ^ a2)));
                col[2] = (uint8_t)(a2 ^ x ^ xtime((uint8_t)(a2 ^ a3)));
                col[3] = (uint8_t)(a3 ^ x ^ xtime((uint8_t)(a3 ^ a0)));
            }
        for (int b = 0; b < 16; ++b) s[b] ^= a->rk[round][b];
    }
    memcpy(out, s, 16);
}

/* SP 800-38D Algorithm 1: x := x * y in GF(2^128), bit 0 = MSB of byte 0. */
static void gf_mul(uint8_t x[16], const uint8_t y[16]) {
    uint8_t z[16] = {0}, v[16];
    memcpy(v, y, 16);
    for (int i = 0; i < 128; ++i) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1)
            for (int b = 0; b < 16; ++b) z[b] ^= v[b];
        const int lsb = v[15] & 1;
        for (int b = 15; b > 0; --b) v[b] = (uint8_t)((v[b] >> 1) | (v[b - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xe1;
    }
    memcpy(x, z, 16);
}

/* Seal (enc = 1: writes tag) or open (enc = 0: returns 1 when tag matches) n bytes. */
static int gcm(const Aes* a, const uint8_t nonce[12], const uint8_t* in, uint64_t n, uint8_t* out, uint8_t tag[16],
               int enc) {
    uint8_t h[16] = {0}, j0[16], ctr[16], ks[16], y[16] = {0};
    aes_encrypt(a, h, h);
    memcpy(j0, nonce, 12);
    j0[12] = j0[13] = j0[14] = 0;
    j0[15] = 1;
    memcpy(ctr, j0, 16);
    for (uint64_t off = 0; off < n; off += 16) {
        const uint32_t c =
            ((uint32_t)ctr[12] << 24 | (uint32_t)ctr[13] << 16 | (uint32_t)ctr[14] << 8 | ctr[15]) + 1u; /* inc32 */
        ctr[12] = (uint8_t)(c >> 24);
        ctr[13] = (uint8_t)(c >> 16);
        ctr[14] = (uint8_t)(c >> 8);
        ctr[15] = (uint8_t)c;
        aes_encrypt(a, ctr, ks);
        const uint64_t m = n - off < 16 ? n - off : 16;
        for (uint64_t b = 0; b < m; ++b) {
            const uint8_t ci = enc ? (uint8_t)(in[off + b] ^ ks[b]) : in[off + b];
            if (out) out[off + b] = (uint8_t)(in[off + b] ^ ks[b]);
            y[b] ^= ci;
        }
        gf_mul(y, h);
    }
    const uint64_t bits = n * 8; /* [len(A)]64 = 0 || [len(C)]64 */
    for (int b = 0; b < 8; ++b) y[15 - b] ^= (uint8_t)(bits >> (8 * b));
    gf_mul(y, h);
    uint8_t ek[16];
    aes_encrypt(a, j0, ek);
    int ok = 1;
    for (int b = 0; b < 16; ++b) {
        const uint8_t t = (uint8_t)(ek[b] ^ y[b]);
        if (enc) tag[b] = t;
        else ok &= tag[b] == t;
    }
    return ok;
}

/* One-shot AES-256-GCM seal, empty AAD (published-vector tests). */
void sym_oracle_gcm_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* in, uint64_t n, uint8_t* out,
                         uint8_t tag[16]) {
    Aes a;
    aes_expand(&a, key);
    gcm(&a, nonce, in, n, out, tag, 1);
}

static uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static void wr32(uint8_t* p, uint32_t v) {
    for (int b = 0; b < 4; ++b) p[b] = (uint8_t)(v >> (8 * b));
}

/* EncryptSymphonyData over n records; returns the output bytes (out_off[n]). */
uint64_t sym_oracle_encrypt_batch(uint64_t n, const uint8_t* in, const uint64_t* rec_off, const uint8_t pub_key[32],
                                  const uint8_t priv_key[32], const uint8_t* nonces, uint8_t* out, uint64_t* out_off,
                                  uint8_t* status) {
    Aes pub, priv;
    aes_expand(&pub, pub_key);
    aes_expand(&priv, priv_key);
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* d = in + rec_off[i];
        const uint64_t L = rec_off[i + 1] - rec_off[i];
        out_off[i] = w;
        if (L < 13) {
            status[i] = CRYPT_TOO_SHORT;
            continue;
        }
        const uint64_t o = rd32(d + 1);
        if (o < 13 || o > L) {
            status[i] = CRYPT_BAD_OFFSET;
            continue;
        }
        status[i] = CRYPT_OK;
        uint8_t* r = out + w;
        const uint64_t np = o - 13, sp = 12 + np + 16;
        memcpy(r, d, 13);
        wr32(r + 1, (uint32_t)(13 + sp));
        memcpy(r + 13, nonces + 24 * i, 12);
        gcm(&pub, nonces + 24 * i, d + 13, np, r + 25, r + 25 + np, 1);
        w += 13 + sp;
        if (o < L) {
            const uint64_t nv = L - o;
            uint8_t* q = r + 13 + sp;
            memcpy(q, nonces + 24 * i + 12, 12);
            gcm(&priv, nonces + 24 * i + 12, d + o, nv, q + 12, q + 12 + nv, 1);
            w += 12 + nv + 16;
        }
    }
    out_off[n] = w;
    return w;
}

/* DecryptSymphonyData over n records; returns the output bytes (out_off[n]). */
uint64_t sym_oracle_decrypt_batch(uint64_t n, const uint8_t* in, const uint64_t* rec_off, const uint8_t pub_key[32],
                                  const uint8_t priv_key[32], uint8_t* out, uint64_t* out_off, uint8_t* status) {
    Aes pub, priv;
    aes_expand(&pub, pub_key);
    aes_expand(&priv, priv_key);
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* d = in + rec_off[i];
        const uint64_t L = rec_off[i + 1] - rec_off[i];
        out_off[i] = w;
        if (L < 13) {
            status[i] = CRYPT_TOO_SHORT;
            continue;
        }
        const uint64_t o = rd32(d + 1);
        if (o < 13 + 28 || o > L) {
            status[i] = CRYPT_BAD_OFFSET;
            continue;
        }
        if (o < L && L - o < 28) { /* "encrypted data too short" */
            status[i] = CRYPT_AUTH_PRIVATE;
            continue;
        }
        const uint64_t np = o - 41, nv = o < L ? L - o - 28 : 0, size = 13 + np + nv;
        uint8_t* r = out + w;
        w += size;
        uint8_t tag[16];
        memcpy(tag, d + o - 16, 16);
        int st = CRYPT_OK;
        if (!gcm(&pub, d + 13, d + 25, np, r + 13, tag, 0)) st = CRYPT_AUTH_PUBLIC;
        if (st == CRYPT_OK && o < L) {
            memcpy(tag, d + L - 16, 16);
            if (!gcm(&priv, d + o, d + o + 12, nv, r + 13 + np, tag, 0)) st = CRYPT_AUTH_PRIVATE;
            else if (nv < 1 || r[13 + np] != 0x01) st = CRYPT_BAD_VERSION;
        }
        status[i] = (uint8_t)st;
        if (st != CRYPT_OK) {
            memset(r, 0, size);
            continue;
        }
        memcpy(r, d, 13);
        wr32(r + 1, (uint32_t)(13 + np));
    }
    out_off[n] = w;
    return w;
}
