// checksum.h — vsr.checksum (src/vsr/checksum.zig:50-74) on the host: the Aegis-128L MAC with an
// all-zero key and nonce over the message as associated data, 128-bit tag.  TigerBeetle stores it in
// every header (checksum of header bytes [16, 128), checksum_body of the body: src/vsr.zig:405-437)
// and the AOF iterator verifies both (src/aof.zig:214-218).  Pinned by the reference's own vectors
// (checksum.zig:83-101, the "checksum stability" hash at :135-184) in tests/test_checksum.py.
//
// Aegis-128L (draft-irtf-cfrg-aegis-aead): eight 16-byte AES blocks S0..S7;
//   Update(M0, M1): S'i = AESRound(S(i-1), Si) with M0 folded into S0 and M1 into S4;
//   init: S = {k^n, C1, C0, C1, k^n, k^C0, k^C1, k^C0}, then 10 x Update(n, k);
//   absorb: Update(ad[0:16], ad[16:32]) per 32-byte block (the last one zero-padded);
//   finalize: t = S2 ^ (LE64(ad bits) || LE64(0)), 7 x Update(t, t), tag = S0^S1^S2^S3^S4^S5^S6.
// Host code only (plain C++, byte-wise AES round); not on the commit path.
#pragma once

#include <cstdint>
#include <cstring>

namespace tbck {

struct Block {
    uint8_t b[16];
};

static inline uint8_t xt(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

static inline uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = xt(a);
        b >>= 1;
    }
    return p;
}

// The AES S-box: multiplicative inverse in GF(2^8), then the affine map (FIPS-197 §5.1.1).
struct SBox {
    uint8_t s[256];
    SBox() {
        for (int x = 0; x < 256; x++) {
            uint8_t inv = 0;
            if (x) {  // x^254
                uint8_t r = 1, base = (uint8_t)x;
                for (int e = 254; e; e >>= 1) {
                    if (e & 1) r = gmul(r, base);
                    base = gmul(base, base);
                }
                inv = r;
            }
            uint8_t y = inv;
            for (int k = 1; k <= 4; k++) y ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
            s[x] = (uint8_t)(y ^ 0x63);
        }
    }
};

static inline const uint8_t* sbox() {
    static const SBox S;
    return S.s;
}

// AESRound(in, rk) = MixColumns(ShiftRows(SubBytes(in))) ^ rk; column-major state (byte 4c + r).
static inline Block aes_round(const Block& in, const Block& rk) {
    const uint8_t* S = sbox();
    Block o;
    for (int c = 0; c < 4; c++) {
        const uint8_t a0 = S[in.b[4 * c + 0]];
        const uint8_t a1 = S[in.b[4 * ((c + 1) & 3) + 1]];
        const uint8_t a2 = S[in.b[4 * ((c + 2) & 3) + 2]];
        const uint8_t a3 = S[in.b[4 * ((c + 3) & 3) + 3]];
        const uint8_t t = a0 ^ a1 ^ a2 ^ a3;
        o.b[4 * c + 0] = (uint8_t)(a0 ^ t ^ xt(a0 ^ a1) ^ rk.b[4 * c + 0]);
        o.b[4 * c + 1] = (uint8_t)(a1 ^ t ^ xt(a1 ^ a2) ^ rk.b[4 * c + 1]);
        o.b[4 * c + 2] = (uint8_t)(a2 ^ t ^ xt(a2 ^ a3) ^ rk.b[4 * c + 2]);
        o.b[4 * c + 3] = (uint8_t)(a3 ^ t ^ xt(a3 ^ a0) ^ rk.b[4 * c + 3]);
    }
    return o;
}

static inline Block bxor(const Block& a, const Block& b) {
    Block o;
    for (int i = 0; i < 16; i++) o.b[i] = a.b[i] ^ b.b[i];
    return o;
}

struct Aegis128L {
    Block s[8];

    void update(const Block& m0, const Block& m1) {
        const Block t7 = s[7];
        Block n[8];
        n[0] = aes_round(t7, bxor(s[0], m0));
        for (int i = 1; i < 8; i++) n[i] = aes_round(s[i - 1], i == 4 ? bxor(s[4], m1) : s[i]);
        for (int i = 0; i < 8; i++) s[i] = n[i];
    }

    void init_zero() {  // key = nonce = 0
        static const uint8_t c0[16] = {0x00, 0x01, 0x01, 0x02, 0x03, 0x05, 0x08, 0x0d,
                                       0x15, 0x22, 0x37, 0x59, 0x90, 0xe9, 0x79, 0x62};
        static const uint8_t c1[16] = {0xdb, 0x3d, 0x18, 0x55, 0x6d, 0xc2, 0x2f, 0xf1,
                                       0x20, 0x11, 0x31, 0x42, 0x73, 0xb5, 0x28, 0xdd};
        Block z{}, C0, C1;
        memcpy(C0.b, c0, 16);
        memcpy(C1.b, c1, 16);
        s[0] = z;
        s[1] = C1;
        s[2] = C0;
        s[3] = C1;
        s[4] = z;
        s[5] = C0;
        s[6] = C1;
        s[7] = C0;
        for (int i = 0; i < 10; i++) update(z, z);
    }
};

// checksum(source) -> 16 tag bytes (the u128 in little-endian memory order).
static inline void checksum(const uint8_t* p, uint64_t len, uint8_t out[16]) {
    Aegis128L st;
    st.init_zero();
    uint64_t i = 0;
    for (; i + 32 <= len; i += 32) {
        Block m0, m1;
        memcpy(m0.b, p + i, 16);
        memcpy(m1.b, p + i + 16, 16);
        st.update(m0, m1);
    }
    if (i < len) {
        uint8_t pad[32] = {0};
        memcpy(pad, p + i, len - i);
        Block m0, m1;
        memcpy(m0.b, pad, 16);
        memcpy(m1.b, pad + 16, 16);
        st.update(m0, m1);
    }
    Block t{};
    const uint64_t bits = len * 8;
    for (int k = 0; k < 8; k++) t.b[k] = (uint8_t)(bits >> (8 * k));
    t = bxor(st.s[2], t);
    for (int k = 0; k < 7; k++) st.update(t, t);
    Block tag = st.s[0];
    for (int k = 1; k < 7; k++) tag = bxor(tag, st.s[k]);
    memcpy(out, tag.b, 16);
}

}  // namespace tbck
