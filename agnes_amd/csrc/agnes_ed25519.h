/*
 * agnes_ed25519.h — Ed25519 signature verification, one vote per lane (SURVEY.md
 * §8(f) row 4; include/agnes.h agnes_wire_ingest).
 *
 * The reference verifies nothing: its README (README.md:8-14, 36-41) leaves
 * signature validation to the consumer and Validator holds the key
 * (validators.rs:4-8, 15-17).  The algorithm is RFC 8032 §5.1.7 in the
 * cofactorless form of OpenSSL 3.0 (ED25519_verify): reject S >= L, decode A
 * (§5.1.3), k = SHA-512(R || A || M) mod L, accept iff encode([S]B - [k]A) == R.
 *
 * gfx950 layout: everything is per-lane scalar integer code (no cross-lane
 * work: every vote is independent), so it is written for VALU throughput:
 *   field    GF(2^255 - 19) in radix 2^25.5, ten int32 limbs (26, 25, 26, ... bits);
 *            a product is 100 int32 x int32 -> int64 multiply-adds (v_mad_i64_i32)
 *            with the 19 x (wrap) and 2 x (two odd limbs) factors folded into
 *            the operands, then one carry chain; add / sub carry at once so
 *            every product operand stays below 2^26.x (no int64 overflow);
 *   points   extended twisted-Edwards (X : Y : Z : T), the unified a = -1
 *            addition (also the doubling), complete on the curve;
 *   scalars  [S]B from a fixed-base table (64 rows of j 16^i B, Niels form, built
 *            once per context: 64 mixed additions, no doubling) and [k](-A) by
 *            2-bit windows (two doublings + one addition per window), branch-free:
 *            the addend {O, -A, -2A, -3A} is selected per lane, so lanes with
 *            different bits do not diverge;
 *   hash     SHA-512 of the 104-byte R || A || M: one compression.
 * Host-compilable as plain C++ (tools/ed25519_host.cpp defines the HIP
 * qualifiers away) so the arithmetic can be unit-tested without a GPU.
 */
#pragma once
#include <stdint.h>

namespace agnes {
namespace ed {

#define AGNES_ED __host__ __device__ __forceinline__

struct fe {
    int32_t v[10];
};
struct ge {
    fe X, Y, Z, T;
};

/* limb widths: 26 bits at even i, 25 at odd i (bit offsets 0, 26, 51, 77, ...) */
AGNES_ED uint32_t fe_w(int i) { return (i & 1) ? 25u : 26u; }

/* carry a wide form into limbs: floor carries (arithmetic shifts) from limb 0 up,
 * the carry out of limb 9 (weight 2^255 = 19) back into limb 0, then limb 0 once
 * more.  |t| < 2^62 in; limbs in [0, 2^w) out except limb 1 (within a few units
 * of it). */
AGNES_ED void fe_carry(fe& h, int64_t t[10]) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int64_t c = t[i] >> fe_w(i);
        t[i + 1] += c;
        t[i] -= c * ((int64_t)1 << fe_w(i));
    }
    const int64_t c9 = t[9] >> 25;
    t[9] -= c9 * ((int64_t)1 << 25);
    t[0] += 19 * c9;
    const int64_t c0 = t[0] >> 26;
    t[0] -= c0 * ((int64_t)1 << 26);
    t[1] += c0;
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = (int32_t)t[i];
}

AGNES_ED void fe_set(fe& h, int32_t x) {
    h.v[0] = x;
#pragma unroll
    for (int i = 1; i < 10; ++i) h.v[i] = 0;
}
AGNES_ED void fe_add(fe& h, const fe& f, const fe& g) {
    int64_t t[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t[i] = (int64_t)f.v[i] + g.v[i];
    fe_carry(h, t);
}
AGNES_ED void fe_sub(fe& h, const fe& f, const fe& g) {
    int64_t t[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t[i] = (int64_t)f.v[i] - g.v[i];
    fe_carry(h, t);
}
AGNES_ED void fe_neg(fe& h, const fe& f) {
    int64_t t[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t[i] = -(int64_t)f.v[i];
    fe_carry(h, t);
}

/* h = f * g mod p: t[(i + j) mod 10] += f_i g_j x (2 if i, j both odd: the limb
 * offsets then sum to one bit more than the product limb's) x (19 if i + j >= 10:
 * 2^255 = 19 mod p).  Operands below 2^26.x: |2 f_i| < 2^27.1, |19 g_j| < 2^30.4,
 * ten products < 2^61. */
AGNES_ED void fe_mul(fe& h, const fe& f, const fe& g) {
    int32_t f2[10], g19[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
        g19[i] = 19 * g.v[i];
    }
    int64_t t[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
#pragma unroll
        for (int j = 0; j < 10; ++j) {
            const int32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
            const int32_t b = (i + j >= 10) ? g19[j] : g.v[j];
            t[(i + j) % 10] += (int64_t)a * b;
        }
    }
    fe_carry(h, t);
}
AGNES_ED void fe_sq(fe& h, const fe& f) { fe_mul(h, f, f); }
AGNES_ED void fe_sqn(fe& h, const fe& f, int n) {
    fe_sq(h, f);
    for (int i = 1; i < n; ++i) fe_sq(h, h);
}

/* z^(2^250 - 1) and z^11 (the shared prefix of inversion and the square root) */
AGNES_ED void fe_pow2_250_1(fe& t250, fe& z11, const fe& z) {
    fe z2, t, z9, z2_5, z2_10, z2_20, z2_50, z2_100;
    fe_sq(z2, z);            /* 2 */
    fe_sqn(t, z2, 2);        /* 8 */
    fe_mul(z9, t, z);        /* 9 */
    fe_mul(z11, z9, z2);     /* 11 */
    fe_sq(t, z11);           /* 22 */
    fe_mul(z2_5, t, z9);     /* 31 = 2^5 - 1 */
    fe_sqn(t, z2_5, 5);
    fe_mul(z2_10, t, z2_5);  /* 2^10 - 1 */
    fe_sqn(t, z2_10, 10);
    fe_mul(z2_20, t, z2_10); /* 2^20 - 1 */
    fe_sqn(t, z2_20, 20);
    fe_mul(t, t, z2_20);     /* 2^40 - 1 */
    fe_sqn(t, t, 10);
    fe_mul(z2_50, t, z2_10); /* 2^50 - 1 */
    fe_sqn(t, z2_50, 50);
    fe_mul(z2_100, t, z2_50); /* 2^100 - 1 */
    fe_sqn(t, z2_100, 100);
    fe_mul(t, t, z2_100);    /* 2^200 - 1 */
    fe_sqn(t, t, 50);
    fe_mul(t250, t, z2_50);  /* 2^250 - 1 */
}
/* z^(p - 2) = z^(2^255 - 21) */
AGNES_ED void fe_invert(fe& out, const fe& z) {
    fe t, z11;
    fe_pow2_250_1(t, z11, z);
    fe_sqn(t, t, 5); /* 2^255 - 32 */
    fe_mul(out, t, z11);
}
/* z^((p - 5) / 8) = z^(2^252 - 3) */
AGNES_ED void fe_pow22523(fe& out, const fe& z) {
    fe t, z11;
    fe_pow2_250_1(t, z11, z);
    fe_sqn(t, t, 2); /* 2^252 - 4 */
    fe_mul(out, t, z);
}

/* the canonical 32 bytes of h (value reduced mod p, little-endian) */
AGNES_ED void fe_tobytes(uint8_t s[32], const fe& h) {
    int64_t t[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t[i] = h.v[i];
    /* three carry passes: every limb in [0, 2^w), value in [0, 2^255) */
    for (int pass = 0; pass < 3; ++pass) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int64_t c = t[i] >> fe_w(i);
            t[i + 1] += c;
            t[i] -= c * ((int64_t)1 << fe_w(i));
        }
        const int64_t c9 = t[9] >> 25;
        t[9] -= c9 * ((int64_t)1 << 25);
        t[0] += 19 * c9;
    }
    /* value >= p  <=>  value + 19 >= 2^255: q = that carry; subtract q p */
    int64_t q = t[0] + 19;
#pragma unroll
    for (int i = 0; i < 10; ++i) q = (i == 0 ? q : t[i] + q) >> fe_w(i);
    t[0] += 19 * q;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int64_t c = t[i] >> fe_w(i);
        t[i + 1] += c;
        t[i] -= c * ((int64_t)1 << fe_w(i));
    }
    t[9] &= ((int64_t)1 << 25) - 1; /* drop q 2^255 */
    uint64_t w[4] = {0, 0, 0, 0};
    uint32_t off = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t x = (uint64_t)t[i];
        w[off >> 6] |= x << (off & 63u);
        if ((off & 63u) + fe_w(i) > 64u) w[(off >> 6) + 1] |= x >> (64u - (off & 63u));
        off += fe_w(i);
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) s[i] = (uint8_t)(w[i >> 3] >> (8 * (i & 7)));
}
/* the low 255 bits of 32 bytes (bit 255 ignored) */
AGNES_ED void fe_frombytes(fe& h, const uint8_t s[32]) {
    uint64_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t x = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) x |= (uint64_t)s[8 * k + b] << (8 * b);
        w[k] = x;
    }
    w[3] &= 0x7FFFFFFFFFFFFFFFull;
    uint32_t off = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint64_t x = w[off >> 6] >> (off & 63u);
        if ((off & 63u) + fe_w(i) > 64u) x |= w[(off >> 6) + 1] << (64u - (off & 63u));
        h.v[i] = (int32_t)(x & ((1ull << fe_w(i)) - 1ull));
        off += fe_w(i);
    }
}
AGNES_ED bool fe_iszero(const fe& f) {
    uint8_t s[32];
    fe_tobytes(s, f);
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) o |= s[i];
    return o == 0u;
}
AGNES_ED uint32_t fe_parity(const fe& f) {
    uint8_t s[32];
    fe_tobytes(s, f);
    return s[0] & 1u;
}
AGNES_ED void fe_select(fe& h, const fe& a, const fe& b, bool pick_b) {
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = pick_b ? b.v[i] : a.v[i];
}

/* constants in limbs (tools/ed25519_consts.py): d = -121665/121666, 2d, sqrt(-1) */
AGNES_ED void fe_d(fe& h) {
    const int32_t k[10] = {56195235, 13857412, 51736253, 6949390, 114729, 24766616, 60832955, 30306712, 48412415, 21499315};
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = k[i];
}
AGNES_ED void fe_2d(fe& h) {
    const int32_t k[10] = {45281625, 27714825, 36363642, 13898781, 229458, 15978800, 54557047, 27058993, 29715967, 9444199};
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = k[i];
}
AGNES_ED void fe_sqrtm1(fe& h) {
    const int32_t k[10] = {34513072, 25610706, 9377949, 3500415, 12389472, 33281959, 41962654, 31548777, 326685, 11406482};
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = k[i];
}

/* ---- points ---- */

AGNES_ED void ge_identity(ge& p) {
    fe_set(p.X, 0);
    fe_set(p.Y, 1);
    fe_set(p.Z, 1);
    fe_set(p.T, 0);
}
/* r = p + q (add-2008-hwcd-3, a = -1; k = 2d): complete, so also the doubling */
AGNES_ED void ge_add(ge& r, const ge& p, const ge& q, const fe& d2) {
    fe a, b, c, d, e, f, g, h, t;
    fe_sub(a, p.Y, p.X);
    fe_sub(t, q.Y, q.X);
    fe_mul(a, a, t);
    fe_add(b, p.Y, p.X);
    fe_add(t, q.Y, q.X);
    fe_mul(b, b, t);
    fe_mul(c, p.T, q.T);
    fe_mul(c, c, d2);
    fe_mul(d, p.Z, q.Z);
    fe_add(d, d, d);
    fe_sub(e, b, a);
    fe_sub(f, d, c);
    fe_add(g, d, c);
    fe_add(h, b, a);
    fe_mul(r.X, e, f);
    fe_mul(r.Y, g, h);
    fe_mul(r.T, e, h);
    fe_mul(r.Z, f, g);
}
/* r = 2p (dbl-2008-hwcd, a = -1): 4 squarings + 4 products */
AGNES_ED void ge_dbl(ge& r, const ge& p) {
    fe a, b, c, e, f, g, h, t;
    fe_sq(a, p.X);
    fe_sq(b, p.Y);
    fe_sq(c, p.Z);
    fe_add(c, c, c);
    fe_add(h, a, b);
    fe_add(t, p.X, p.Y);
    fe_sq(t, t);
    fe_sub(e, h, t);
    fe_sub(g, a, b);
    fe_add(f, c, g);
    fe_mul(r.X, e, f);
    fe_mul(r.Y, g, h);
    fe_mul(r.T, e, h);
    fe_mul(r.Z, f, g);
}
/* RFC 8032 §5.1.3: false when s encodes no point (y >= p, no square root, or x = 0
 * with the sign bit set) */
AGNES_ED bool ge_frombytes(ge& p, const uint8_t s[32]) {
    /* y < p: the low 255 bits are not in [p, 2^255) */
    {
        bool ge_p = (s[31] & 0x7F) == 0x7F && s[0] >= 0xED;
#pragma unroll
        for (int i = 1; i < 31; ++i) ge_p = ge_p && s[i] == 0xFF;
        if (ge_p) return false;
    }
    const uint32_t sign = s[31] >> 7;
    fe y, u, v, v3, x, t, d;
    fe_frombytes(y, s);
    fe_d(d);
    fe_sq(u, y);
    fe_mul(v, u, d);
    fe one;
    fe_set(one, 1);
    fe_sub(u, u, one); /* y^2 - 1 */
    fe_add(v, v, one); /* d y^2 + 1 */
    fe_sq(v3, v);
    fe_mul(v3, v3, v); /* v^3 */
    fe_sq(x, v3);
    fe_mul(x, x, v);
    fe_mul(x, x, u); /* u v^7 */
    fe_pow22523(x, x);
    fe_mul(x, x, v3);
    fe_mul(x, x, u); /* u v^3 (u v^7)^((p-5)/8) */
    fe_sq(t, x);
    fe_mul(t, t, v); /* v x^2 */
    fe chk;
    fe_sub(chk, t, u);
    if (!fe_iszero(chk)) {
        fe_add(chk, t, u);
        if (!fe_iszero(chk)) return false;
        fe m1;
        fe_sqrtm1(m1);
        fe_mul(x, x, m1);
    }
    const uint32_t par = fe_parity(x);
    if (fe_iszero(x) && sign) return false;
    if (par != sign) fe_neg(x, x);
    p.X = x;
    p.Y = y;
    fe_set(p.Z, 1);
    fe_mul(p.T, x, y);
    return true;
}
AGNES_ED void ge_tobytes(uint8_t s[32], const ge& p) {
    fe zi, x, y;
    fe_invert(zi, p.Z);
    fe_mul(x, p.X, zi);
    fe_mul(y, p.Y, zi);
    fe_tobytes(s, y);
    s[31] ^= (uint8_t)(fe_parity(x) << 7);
}

/* ---- scalars mod L = 2^252 + 27742317777372353535851937790883648493 ---- */

/* r = x mod L for a 64-byte little-endian x: the bytes above 32 folded down with
 * 2^256 = 16 x 2^252 = -16 (L - 2^252) (mod L), then the bits above 252 */
AGNES_ED void sc_reduce(uint8_t r[32], const uint8_t in[64]) {
    const int64_t Lb[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                            0xa2, 0xde, 0xf9, 0xde, 0x14, 0,    0,    0,    0,    0,    0,
                            0,    0,    0,    0,    0,    0,    0,    0,    0,    0x10};
    int64_t x[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) x[i] = in[i];
    for (int i = 63; i >= 32; --i) {
        int64_t carry = 0;
        int j;
        for (j = i - 32; j < i - 12; ++j) {
            x[j] += carry - 16 * x[i] * Lb[j - (i - 32)];
            carry = (x[j] + 128) >> 8;
            x[j] -= carry * 256;
        }
        x[j] += carry;
        x[i] = 0;
    }
    int64_t carry = 0;
    for (int j = 0; j < 32; ++j) {
        x[j] += carry - (x[31] >> 4) * Lb[j];
        carry = x[j] >> 8;
        x[j] &= 255;
    }
    for (int j = 0; j < 32; ++j) x[j] -= carry * Lb[j];
    for (int i = 0; i < 32; ++i) {
        x[i + 1] += x[i] >> 8;
        r[i] = (uint8_t)(x[i] & 255);
    }
}
/* s < L (little-endian 32 bytes) */
AGNES_ED bool sc_canonical(const uint8_t s[32]) {
    const uint8_t Lb[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                            0xa2, 0xde, 0xf9, 0xde, 0x14, 0,    0,    0,    0,    0,    0,
                            0,    0,    0,    0,    0,    0,    0,    0,    0,    0x10};
    for (int i = 31; i >= 0; --i) {
        if (s[i] < Lb[i]) return true;
        if (s[i] > Lb[i]) return false;
    }
    return false; /* s == L */
}

/* ---- SHA-512 (FIPS 180-4), one message of at most 111 bytes ---- */

AGNES_ED uint64_t rotr64(uint64_t x, uint32_t n) { return (x >> n) | (x << (64u - n)); }

AGNES_ED void sha512_short(uint8_t out[64], const uint8_t* msg, uint32_t len) {
    const uint64_t K[80] = {
        0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
        0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
        0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
        0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
        0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
        0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
        0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
        0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
        0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
        0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
        0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
        0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
        0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
        0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
        0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
        0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
        0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
        0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
        0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
        0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
    uint64_t W[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = 0;
    for (uint32_t i = 0; i < len; ++i) W[i >> 3] |= (uint64_t)msg[i] << (56u - 8u * (i & 7u));
    W[len >> 3] |= 0x80ull << (56u - 8u * (len & 7u));
    W[15] = 8ull * len;
    uint64_t a = 0x6a09e667f3bcc908ull, b = 0xbb67ae8584caa73bull, c = 0x3c6ef372fe94f82bull,
             d = 0xa54ff53a5f1d36f1ull, e = 0x510e527fade682d1ull, f = 0x9b05688c2b3e6c1full,
             g = 0x1f83d9abfb41bd6bull, h = 0x5be0cd19137e2179ull;
    const uint64_t H0[8] = {a, b, c, d, e, f, g, h};
    for (int t = 0; t < 80; ++t) {
        uint64_t w;
        if (t < 16) {
            w = W[t];
        } else {
            const uint64_t w15 = W[(t + 1) & 15], w2 = W[(t + 14) & 15];
            const uint64_t s0 = rotr64(w15, 1) ^ rotr64(w15, 8) ^ (w15 >> 7);
            const uint64_t s1 = rotr64(w2, 19) ^ rotr64(w2, 61) ^ (w2 >> 6);
            w = W[t & 15] + s0 + W[(t + 9) & 15] + s1;
            W[t & 15] = w;
        }
        const uint64_t S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
        const uint64_t ch = (e & f) ^ (~e & g);
        const uint64_t t1 = h + S1 + ch + K[t] + w;
        const uint64_t S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
        const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
        const uint64_t t2 = S0 + mj;
        h = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    const uint64_t Hs[8] = {a + H0[0], b + H0[1], c + H0[2], d + H0[3], e + H0[4], f + H0[5], g + H0[6], h + H0[7]};
#pragma unroll
    for (int i = 0; i < 64; ++i) out[i] = (uint8_t)(Hs[i >> 3] >> (56u - 8u * (i & 7u)));
}

/* ---- verification ---- */

/* the base point B: y = 4/5, x even (RFC 8032 §5.1); limbs from tools/ed25519_consts.py */
AGNES_ED void ge_base(ge& b) {
    const int32_t bx[10] = {52811034, 25909283, 16144682, 17082669, 27570973, 30858332, 40966398, 8378388, 20764389, 8758491};
    const int32_t by[10] = {40265304, 26843545, 13421772, 20132659, 26843545, 6710886, 53687091, 13421772, 40265318, 26843545};
    const int32_t bt[10] = {28827043, 27438313, 39759291, 244362, 8635006, 11264893, 19351346, 13413597, 16611511, 27139452};
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        b.X.v[i] = bx[i];
        b.Y.v[i] = by[i];
        b.T.v[i] = bt[i];
    }
    fe_set(b.Z, 1);
}

/* a point in affine "Niels" form: y + x, y - x, 2 d x y (identity: 1, 1, 0) */
struct ge_niels {
    fe ypx, ymx, xy2d;
};
/* r = p + q, q affine (madd-2008-hwcd-3, a = -1): 7 products */
AGNES_ED void ge_madd(ge& r, const ge& p, const ge_niels& q) {
    fe a, b, c, d, e, f, g, h;
    fe_sub(a, p.Y, p.X);
    fe_mul(a, a, q.ymx);
    fe_add(b, p.Y, p.X);
    fe_mul(b, b, q.ypx);
    fe_mul(c, p.T, q.xy2d);
    fe_add(d, p.Z, p.Z);
    fe_sub(e, b, a);
    fe_sub(f, d, c);
    fe_add(g, d, c);
    fe_add(h, b, a);
    fe_mul(r.X, e, f);
    fe_mul(r.Y, g, h);
    fe_mul(r.T, e, h);
    fe_mul(r.Z, f, g);
}

/* the fixed-base table: row i (0..63) holds j 16^i B for j = 0..15 in Niels form,
 * 16 x 3 x 10 int32 (agnes_wire.hip builds it once per context, one thread a row) */
constexpr int BASE_ROW_WORDS = 16 * 3 * 10;
AGNES_ED void build_base_row(int i, int32_t* out) {
    ge bi, acc;
    ge_base(bi);
    for (int k = 0; k < 4 * i; ++k) ge_dbl(bi, bi);
    ge_identity(acc);
    fe d2;
    fe_2d(d2);
    for (int j = 0; j < 16; ++j) {
        fe zi, x, y, s, dd, m;
        fe_invert(zi, acc.Z);
        fe_mul(x, acc.X, zi);
        fe_mul(y, acc.Y, zi);
        fe_add(s, y, x);
        fe_sub(dd, y, x);
        fe_mul(m, x, y);
        fe_mul(m, m, d2);
        for (int l = 0; l < 10; ++l) {
            out[(j * 3 + 0) * 10 + l] = s.v[l];
            out[(j * 3 + 1) * 10 + l] = dd.v[l];
            out[(j * 3 + 2) * 10 + l] = m.v[l];
        }
        ge_add(acc, acc, bi, d2);
    }
}

/* RFC 8032 §5.1.7, cofactorless (OpenSSL 3.0 ED25519_verify): sig = R || S over
 * msg (len <= 47: R || A || msg fits one SHA-512 block) with public key pub.
 * [S]B = sum over the 64 nibbles s_i of S of the table entry s_i 16^i B (no
 * doubling); [k](-A) by 2-bit windows from the top (two doublings and one
 * addition of {O, -A, -2A, -3A} per window, chosen per lane by selects). */
AGNES_ED bool verify(const uint8_t pub[32], const uint8_t* msg, uint32_t len, const uint8_t sig[64],
                     const int32_t* base_table) {
    if (!sc_canonical(sig + 32)) return false;
    ge A;
    if (!ge_frombytes(A, pub)) return false;
    uint8_t hin[111], h[64], k[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        hin[i] = sig[i];
        hin[32 + i] = pub[i];
    }
    for (uint32_t i = 0; i < len; ++i) hin[64 + i] = msg[i];
    sha512_short(h, hin, 64u + len);
    sc_reduce(k, h);
    fe d2;
    fe_2d(d2);
    /* [S]B */
    const uint8_t* S = sig + 32;
    ge P;
    ge_identity(P);
    for (int i = 0; i < 64; ++i) {
        const uint32_t nib = (S[i >> 1] >> (4 * (i & 1))) & 15u;
        const int32_t* e = base_table + (i * 16 + (int)nib) * 30;
        ge_niels q;
#pragma unroll
        for (int l = 0; l < 10; ++l) {
            q.ypx.v[l] = e[l];
            q.ymx.v[l] = e[10 + l];
            q.xy2d.v[l] = e[20 + l];
        }
        ge_madd(P, P, q);
    }
    /* [k](-A) */
    ge n1, n2, n3;
    fe_neg(n1.X, A.X);
    n1.Y = A.Y;
    n1.Z = A.Z;
    fe_neg(n1.T, A.T);
    ge_dbl(n2, n1);
    ge_add(n3, n2, n1, d2);
    ge Q;
    ge_identity(Q);
    for (int i = 252; i >= 0; i -= 2) { /* windows (i + 1, i); k < 2^253: bits 253.. are zero */
        ge_dbl(Q, Q);
        ge_dbl(Q, Q);
        const uint32_t dgt = (k[i >> 3] >> (i & 7)) & 3u; /* (i even: the pair never straddles a byte) */
        ge T;
        ge_identity(T);
        fe_select(T.X, T.X, n1.X, dgt == 1u);
        fe_select(T.Y, T.Y, n1.Y, dgt == 1u);
        fe_select(T.Z, T.Z, n1.Z, dgt == 1u);
        fe_select(T.T, T.T, n1.T, dgt == 1u);
        fe_select(T.X, T.X, n2.X, dgt == 2u);
        fe_select(T.Y, T.Y, n2.Y, dgt == 2u);
        fe_select(T.Z, T.Z, n2.Z, dgt == 2u);
        fe_select(T.T, T.T, n2.T, dgt == 2u);
        fe_select(T.X, T.X, n3.X, dgt == 3u);
        fe_select(T.Y, T.Y, n3.Y, dgt == 3u);
        fe_select(T.Z, T.Z, n3.Z, dgt == 3u);
        fe_select(T.T, T.T, n3.T, dgt == 3u);
        ge_add(Q, Q, T, d2);
    }
    ge_add(Q, Q, P, d2);
    uint8_t rc[32];
    ge_tobytes(rc, Q);
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) diff |= (uint32_t)(rc[i] ^ sig[i]);
    return diff == 0u;
}

#undef AGNES_ED
} // namespace ed
} // namespace agnes
