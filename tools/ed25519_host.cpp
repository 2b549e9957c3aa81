/* Host build of agnes_amd/csrc/agnes_ed25519.h for unit-testing its arithmetic
 * without a GPU (development tool; the product is the HIP kernel).
 *   g++ -O2 -shared -fPIC -o /tmp/libedhost.so tools/ed25519_host.cpp */
#define __host__
#define __device__
#define __forceinline__ inline
#include "../agnes_amd/csrc/agnes_ed25519.h"
using namespace agnes::ed;
static int32_t g_tab[64 * BASE_ROW_WORDS];
static bool g_tab_ok = false;
extern "C" {
int ed_verify(const uint8_t* pub, const uint8_t* msg, uint32_t len, const uint8_t* sig) {
    if (!g_tab_ok) {
        for (int i = 0; i < 64; ++i) build_base_row(i, g_tab + i * BASE_ROW_WORDS);
        g_tab_ok = true;
    }
    return verify(pub, msg, len, sig, g_tab) ? 1 : 0;
}
void ed_sc_reduce(const uint8_t* in, uint8_t* out) { sc_reduce(out, in); }
void ed_fe_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
    fe x, y, z;
    fe_frombytes(x, a);
    fe_frombytes(y, b);
    fe_mul(z, x, y);
    fe_tobytes(out, z);
}
void ed_fe_invert(const uint8_t* a, uint8_t* out) {
    fe x, z;
    fe_frombytes(x, a);
    fe_invert(z, x);
    fe_tobytes(out, z);
}
void ed_fe_sub(const uint8_t* a, const uint8_t* b, uint8_t* out) {
    fe x, y, z;
    fe_frombytes(x, a);
    fe_frombytes(y, b);
    fe_sub(z, x, y);
    fe_tobytes(out, z);
}
int ed_decode_encode(const uint8_t* in, uint8_t* out) {
    ge p;
    if (!ge_frombytes(p, in)) return 0;
    ge_tobytes(out, p);
    return 1;
}
void ed_sha512(const uint8_t* m, uint32_t len, uint8_t* out) { sha512_short(out, m, len); }
}
