// Host check of the pixel kernel's IDCT forms (tests/test_idct_forms.py): the
// packed row pass with dot2 accumulation chains (idct8_row_pk) and the
// high-half column pass (idct8_col_hi, stored with ds_write_b16_d16_hi) against
// the plain restatement idct8<false>/idct8<true, L> (itself pinned to the
// oracle and the reference's known answers), on random blocks of the
// reference's legal domain (forward DCT of bounded samples, quantised with
// q = 1..255, clamping in play) and the clamp-edge known answers.  The same
// __host__ __device__ code the kernels run; the device-only instructions
// (v_dot2_i32_i16, v_mul_i32_i24) compute the same integers on this domain.
#include "hjd_device.hpp"
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
using namespace hjd;
template <int L>
static int check_block(const int (&blk)[64])
{
    int ref[64], got[64];
    for (int i = 0; i < 64; ++i) ref[i] = got[i] = blk[i];
    // reference: rows then columns (unscaled)
    for (int r = 0; r < 8; ++r) { int v[8]; for (int c = 0; c < 8; ++c) v[c] = ref[r * 8 + c]; idct8<false>(v); for (int c = 0; c < 8; ++c) ref[r * 8 + c] = v[c]; }
    for (int c = 0; c < 8; ++c) { int v[8]; for (int r = 0; r < 8; ++r) v[r] = ref[r * 8 + c]; idct8<true, L>(v); for (int r = 0; r < 8; ++r) ref[r * 8 + c] = v[r]; }
    // new: packed row pass, high-half column pass
    for (int r = 0; r < 8; ++r) {
        const int* b = got + r * 8;
        RowPk p;
        p.p04 = s16x2{(short)b[0], (short)b[4]}; p.p17 = s16x2{(short)b[1], (short)b[7]};
        p.p35 = s16x2{(short)b[3], (short)b[5]}; p.p26 = s16x2{(short)b[2], (short)b[6]};
        int v[8]; idct8_row_pk(p, v); for (int c = 0; c < 8; ++c) got[r * 8 + c] = v[c];
    }
    for (int c = 0; c < 8; ++c) { int v[8]; for (int r = 0; r < 8; ++r) v[r] = got[r * 8 + c]; idct8_col_hi<L>(v); for (int r = 0; r < 8; ++r) got[r * 8 + c] = (short)((unsigned)v[r] >> 16); }
    int bad = 0;
    for (int i = 0; i < 64; ++i) bad += ref[i] != got[i];
    return bad;
}
int main(int argc, char** argv)
{
    std::mt19937 rng(1);
    long nb = 0, bad = 0, clamped = 0;
    double C[8][8];
    for (int u = 0; u < 8; ++u) for (int x = 0; x < 8; ++x) C[u][x] = (u ? 1.0 : std::sqrt(0.5)) * std::cos((2 * x + 1) * u * M_PI / 16) / 2;
    const int iters = argc > 1 ? atoi(argv[1]) : 400000;
    for (int it = 0; it < iters; ++it) {
        double px[8][8];
        const int amp = 50 + rng() % 400, base = (int)(rng() % 600) - 300;
        const int mode = rng() % 3;
        for (int y = 0; y < 8; ++y) for (int x = 0; x < 8; ++x)
            px[y][x] = mode == 0 ? base + ((int)(rng() % (2 * amp + 1)) - amp)
                     : mode == 1 ? ((x + y) & 1 ? 255 : -256) * (amp > 200 ? 1 : -1)
                     : base + (x * 37 + y * 11) % amp - amp / 2;
        const int q = 1 + (rng() % 4 == 0 ? rng() % 255 : rng() % 8);
        int blk[64];
        for (int u = 0; u < 8; ++u) for (int v = 0; v < 8; ++v) {
            double s = 0;
            for (int y = 0; y < 8; ++y) for (int x = 0; x < 8; ++x) s += C[u][y] * C[v][x] * px[y][x];
            int c = (int)std::lround(s / q) * q;
            if (c > 32767) c = 32767; if (c < -32768) c = -32768;
            blk[u * 8 + v] = c;
        }
        // legal domain: raw column outputs in [-512, 511]
        int tmp[64]; for (int i = 0; i < 64; ++i) tmp[i] = blk[i];
        for (int r = 0; r < 8; ++r) { int v[8]; for (int c = 0; c < 8; ++c) v[c] = tmp[r * 8 + c]; idct8<false>(v); for (int c = 0; c < 8; ++c) tmp[r * 8 + c] = v[c]; }
        bool legal = true;
        // (approximate check by the unclamped double IDCT)
        for (int y = 0; y < 8 && legal; ++y) for (int x = 0; x < 8; ++x) {
            double s = 0; for (int u = 0; u < 8; ++u) for (int v = 0; v < 8; ++v) s += C[u][y] * C[v][x] * blk[u * 8 + v];
            if (s < -500 || s > 500) { legal = false; break; }
            if (s < -256 || s > 255) ++clamped;
        }
        if (!legal) continue;
        ++nb;
        bad += check_block<0>(blk) + check_block<128>(blk);
    }
    // known answers: DC-only +-2100, 2016, and the {b0=1000,b1=-900,b8=700} block
    int kb[4][64] = {};
    kb[0][0] = 2100; kb[1][0] = -2100; kb[2][0] = 2016; kb[3][0] = 1000; kb[3][1] = -900; kb[3][8] = 700;
    for (auto& b : kb) bad += check_block<0>(b) + check_block<128>(b);
    printf("blocks %ld (clamped samples %ld) mismatches %ld\n", nb, clamped, bad);
    return bad != 0;
}
