// Host check of the chain kernel's slot-map composition (slot_compose,
// hjd_entropy.hpp; tests/test_idct_forms.py runs it): against the bytewise
// definition r[s] = f[s] == 0xFF ? 0xFF : g[f[s]] on random maps whose bytes
// are slots < 19 or 0xFF, byte 19 always 0xFF (the cmap row format).
#include <hip/hip_runtime.h>
#include "hjd_entropy.hpp"
#include <cstdio>
#include <cstdlib>
#include <random>
using namespace hjd::ent;
int main(int argc, char** argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 200000;
    std::mt19937 rng(7);
    long bad = 0;
    for (int it = 0; it < iters; ++it) {
        uint8_t fb[20], gb[20];
        const int pnone = rng() % 4;   // density of "no slot"
        for (int s = 0; s < 20; ++s) {
            fb[s] = s == 19 || (int)(rng() % 8) < pnone ? 0xFF : rng() % 19;
            gb[s] = s == 19 || (int)(rng() % 8) < pnone ? 0xFF : rng() % 19;
        }
        uint32_t f[5], g[5], r[5];
        for (int i = 0; i < 5; ++i) {
            f[i] = fb[4 * i] | fb[4 * i + 1] << 8 | fb[4 * i + 2] << 16 | (uint32_t)fb[4 * i + 3] << 24;
            g[i] = gb[4 * i] | gb[4 * i + 1] << 8 | gb[4 * i + 2] << 16 | (uint32_t)gb[4 * i + 3] << 24;
        }
        slot_compose(f, g, r);
        for (int s = 0; s < 20; ++s) {
            const uint32_t want = fb[s] == 0xFF ? 0xFF : gb[fb[s]];
            const uint32_t got = (r[s >> 2] >> (8 * (s & 3))) & 0xFF;
            bad += want != got;
        }
    }
    printf("slot maps %d mismatches %ld\n", iters, bad);
    return bad != 0;
}
