// Host-decoder robustness harness, built with AddressSanitizer + UBSan on the
// CPU (tools/fuzz/run.sh): mutates the JPEG files named on the command line
// (byte flips, truncation, marker-segment damage) and decodes every mutant
// with hjd_jpeg_decode_coefs.  Any out-of-bounds access aborts the run.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "hjd_host.h"
#include "hjd_internal.h"

int hjd_internal::set_error(int code, const char*, ...) { return code; }

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s ITERATIONS file.jpg...\n", argv[0]);
        return 2;
    }
    const int iters = atoi(argv[1]);
    std::mt19937 rng(12345);
    long ok = 0, bad = 0;
    for (int a = 2; a < argc; ++a) {
        FILE* fp = fopen(argv[a], "rb");
        if (!fp) return 2;
        std::vector<uint8_t> src;
        for (int c; (c = fgetc(fp)) != EOF;) src.push_back(static_cast<uint8_t>(c));
        fclose(fp);
        hjd_jpeg_info info;
        if (hjd_jpeg_parse(src.data(), src.size(), &info)) return 3;
        const int64_t cap = info.nblocks + 64;
        std::vector<int16_t> coefs(static_cast<size_t>(cap) * 64);
        for (int i = 0; i < iters; ++i) {
            std::vector<uint8_t> d = src;
            const int nflip = 1 + static_cast<int>(rng() % 8);
            for (int k = 0; k < nflip; ++k) {
                const size_t at = rng() % d.size();
                d[at] = (rng() % 3 == 0) ? 0xFF : static_cast<uint8_t>(rng());
            }
            if (rng() % 4 == 0) d.resize(rng() % d.size() + 1);
            // exact-size heap copy so ASan sees reads past the end
            uint8_t* buf = static_cast<uint8_t*>(malloc(d.size()));
            std::copy(d.begin(), d.end(), buf);
            hjd_jpeg_info mi;
            if (hjd_jpeg_parse(buf, d.size(), &mi) == HJD_OK && mi.nblocks <= cap &&
                hjd_jpeg_decode_coefs(buf, d.size(), &mi, coefs.data(), cap) == HJD_OK)
                ++ok;
            else
                ++bad;
            free(buf);
        }
    }
    printf("mutants decoded: %ld ok, %ld rejected\n", ok, bad);
    return 0;
}
