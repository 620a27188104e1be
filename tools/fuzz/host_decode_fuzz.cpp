// Host-decoder robustness harness, built with AddressSanitizer + UBSan on the
// CPU (tools/fuzz/run.sh): mutates the JPEG files named on the command line
// (byte flips, truncation, marker-segment damage) and decodes every mutant
// with hjd_jpeg_decode_coefs, and every mutant together with the previous one
// through the two-file interleaved decode (hjd_internal::jpeg_decode_coefs_two),
// whose per-file results must equal the one-file decodes; the one-file decode
// with the de-stuffed reader (default) must equal the byte-wise reader's
// (hjd_debug_host_reader(1)).  Any out-of-bounds access aborts the run.
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
    long ok = 0, bad = 0, pairs = 0, readers = 0;
    std::vector<uint8_t> prev;   // the previous mutant (any source file), its one-file result
    int prev_rc = 0;
    int64_t prev_cap = 0;
    std::vector<int16_t> prev_coefs;
    for (int a = 2; a < argc; ++a) {
        FILE* fp = fopen(argv[a], "rb");
        if (!fp) return 2;
        std::vector<uint8_t> src;
        for (int c; (c = fgetc(fp)) != EOF;) src.push_back(static_cast<uint8_t>(c));
        fclose(fp);
        hjd_jpeg_info info;
        if (hjd_jpeg_parse(src.data(), src.size(), &info)) return 3;
        const int64_t cap = info.nblocks + 64;
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
            // the one-file decode, into a fresh buffer
            hjd_jpeg_info mi;
            int rc = hjd_jpeg_parse(buf, d.size(), &mi);
            const int64_t nb = rc == HJD_OK ? mi.nblocks : 0;
            std::vector<int16_t> one(static_cast<size_t>(cap) * 64, 0);
            if (rc == HJD_OK) rc = hjd_jpeg_decode_coefs(buf, d.size(), &mi, one.data(), cap);
            if (rc == HJD_OK) ++ok; else ++bad;
            one.resize(rc == HJD_OK ? static_cast<size_t>(nb) * 64 : 0);
            if (nb > 0) {
                // the same file through the byte-wise reader
                std::vector<int16_t> bw(static_cast<size_t>(cap) * 64, 0);
                hjd_debug_host_reader(1);
                const int brc = hjd_jpeg_decode_coefs(buf, d.size(), &mi, bw.data(), cap);
                hjd_debug_host_reader(0);
                bw.resize(brc == HJD_OK ? static_cast<size_t>(nb) * 64 : 0);
                if (brc != rc || bw != one) {
                    fprintf(stderr, "de-stuffed and byte-wise readers differ (iteration %d of %s: rc %d vs %d)\n", i,
                            argv[a], rc, brc);
                    return 5;
                }
                ++readers;
            }
            if (!prev.empty()) {
                // (previous mutant, this one) through the two-file decode on one thread
                uint8_t* pbuf = static_cast<uint8_t*>(malloc(prev.size()));
                std::copy(prev.begin(), prev.end(), pbuf);
                std::vector<int16_t> c0(static_cast<size_t>(prev_cap) * 64, 0), c1(static_cast<size_t>(cap) * 64, 0);
                hjd_jpeg_info i0, i1;
                const uint8_t* dd[2] = {pbuf, buf};
                const size_t nn[2] = {prev.size(), d.size()};
                hjd_jpeg_info* ii[2] = {&i0, &i1};
                int16_t* const cc[2] = {c0.data(), c1.data()};
                const int64_t caps[2] = {prev_cap, cap};
                int prc[2];
                hjd_internal::jpeg_decode_coefs_two(dd, nn, ii, cc, caps, prc);
                c0.resize(prc[0] == HJD_OK ? prev_coefs.size() : 0);
                c1.resize(prc[1] == HJD_OK ? one.size() : 0);
                if ((prc[0] == HJD_OK) != (prev_rc == HJD_OK) || (prc[1] == HJD_OK) != (rc == HJD_OK) ||
                    c0 != prev_coefs || c1 != one) {
                    fprintf(stderr, "pair decode differs from the one-file decodes (iteration %d of %s)\n", i,
                            argv[a]);
                    return 4;
                }
                ++pairs;
                free(pbuf);
            }
            prev = d;
            prev_rc = rc;
            prev_cap = cap;
            prev_coefs.swap(one);
            free(buf);
        }
    }
    printf("mutants decoded: %ld ok, %ld rejected; %ld pairs equal to their one-file decodes; %ld equal under both "
           "readers\n", ok, bad, pairs, readers);
    return 0;
}
