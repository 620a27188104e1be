// Robustness harness for the GPU entropy decoder's algorithm, run on the CPU
// with AddressSanitizer + UBSan (tools/fuzz/run_entropy.sh): mutates JPEG
// files (byte flips, 0xFF runs, truncation) and decodes every sequential
// mutant (one scan or several) with hjd_debug_entropy_emulate -- the host build of the same
// destuff, sync/link/repair (round-based and speculative) and write code the
// gfx950 kernels run, over
// buffers laid out as on the device (each frame's bit string followed by its
// kDataPad read-ahead bytes; the staging block is sized to the file).  The
// output buffer is an exact-size heap block, so a write past the frame's
// blocks, or a read past the padded bit string, aborts the run.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "hjd_host.h"

extern "C" int hjd_debug_entropy_emulate(const uint8_t* data, size_t size, int sub_bits, int16_t* coefs,
                                         int64_t capacity_blocks, int32_t* status);

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s ITERATIONS file.jpg...\n", argv[0]);
        return 2;
    }
    const int iters = atoi(argv[1]);
    std::mt19937 rng(4242);
    const int subs[] = {32, 33, 64, 100, 256, 1024, 2048, 4096};
    long ok = 0, corrupt = 0, rejected = 0;
    for (int a = 2; a < argc; ++a) {
        FILE* fp = fopen(argv[a], "rb");
        if (!fp) return 2;
        std::vector<uint8_t> src;
        for (int c; (c = fgetc(fp)) != EOF;) src.push_back(static_cast<uint8_t>(c));
        fclose(fp);
        hjd_jpeg_info info;
        if (hjd_jpeg_parse(src.data(), src.size(), &info) || info.process == 2) continue;
        for (int i = 0; i < iters; ++i) {
            std::vector<uint8_t> d = src;
            const int nflip = 1 + static_cast<int>(rng() % 8);
            for (int k = 0; k < nflip; ++k) {
                const size_t at = rng() % d.size();
                const int kind = static_cast<int>(rng() % 4);
                if (kind == 0) d[at] = 0xFF;
                else if (kind == 1 && at + 1 < d.size()) { d[at] = 0xFF; d[at + 1] = static_cast<uint8_t>(0xD0 + rng() % 8); }
                else d[at] = static_cast<uint8_t>(rng());
            }
            if (rng() % 4 == 0) d.resize(rng() % d.size() + 1);
            uint8_t* buf = static_cast<uint8_t*>(malloc(d.size()));
            std::copy(d.begin(), d.end(), buf);
            hjd_jpeg_info mi;
            if (hjd_jpeg_parse(buf, d.size(), &mi) != HJD_OK || mi.process == 2 || mi.nblocks <= 0 ||
                mi.nblocks > 1 << 20) {
                ++rejected;
                free(buf);
                continue;
            }
            // exact-size output: the frame's blocks and nothing more
            int16_t* coefs = static_cast<int16_t*>(malloc(static_cast<size_t>(mi.nblocks) * 128));
            int32_t status = 0;
            // every other mutant through the speculative sync (latency decoders),
            // with a random lead-in of its spec runs
            setenv("HJD_SYNC_SPEC", i % 2 ? "1" : "0", 1);
            const char* leads[] = {"0", "100", "512", "1024"};
            setenv("HJD_SPEC_LEAD", leads[rng() % 4], 1);
            const int rc = hjd_debug_entropy_emulate(buf, d.size(), subs[rng() % 8], coefs, mi.nblocks, &status);
            if (rc == HJD_OK) ++ok;
            else ++corrupt;
            free(coefs);
            free(buf);
        }
    }
    printf("entropy mutants: %ld decoded, %ld flagged corrupt, %ld rejected by the parser\n", ok, corrupt, rejected);
    return 0;
}
