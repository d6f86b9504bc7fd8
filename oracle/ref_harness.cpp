// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
// Drives the reference's own sources, compiled where they lie under
// /root/reference (no copies, no stand-ins): och::simplex_n from
// ORT/och_noise.h:18-367 and och::z_encode_16_noninline from
// ORT/och_z_order.cpp.  Built by oracle/Makefile into oracle/_ref/ (git-ignored).
// Protocol: argv[1] = noise2 | noise3 | zenc, argv[2] = frequency (noise);
// binary little-endian records on stdin -> results on stdout:
//   noise2: f32 x, f32 y      -> f32
//   noise3: f32 x, f32 y, f32 z -> f32
//   zenc:   u16 x, u16 y, u16 z -> u64
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "och_noise.h"
#include "och_z_order.h"

int main(int argc, char** argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: ref_harness noise2|noise3|zenc [freq]\n"); return 2; }
    const float freq = argc > 2 ? std::strtof(argv[2], nullptr) : 1.0F;
    och::simplex_n noise(freq);
    if (!std::strcmp(argv[1], "noise2")) {
        float in[2];
        while (std::fread(in, sizeof in, 1, stdin) == 1) { float r = noise(in[0], in[1]); std::fwrite(&r, 4, 1, stdout); }
    } else if (!std::strcmp(argv[1], "noise3")) {
        float in[3];
        while (std::fread(in, sizeof in, 1, stdin) == 1) { float r = noise(in[0], in[1], in[2]); std::fwrite(&r, 4, 1, stdout); }
    } else if (!std::strcmp(argv[1], "zenc")) {
        uint16_t in[3];
        while (std::fread(in, sizeof in, 1, stdin) == 1) { uint64_t r = och::z_encode_16_noninline(in[0], in[1], in[2]); std::fwrite(&r, 8, 1, stdout); }
    } else {
        return 2;
    }
    return 0;
}
