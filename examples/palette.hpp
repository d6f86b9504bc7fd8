// examples/palette.hpp -- the reference palette and a PPM writer for the examples.
#pragma once
#include <cstdint>
#include <cstdio>
#include <vector>

namespace examples {

// voxels.txt (ORT/voxels.txt): Stone, Grass, Dark Grass, Dirt; faces x_pos..z_neg,
// as olc::Pixel words (r in the low byte, alpha 0xFF).
inline std::vector<uint32_t> reference_palette()
{
    const uint32_t rgb[4][6] = {
        {0x44445D, 0x4E4E5B, 0x4E6155, 0x2B352F, 0x33333A, 0x232328},
        {0x5D2917, 0x3D260F, 0x4F2E14, 0x603718, 0x6D2E0D, 0x3F8527},
        {0x5D2917, 0x3D260F, 0x4F2E14, 0x603718, 0x6D2E0D, 0x317D1A},
        {0x5D2917, 0x3D260F, 0x4F2E14, 0x603718, 0x6D2E0D, 0x56220F}};
    std::vector<uint32_t> out;
    for (auto &v : rgb)
        for (uint32_t c : v) out.push_back(0xFF000000u | ((c & 0xFF) << 16) | (c & 0xFF00) | (c >> 16));
    return out;
}

inline bool write_ppm(const char *path, const uint32_t *rgba, int w, int h)
{
    FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%d %d\n255\n", w, h);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const uint32_t p = rgba[i];
        const unsigned char px[3] = {(unsigned char)(p & 0xFF), (unsigned char)((p >> 8) & 0xFF),
                                     (unsigned char)((p >> 16) & 0xFF)};
        std::fwrite(px, 1, 3, f);
    }
    return std::fclose(f) == 0;
}

}  // namespace examples
