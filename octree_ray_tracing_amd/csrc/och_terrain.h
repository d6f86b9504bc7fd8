// och_terrain.h -- the demo terrain's voxel function, host + device.
//
// Restates, in IEEE float with no contraction (build with -ffp-contract=off):
//   och::simplex_n 2-D / 3-D           ORT/och_noise.h:73-179, :181-366
//   get_terrain_heigth                 ORT/test_och_h_octree.cpp:561-569
//   splatter_noise tunnels (-0.5, 1/16) ORT/test_och_h_octree.cpp:745-765, :770
//   initialize_h_octree voxel values   ORT/test_och_h_octree.cpp:767-787
// so that the voxel content is a pure function of (x, y, z): the builder can
// evaluate it in any order, on any number of threads or on the GPU.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define OCH_HD __host__ __device__ __forceinline__
#else
#define OCH_HD inline
#endif

namespace och_terrain {

struct Tables {
    uint8_t perm[256];
    int8_t grad[12][3];
};

// Ken Perlin's reference permutation as used by simplex_n (ORT/och_noise.h:20-53).
#define OCH_PERM_TABLE                                                                              \
    {151, 160, 137, 91, 90, 15, 131, 13, 201, 95, 96, 53, 194, 233, 7, 225, 140, 36, 103, 30,       \
     69, 142, 8, 99, 37, 240, 21, 10, 23, 190, 6, 148, 247, 120, 234, 75, 0, 26, 197, 62, 94, 252,   \
     219, 203, 117, 35, 11, 32, 57, 177, 33, 88, 237, 149, 56, 87, 174, 20, 125, 136, 171, 168, 68,  \
     175, 74, 165, 71, 134, 139, 48, 27, 166, 77, 146, 158, 231, 83, 111, 229, 122, 60, 211, 133,    \
     230, 220, 105, 92, 41, 55, 46, 245, 40, 244, 102, 143, 54, 65, 25, 63, 161, 1, 216, 80, 73, 209, \
     76, 132, 187, 208, 89, 18, 169, 200, 196, 135, 130, 116, 188, 159, 86, 164, 100, 109, 198, 173,  \
     186, 3, 64, 52, 217, 226, 250, 124, 123, 5, 202, 38, 147, 118, 126, 255, 82, 85, 212, 207, 206,  \
     59, 227, 47, 16, 58, 17, 182, 189, 28, 42, 223, 183, 170, 213, 119, 248, 152, 2, 44, 154, 163,   \
     70, 221, 153, 101, 155, 167, 43, 172, 9, 129, 22, 39, 253, 19, 98, 108, 110, 79, 113, 224, 232,  \
     178, 185, 112, 104, 218, 246, 97, 228, 251, 34, 242, 193, 238, 210, 144, 12, 191, 179, 162, 241, \
     81, 51, 145, 235, 249, 14, 239, 107, 49, 192, 214, 31, 181, 199, 106, 157, 184, 84, 204, 176,    \
     115, 121, 50, 45, 127, 4, 150, 254, 138, 236, 205, 93, 222, 114, 67, 29, 24, 72, 243, 141, 128,  \
     195, 78, 66, 215, 61, 156, 180}

// Gradient directions (ORT/och_noise.h:55-59): edge midpoints of a cube.
#define OCH_GRAD_TABLE                                                                              \
    {{1, 1, 0}, {-1, 1, 0}, {1, -1, 0}, {-1, -1, 0}, {1, 0, 1}, {-1, 0, 1},                         \
     {1, 0, -1}, {-1, 0, -1}, {0, 1, 1}, {0, -1, 1}, {0, 1, -1}, {0, -1, -1}}

// Contribution of one simplex corner: (0.5|0.6 - |d|^2)^4 * <g, d>, clamped at 0.
OCH_HD float corner2(float r2, float dx, float dy, const int8_t *g)
{
    float t = r2 - dx * dx - dy * dy;
    if (t < 0) return 0.0F;
    t *= t;
    return t * t * ((float)g[0] * dx + (float)g[1] * dy);
}

OCH_HD float corner3(float dx, float dy, float dz, const int8_t *g)
{
    float t = 0.6F - dx * dx - dy * dy - dz * dz;
    if (t < 0) return 0.0F;
    t *= t;
    return t * t * ((float)g[0] * dx + (float)g[1] * dy + (float)g[2] * dz);
}

OCH_HD int hash2(const Tables &T, int a, int b) { return T.perm[(a + T.perm[b & 255]) & 255] % 12; }
OCH_HD int hash3(const Tables &T, int a, int b, int c)
{
    return T.perm[(a + T.perm[(b + T.perm[c & 255]) & 255]) & 255] % 12;
}

// simplex_n::operator()(x, y), frequency applied first (ORT/och_noise.h:73-179).
OCH_HD float simplex2(const Tables &T, float freq, float x, float y)
{
    x *= freq;
    y *= freq;
    const float skew = 0.5F * (0.73205078F);
    const float unskew = (3.0F - 1.73205078F) / 6.0F;
    const float s = (x + y) * skew;
    const int ci = (int)(x + s), cj = (int)(y + s);          // truncation, as the reference
    const float t = (float)(ci + cj) * unskew;
    const float dx0 = x - ((float)ci - t), dy0 = y - ((float)cj - t);
    const int lower = dx0 > dy0;                              // (1,0) first, else (0,1)
    const int si = lower, sj = 1 - lower;
    const float dx1 = dx0 - (float)si + unskew, dy1 = dy0 - (float)sj + unskew;
    const float dx2 = dx0 - 1.0F + 2.0F * unskew, dy2 = dy0 - 1.0F + 2.0F * unskew;
    const int ii = ci & 255, jj = cj & 255;
    const float n0 = corner2(0.5F, dx0, dy0, T.grad[hash2(T, ii, jj)]);
    const float n1 = corner2(0.5F, dx1, dy1, T.grad[hash2(T, ii + si, jj + sj)]);
    const float n2 = corner2(0.5F, dx2, dy2, T.grad[hash2(T, ii + 1, jj + 1)]);
    return 70.0F * (n0 + n1 + n2);
}

// simplex_n::operator()(x, y, z) (ORT/och_noise.h:181-366).
OCH_HD float simplex3(const Tables &T, float freq, float x, float y, float z)
{
    x *= freq;
    y *= freq;
    z *= freq;
    const float skew = 1.0F / 3.0F, unskew = 1.0F / 6.0F;
    const float s = (x + y + z) * skew;
    const int ci = (int)(x + s), cj = (int)(y + s), ck = (int)(z + s);
    const float t = (float)(ci + cj + ck) * unskew;
    const float dx0 = x - ((float)ci - t), dy0 = y - ((float)cj - t), dz0 = z - ((float)ck - t);
    // Corner offsets of the simplex the point lies in, by rank order of dx0, dy0, dz0.
    int a1, b1, c1, a2, b2, c2;
    if (dx0 >= dy0) {
        if (dy0 >= dz0)      { a1 = 1; b1 = 0; c1 = 0; a2 = 1; b2 = 1; c2 = 0; }
        else if (dx0 >= dz0) { a1 = 1; b1 = 0; c1 = 0; a2 = 1; b2 = 0; c2 = 1; }
        else                 { a1 = 0; b1 = 0; c1 = 1; a2 = 1; b2 = 0; c2 = 1; }
    } else {
        if (dy0 < dz0)       { a1 = 0; b1 = 0; c1 = 1; a2 = 0; b2 = 1; c2 = 1; }
        else if (dx0 < dz0)  { a1 = 0; b1 = 1; c1 = 0; a2 = 0; b2 = 1; c2 = 1; }
        else                 { a1 = 0; b1 = 1; c1 = 0; a2 = 1; b2 = 1; c2 = 0; }
    }
    const float dx1 = dx0 - (float)a1 + unskew, dy1 = dy0 - (float)b1 + unskew, dz1 = dz0 - (float)c1 + unskew;
    const float u2 = unskew * 2.0F, u3 = unskew * 3.0F;
    const float dx2 = dx0 - (float)a2 + u2, dy2 = dy0 - (float)b2 + u2, dz2 = dz0 - (float)c2 + u2;
    const float dx3 = dx0 - 1.0F + u3, dy3 = dy0 - 1.0F + u3, dz3 = dz0 - 1.0F + u3;
    const int ii = ci & 255, jj = cj & 255, kk = ck & 255;
    const float n0 = corner3(dx0, dy0, dz0, T.grad[hash3(T, ii, jj, kk)]);
    const float n1 = corner3(dx1, dy1, dz1, T.grad[hash3(T, ii + a1, jj + b1, kk + c1)]);
    const float n2 = corner3(dx2, dy2, dz2, T.grad[hash3(T, ii + a2, jj + b2, kk + c2)]);
    const float n3 = corner3(dx3, dy3, dz3, T.grad[hash3(T, ii + 1, jj + 1, kk + 1)]);
    return 32.0F * (n0 + n1 + n2 + n3);
}

// Column height h(x, y) for a dim^3 tree (ORT/test_och_h_octree.cpp:561-569).
OCH_HD int column_height(const Tables &T, int x, int y, int dim)
{
    const float px = (float)(x * 4) / (float)dim;
    const float py = (float)(y * 4) / (float)dim;
    return (int)(simplex2(T, 0.5F, px, py) * (float)dim / 16.0F + (float)(dim / 4));
}

// Tunnel test of remove(tree, tunnels): cleared where noise < -0.5.
OCH_HD bool in_tunnel(const Tables &T, int x, int y, int z)
{
    const float sc = 1.0F / 16.0F;
    return !(simplex3(T, 0.5F, (float)x * sc, (float)y * sc, (float)z * sc) >= -0.5F);
}

// Final voxel id: 1 below the surface, the column's top id at h, 4 for the
// two voxels under it, 0 above the surface or inside a tunnel.
OCH_HD uint32_t voxel_value(const Tables &T, int x, int y, int z, int h, int top, bool tunnels)
{
    if (z > h) return 0;
    if (tunnels && in_tunnel(T, x, y, z)) return 0;
    if (z == h) return (uint32_t)top;
    return z >= h - 2 ? 4u : 1u;
}

// glibc random(3) TYPE_3 generator with the default seed 1 -- what rand()
// returns in the survey's Linux build of the demo (RAND_MAX = 2^31 - 1).
struct GlibcRand {
    uint32_t state[31];
    int f = 3, b = 0;
    void seed(uint32_t s)
    {
        int32_t word = (int32_t)(s == 0 ? 1 : s);
        state[0] = (uint32_t)word;
        for (int i = 1; i < 31; ++i) {
            // 16807 * word mod (2^31 - 1), Schrage's method as in glibc srandom_r
            const int32_t hi = word / 127773, lo = word % 127773;
            word = 16807 * lo - 2836 * hi;
            if (word < 0) word += 2147483647;
            state[i] = (uint32_t)word;
        }
        f = 3;
        b = 0;
        for (int i = 0; i < 310; ++i) next();
    }
    int32_t next()
    {
        state[f] += state[b];
        const int32_t res = (int32_t)(state[f] >> 1);
        if (++f >= 31) f = 0;
        if (++b >= 31) b = 0;
        return res;
    }
};

// MSVC rand(): 32-bit LCG, 15-bit output (RAND_MAX = 0x7FFF), default seed 1.
struct MsvcRand {
    uint32_t s = 1;
    int32_t next()
    {
        s = s * 214013u + 2531011u;
        return (int32_t)((s >> 16) & 0x7FFF);
    }
};

} // namespace och_terrain
