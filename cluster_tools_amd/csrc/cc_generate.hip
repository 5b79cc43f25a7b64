// cc_generate.hip -- synthetic boundary map on the device (definition and CPU
// restatement in oracle/synth.py and oracle/cc_oracle.c, checked bit-identical by the tests).
#include "cc_common.hpp"

namespace cc {

__device__ __forceinline__ u64 splitmix64(u64 x) {
    u64 z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr int GEN_PITCH = 32;
constexpr u64 GEN_NOISE_SALT = 0x5851F42D4C957F2Dull;

// One thread per voxel along x; a block handles one (z, y) row segment of 256 voxels.  The 27
// seeds of the 3x3x3 cells around a row's cells are shared by the row, so they are computed
// once per block into LDS (the row spans at most 9 cells along x -> 3*3*11 seeds).
__global__ __launch_bounds__(256) void k_generate(float* __restrict__ out, int64_t Z, int64_t Y, int64_t X,
                                                  int64_t oz, int64_t oy, int64_t ox, u64 seed, int dither) {
    __shared__ int64_t sp[3][3][11][3];
    const int64_t nxb = (X + 255) / 256;
    const int64_t row = (int64_t)blockIdx.y * Y + blockIdx.x / nxb;   // grid (Y * nxb, Z)
    const int64_t xb = blockIdx.x % nxb;
    const int64_t z = row / Y + oz, y = row % Y + oy;
    const int64_t xs = xb * 256 + ox;
    const int64_t cz = z / GEN_PITCH, cy = y / GEN_PITCH, cx0 = xs / GEN_PITCH - 1;
    for (int i = threadIdx.x; i < 3 * 3 * 11; i += 256) {
        const int dz = i / 33 - 1, dy = (i / 11) % 3 - 1, ix = i % 11;
        const int64_t nz = cz + dz, ny = cy + dy, nx = cx0 + ix;
        const u64 key = ((u64)(nz + 1) << 42) | ((u64)(ny + 1) << 21) | (u64)(nx + 1);
        const u64 h = splitmix64(seed ^ key);
        sp[dz + 1][dy + 1][ix][0] = nz * GEN_PITCH + (int64_t)(h & 31);
        sp[dz + 1][dy + 1][ix][1] = ny * GEN_PITCH + (int64_t)((h >> 5) & 31);
        sp[dz + 1][dy + 1][ix][2] = nx * GEN_PITCH + (int64_t)((h >> 10) & 31);
    }
    __syncthreads();
    const int64_t xl = xb * 256 + threadIdx.x;
    if (xl >= X) return;
    const int64_t x = xl + ox;
    const int ixc = (int)(x / GEN_PITCH - cx0);     // in [1, 9]
    int64_t d1 = (int64_t)1 << 62, d2 = (int64_t)1 << 62;
#pragma unroll
    for (int dz = 0; dz < 3; ++dz)
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const int64_t* s = sp[dz][dy][ixc + dx];
                const int64_t a = z - s[0], b = y - s[1], c = x - s[2];
                const int64_t d = a * a + b * b + c * c;
                if (d < d1) { d2 = d1; d1 = d; }
                else if (d < d2) { d2 = d; }
            }
    int64_t m = 255 - (d2 - d1);
    if (m < 0) m = 0;
    const u64 vkey = ((u64)z << 42) | ((u64)y << 21) | (u64)x;
    const u64 nh = splitmix64((seed + GEN_NOISE_SALT) ^ vkey);
    int64_t q = m + (int64_t)(nh % 33) - 16;
    q = q < 0 ? 0 : (q > 255 ? 255 : q);
    // continuous variant: (q * 2^16 + 16-bit dither) / 2^24, exact in float32
    const float v = dither ? (float)((u32)q * 65536u + (u32)((nh >> 16) & 0xFFFF)) / 16777216.0f : (float)q / 256.0f;
    out[((row / Y) * Y + (row % Y)) * X + xl] = v;
}

}  // namespace cc
