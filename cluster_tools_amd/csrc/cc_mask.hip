// cc_mask.hip -- masks whose shape differs from the volume's (block_components.py:274-275 ->
// volume_utils.py:174-184: elf ResizedVolume(mask, shape, order=0), nearest neighbour).
//
// out[z, y, x] = mask[src_z(z), src_y(y), src_x(x)] != 0 with, per axis (mask extent m, volume
// extent S), the pixel-centre nearest neighbour of skimage's resize(order=0):
//     src(c) = floor((c + 0.5) * m / S) = floor((2c + 1) m / (2S))      (integer arithmetic)
// i.e. the whole mask resized at once (elf resizes each requested block's crop; elf is not
// available here, so the block-crop rounding of the reference is not reproduced: parity
// unpinned).  The full-resolution uint8 mask then feeds k_spec like any mask.
#include "cc_common.hpp"

namespace cc {

__device__ __forceinline__ int64_t nn_src(int64_t c, int64_t m, int64_t S) {
    const int64_t s = ((2 * c + 1) * m) / (2 * S);
    return s < m ? s : m - 1;
}

// x source table (one entry per volume column)
__global__ void k_mask_xmap(int64_t X, int64_t mX, int32_t* xmap) {
    CC_FOR(x, X) xmap[x] = (int32_t)nn_src(x, mX, X);
}

// grid: (ceil(X / 1024), nz * Y); thread = 4 consecutive x of one (z, y) row, uchar4 stores
// when X % 4 == 0 (rows 4-B aligned), byte stores otherwise
__global__ __launch_bounds__(256) void k_mask_resize(const u8* __restrict__ mask, int64_t mZ, int64_t mY, int64_t mX,
                                                     int64_t Z, int64_t Y, int64_t X, int64_t z0,
                                                     const int32_t* __restrict__ xmap, u8* __restrict__ out) {
    const int64_t row = blockIdx.y;                // local row: (z - z0) * Y + y
    const int64_t z = z0 + row / Y, y = row % Y;
    const u8* src = mask + (nn_src(z, mZ, Z) * mY + nn_src(y, mY, Y)) * mX;
    u8* dst = out + row * X;
    const int64_t x = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (x >= X) return;
    if ((X & 3) == 0) {
        uchar4 v;
        v.x = src[xmap[x]] != 0; v.y = src[xmap[x + 1]] != 0; v.z = src[xmap[x + 2]] != 0; v.w = src[xmap[x + 3]] != 0;
        *reinterpret_cast<uchar4*>(dst + x) = v;
    } else {
        for (int k = 0; k < 4 && x + k < X; ++k) dst[x + k] = src[xmap[x + k]] != 0;
    }
}

// per-axis source tables: map[0 .. X) x, map[X .. X + Y) y, map[X + Y .. X + Y + Z) z
__global__ void k_mask_maps(int64_t X, int64_t Y, int64_t Z, int64_t mX, int64_t mY, int64_t mZ, int32_t* map) {
    CC_FOR(i, X + Y + Z) {
        if (i < X) map[i] = (int32_t)nn_src(i, mX, X);
        else if (i < X + Y) map[i] = (int32_t)nn_src(i - X, mY, Y);
        else map[i] = (int32_t)nn_src(i - X - Y, mZ, Z);
    }
}

// rows of X % 16 == 0 (the common case): a thread makes 16 consecutive bytes of one row -- the
// x sources as four int4 of the table, one 16-B store -- walking (row, 16-byte unit) with a grid
// stride; the row's source offset comes from the y / z tables (no 64-bit division per thread).
// The one-workgroup-per-row form left half of each 256-thread workgroup idle at X = 2048 and
// launched a workgroup per row (4.6 ms for a C3 volume from a half-size mask; this: DESIGN.md §1).
__global__ __launch_bounds__(256) void k_mask_resize16(const u8* __restrict__ mask, int64_t mY, int64_t mX, int64_t Y,
                                                       int64_t X, int64_t z0, int64_t rows /* nz * Y */,
                                                       const int32_t* __restrict__ map, u8* __restrict__ out) {
    const u32 upr = (u32)(X / 16), yy = (u32)Y;
    const int64_t n = rows * upr;
    CC_FOR(u, n) {
        const u32 row = (u32)(u / upr), xc = (u32)(u - (int64_t)row * upr);
        const u32 zl = row / yy, y = row - zl * yy;
        const u8* src = mask + ((int64_t)map[X + Y + z0 + zl] * mY + map[X + y]) * mX;
        const int4* xm = reinterpret_cast<const int4*>(map + 16 * (int64_t)xc);
        u32 w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int4 s4 = xm[q];
            w[q] = (u32)(src[s4.x] != 0) | ((u32)(src[s4.y] != 0) << 8) | ((u32)(src[s4.z] != 0) << 16) |
                   ((u32)(src[s4.w] != 0) << 24);
        }
        *reinterpret_cast<uint4*>(out + (int64_t)row * X + 16 * (int64_t)xc) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

}  // namespace cc
