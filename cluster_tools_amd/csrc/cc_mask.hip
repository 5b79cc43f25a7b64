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

}  // namespace cc
