// cc_stage_kernels.hip -- device kernels of the stage-level entry points (one reference job each):
// block_faces (block_faces.py:87-137), merge_assignments (merge_assignments.py:105-130) and
// write with offsets (write.py:185-202).  These operate on uint64 label volumes, like the
// reference's intermediate n5 datasets; the fused path (cc_kernels.hip) never materialises them.
#include "cc_common.hpp"

namespace cc {

// Face pairs of one axis.  Voxel (p) on the last plane of its block along `axis` pairs with
// p + e_axis in the next block (volume_utils.py:187-215, halo 1).
__global__ void k_face_pairs(int axis, int64_t Z, int64_t Y, int64_t X, int64_t bz, int64_t by, int64_t bx,
                             int64_t nbz, int64_t nby, int64_t nbx, const u64* __restrict__ L,
                             const u64* __restrict__ off, u64* pa, u64* pb, unsigned long long* counter,
                             u64 cap, u8* bflag) {
    const int64_t S[3] = {Z, Y, X}, B[3] = {bz, by, bx};
    const int64_t nplanes = (S[axis] - 1) / B[axis];       // block faces with an upper neighbour
    const int64_t plane = (axis == 0 ? Y * X : axis == 1 ? Z * X : Z * Y);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nplanes * plane) return;
    const int64_t k = i / plane, r = i % plane;
    int64_t p[3];
    const int a1 = axis == 0 ? 1 : 0, a2 = axis == 2 ? 1 : 2;
    p[axis] = (k + 1) * B[axis] - 1;
    p[a1] = r / S[a2];
    p[a2] = r % S[a2];
    const int64_t idx = (p[0] * Y + p[1]) * X + p[2];
    const int64_t stride = axis == 0 ? Y * X : axis == 1 ? X : 1;
    const u64 la = L[idx], lb = L[idx + stride];
    if (!la || !lb) return;
    const int64_t ba = ((p[0] / bz) * nby + p[1] / by) * nbx + p[2] / bx;
    int64_t q[3] = {p[0], p[1], p[2]};
    q[axis] += 1;
    const int64_t bb = ((q[0] / bz) * nby + q[1] / by) * nbx + q[2] / bx;
    const unsigned long long pos = atomicAdd(counter, 1ull);
    if (pos < cap) { pa[pos] = la + off[ba]; pb[pos] = lb + off[bb]; }
    if (bflag) bflag[ba] = 1;      // block ba's face job has a pair (block_faces.py:116-137)
    (void)nbz;
}

__global__ void k_interleave(int64_t n, const u64* a, const u64* b, u64* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[2 * i] = a[i];
    out[2 * i + 1] = b[i];
}

__global__ void k_unique_flags(int64_t n, const u64* a, const u64* b, u8* flags) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flags[i] = (i == 0 || a[i] != a[i - 1] || b[i] != b[i - 1]) ? 1 : 0;
}

// union-find over ids (merge_assignments.py:125-130); representative = smallest id
__device__ __forceinline__ u64 gload64(u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void gstore64(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ u64 gfind64(u64* P, u64 x) {
    while (true) {
        u64 p = gload64(P + x);
        if (p == x) return x;
        u64 gp = gload64(P + p);
        if (gp == p) return p;
        gstore64(P + x, gp);
        x = gp;
    }
}

__global__ void k_iota64(u64 n, u64* P) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) P[i] = i;
}

__global__ void k_union_pairs(int64_t n, const u64* pairs, u64 n_labels, u64* P, u32* err) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u64 a = pairs[2 * i], b = pairs[2 * i + 1];
    if (a >= n_labels || b >= n_labels) { atomicOr(err, 1u); return; }
    while (true) {
        a = gfind64(P, a);
        b = gfind64(P, b);
        if (a == b) return;
        if (a < b) { u64 t = a; a = b; b = t; }
        const unsigned long long old = atomicCAS((unsigned long long*)(P + a), (unsigned long long)a,
                                                 (unsigned long long)b);
        if (old == a) return;
    }
}

__global__ void k_resolve64(u64 n, u64* P) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) P[i] = gfind64(P, i);
}

// write.py:199-200 -- seg[seg != 0] += off[block]; seg = lut[seg]
__global__ void k_write_offsets(int64_t Z, int64_t Y, int64_t X, int64_t bz, int64_t by, int64_t bx,
                                int64_t nby, int64_t nbx, u64* __restrict__ L, const u64* __restrict__ off,
                                const u64* __restrict__ lut, u64 n_labels, u32* err) {
    CC_FOR(i, Z * Y * X) {
        const u64 v = L[i];
        if (!v) continue;
        const int64_t z = i / (Y * X), y = (i / X) % Y, x = i % X;
        const u64 id = v + off[((z / bz) * nby + y / by) * nbx + x / bx];
        if (id >= n_labels) { atomicOr(err, 1u); continue; }
        L[i] = lut[id];
    }
}

}  // namespace cc
