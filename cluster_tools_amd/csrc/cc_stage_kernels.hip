// cc_stage_kernels.hip -- device kernels of the stage-level entry points (one reference job each):
// block_faces (block_faces.py:87-137), merge_assignments (merge_assignments.py:105-130) and
// write with offsets (write.py:185-202).  These operate on uint64 label volumes, like the
// reference's intermediate n5 datasets; the fused path (cc_kernels.hip) never materialises them.
#include "cc_common.hpp"

namespace cc {

// Face pairs of one axis (volume_utils.py:187-215, halo 1; block_faces.py:87-113): voxel p on the
// last plane of its block along `axis` pairs with p + e_axis in the next block when both labels
// are non-zero.  Grid: one workgroup per (face plane k, row r, chunk of 1024 along the row's
// contiguous dimension f); the row walks f = x (z / y faces: coalesced uint64 loads) or f = y
// (x faces).  A pair equal to that of the voxel before it along f or the one in the previous
// row is not emitted (the dedup that follows sees every distinct pair at least once: its first
// voxel in index order always emits), and appends are aggregated per workgroup: one global
// atomic per 1024 voxels instead of one per pair.  maxid (atomicMax per workgroup) sizes the
// packed sort of dedup_pairs.  No 64-bit division: the coordinates come from the grid, block
// indices from 32-bit divisions.
constexpr int FACE_PAIR_THREADS = 1024;

struct FaceGeom {
    int64_t S[3], B[3], nb[3];
    int axis, fdim, rdim;          // face normal, the plane's fast (row) and slow (row index) dimensions
    int64_t nrow;                  // rows per face plane = S[rdim]
    int64_t nchunk;                // chunks of FACE_PAIR_THREADS along fdim
};

__device__ __forceinline__ int64_t fg_index(const FaceGeom& G, const int64_t p[3]) {
    return (p[0] * G.S[1] + p[1]) * G.S[2] + p[2];
}
__device__ __forceinline__ int64_t fg_block(const FaceGeom& G, const int64_t p[3]) {
    return (((int64_t)((u32)p[0] / (u32)G.B[0])) * G.nb[1] + (int64_t)((u32)p[1] / (u32)G.B[1])) * G.nb[2] +
           (int64_t)((u32)p[2] / (u32)G.B[2]);
}

__global__ __launch_bounds__(FACE_PAIR_THREADS) void k_face_pairs(FaceGeom G, const u64* __restrict__ L,
                                                                  const u64* __restrict__ off, u64* pa, u64* pb,
                                                                  unsigned long long* counter, u64 cap,
                                                                  unsigned long long* maxid, u8* bflag) {
    __shared__ u32 wcnt[FACE_PAIR_THREADS / 64];
    __shared__ unsigned long long gbase;
    const int64_t w = blockIdx.x;
    const int64_t chunk = w % G.nchunk, row = (w / G.nchunk) % G.nrow, k = w / (G.nchunk * G.nrow);
    const int ax = G.axis, fd = G.fdim, rd = G.rdim;
    int64_t p[3];
    p[ax] = (k + 1) * G.B[ax] - 1;
    p[rd] = row;
    p[fd] = chunk * FACE_PAIR_THREADS + threadIdx.x;
    const int64_t stride = ax == 0 ? G.S[1] * G.S[2] : ax == 1 ? G.S[2] : 1;
    bool emit = false;
    u64 a = 0, b = 0;
    if (p[fd] < G.S[fd]) {
        const int64_t i = fg_index(G, p);
        const u64 la = L[i], lb = L[i + stride];
        if (la && lb) {
            int64_t q[3] = {p[0], p[1], p[2]};
            q[ax] += 1;
            const int64_t ba = fg_block(G, p), bb = fg_block(G, q);
            a = la + off[ba];
            b = lb + off[bb];
            emit = true;
            if (bflag) bflag[ba] = 1;      // block ba's face job has a pair (block_faces.py:116-137)
            // the same pair at the voxel before (f - 1) or in the previous row (r - 1): drop
            for (int d = 0; d < 2 && emit; ++d) {
                const int dim = d == 0 ? fd : rd;
                if (p[dim] == 0) continue;
                int64_t pn[3] = {p[0], p[1], p[2]};
                pn[dim] -= 1;
                const int64_t in = fg_index(G, pn);
                const u64 na = L[in], nbv = L[in + stride];
                if (na && nbv) {
                    int64_t qn[3] = {pn[0], pn[1], pn[2]};
                    qn[ax] += 1;
                    if (na + off[fg_block(G, pn)] == a && nbv + off[fg_block(G, qn)] == b) emit = false;
                }
            }
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 m = __ballot(emit);
    u64 mx = emit ? (a > b ? a : b) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { const u64 t = __shfl_xor(mx, o, 64); mx = t > mx ? t : mx; }
    __shared__ unsigned long long wmax[FACE_PAIR_THREADS / 64];
    if (lane == 0) { wcnt[wave] = (u32)__popcll(m); wmax[wave] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 tot = 0;
        unsigned long long gm = 0;
        for (int v = 0; v < FACE_PAIR_THREADS / 64; ++v) {
            const u32 c = wcnt[v]; wcnt[v] = tot; tot += c;
            gm = wmax[v] > gm ? wmax[v] : gm;
        }
        gbase = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
        if (tot) atomicMax(maxid, gm);
    }
    __syncthreads();
    if (emit) {
        const unsigned long long pos = gbase + wcnt[wave] + __popcll(m & ((1ull << lane) - 1));
        if (pos < cap) { pa[pos] = a; pb[pos] = b; }
    }
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

// packed pair keys (a << nb | b, both < 2^nb, 2 nb <= 64): one radix sort instead of two
__global__ void k_pack_pairs(int64_t n, const u64* a, const u64* b, int nb, u64* key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) key[i] = (a[i] << nb) | b[i];
}
__global__ void k_unpack_pairs(const int* n, const u64* key, int nb, u64* a, u64* b) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < *n) { const u64 k = key[i]; a[i] = k >> nb; b[i] = k & ((1ull << nb) - 1); }
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

// write.py:185-202 -- per non-empty block seg[seg != 0] += off[block]; seg = lut[seg], in place.
// One workgroup per (row (z, y), chunk of 512 voxels): the row's block-row index comes from the
// grid, the x block from a 32-bit division; each lane moves two voxels with one 16-B load and (if
// either is non-zero) one 16-B store -- background pairs are not rewritten (they stay 0).
constexpr int WRITE_THREADS = 256, WRITE_CHUNK = 2 * WRITE_THREADS;

__global__ __launch_bounds__(WRITE_THREADS) void k_write_offsets(int64_t Y, int64_t X, int64_t bz, int64_t by,
                                                                 u32 bx, int64_t nby, int64_t nbx, int64_t nchunk,
                                                                 u64* __restrict__ L, const u64* __restrict__ off,
                                                                 const u64* __restrict__ lut, u64 n_labels, u32* err) {
    const int64_t w = blockIdx.x;
    const int64_t row = w / nchunk, chunk = w % nchunk;
    const int64_t z = row / Y, y = row % Y;
    const u64* offr = off + ((z / bz) * nby + y / by) * nbx;
    u64* Lr = L + row * X;
    const int64_t x = chunk * WRITE_CHUNK + 2 * (int64_t)threadIdx.x;
    if (x >= X) return;
    bool bad = false;
    auto map = [&](u64 v, int64_t xx) -> u64 {
        if (!v) return 0ull;
        const u64 id = v + offr[(u32)xx / bx];
        if (id >= n_labels) { bad = true; return v; }
        return lut[id];
    };
    if ((X & 1) == 0) {
        ulonglong2 v = *reinterpret_cast<const ulonglong2*>(Lr + x);
        if (v.x | v.y) {
            v.x = map(v.x, x);
            v.y = map(v.y, x + 1);
            *reinterpret_cast<ulonglong2*>(Lr + x) = v;
        }
    } else {
        for (int k = 0; k < 2 && x + k < X; ++k) {
            const u64 v = Lr[x + k];
            if (v) Lr[x + k] = map(v, x + k);
        }
    }
    if (bad) atomicOr(err, 1u);
}

}  // namespace cc
