// cc_stage_kernels.hip -- device kernels of the stage-level entry points (one reference job each):
// block_faces (block_faces.py:87-137), merge_assignments (merge_assignments.py:105-130) and
// write with offsets (write.py:185-202).  These operate on uint64 label volumes, like the
// reference's intermediate n5 datasets; the fused path (cc_kernels.hip) never materialises them.
#include "cc_common.hpp"

namespace cc {

// Face pairs of one axis (volume_utils.py:187-215, halo 1; block_faces.py:87-113): voxel p on the
// last plane of its block along `axis` pairs with p + e_axis in the next block when both labels
// are non-zero.  Grid (chunk, row group, face plane k): a face plane is walked in rows along its
// fast dimension f (x for z / y faces: coalesced 16-B loads, two voxels each; y for x faces:
// strided by nature), FP_PER voxels per thread, FP_ROWS consecutive rows per workgroup.  A pair
// equal to that of the voxel before it along f or of the voxel in the previous row is not emitted
// (the dedup that follows sees every distinct pair at least once: its first voxel in index order
// always emits); the previous row's pairs stay in registers from one row to the next.  Appends
// collect in an LDS buffer and leave with ONE global atomic per workgroup (per FP_BUF pairs):
// one atomic per row chunk serialised on the counter at ~24 ns each (1.48 ms for the 61 k
// workgroups of C3's z faces, profiles/r03_stage_summary.txt).  maxid (atomicMax) sizes the packed
// sort of dedup_pairs.  No 64-bit division: coordinates from the grid, the block index along f
// from one 32-bit division per thread.
constexpr int FACE_PAIR_THREADS = 256, FP_PER = 4, FP_CHUNK = FACE_PAIR_THREADS * FP_PER, FP_ROWS = 16;
constexpr int FP_BUF = 2 * FP_CHUNK;       // LDS pair buffer: a row chunk emits at most FP_CHUNK pairs

struct FaceGeom {
    int64_t S[3], B[3], nb[3];
    int axis, fdim, rdim;          // face normal, the plane's fast (row) and slow (row index) dimensions
};

__global__ __launch_bounds__(FACE_PAIR_THREADS) void k_face_pairs(FaceGeom G, const u64* __restrict__ L,
                                                                  const u64* __restrict__ off, u64* pa, u64* pb,
                                                                  unsigned long long* counter, u64 cap,
                                                                  unsigned long long* maxid, u8* bflag) {
    __shared__ u32 wcnt[FACE_PAIR_THREADS / 64];
    __shared__ unsigned long long wmax[FACE_PAIR_THREADS / 64];
    __shared__ unsigned long long gbase;
    __shared__ u64 bufa[FP_BUF], bufb[FP_BUF];
    const int ax = G.axis, fd = G.fdim, rd = G.rdim;
    const int64_t k = blockIdx.z;
    const int64_t row0 = (int64_t)blockIdx.y * FP_ROWS, nrow = G.S[rd];
    const int64_t f0 = ((int64_t)blockIdx.x * FACE_PAIR_THREADS + threadIdx.x) * FP_PER;
    const int64_t Sf = G.S[fd];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // strides of the three roles in the C-order volume
    const int64_t st[3] = {G.S[1] * G.S[2], G.S[2], 1};
    const int64_t pax = (k + 1) * G.B[ax] - 1;                 // last plane of block row k along ax
    const int64_t sf = st[fd], sa = st[ax], sr = st[rd];
    int64_t mul[3];                                            // block-index strides per dimension
    mul[0] = G.nb[1] * G.nb[2]; mul[1] = G.nb[2]; mul[2] = 1;
    const u32 Bf = (u32)G.B[fd], Br = (u32)G.B[rd];
    const u32 bf0 = (u32)f0 / Bf;                              // block index along f of voxel f0
    const u32 fe = (bf0 + 1) * Bf;                             // first f of the next block
    bool in[FP_PER];
    u32 bfj[FP_PER];
#pragma unroll
    for (int j = 0; j < FP_PER; ++j) {
        const int64_t f = f0 + j;
        in[j] = f < Sf;
        // FP_PER consecutive voxels cross at most one block face when B_f >= FP_PER
        bfj[j] = Bf >= (u32)FP_PER ? bf0 + ((u64)f >= fe ? 1u : 0u) : (u32)f / Bf;
    }
    const bool hp = f0 > 0 && f0 - 1 < Sf;
    const u32 bfp = hp ? (u32)(f0 - 1) / Bf : 0u;
    // 16-B loads of voxel pairs along f (z / y faces) when the row start is 16-B aligned
    const bool vec = sf == 1 && (((pax * sa) | sr | sa) & 1) == 0;
    u64 pra[FP_PER], prb[FP_PER];                              // the previous row's pairs (0: none)
    u64 mx = 0;
    u32 nbuf = 0;                                              // pairs in the LDS buffer (uniform)
    auto flush = [&]() {
        if (threadIdx.x == 0) gbase = nbuf ? atomicAdd(counter, (unsigned long long)nbuf) : 0ull;
        __syncthreads();
        const unsigned long long b0 = gbase;
        for (u32 i = threadIdx.x; i < nbuf; i += FACE_PAIR_THREADS)
            if (b0 + i < cap) { pa[b0 + i] = bufa[i]; pb[b0 + i] = bufb[i]; }
        __syncthreads();
        nbuf = 0;
    };
    for (int64_t row = row0; row < row0 + FP_ROWS && row < nrow; ++row) {
        const int64_t base = pax * sa + row * sr;              // voxel (pax, row, f = 0)
        const u32 bi_r = (u32)row / Br;
        const int64_t ba_fix = k * mul[ax] + (int64_t)bi_r * mul[rd], bb_fix = ba_fix + mul[ax];
        u64 la[FP_PER], lb[FP_PER];
        if (vec && in[FP_PER - 1]) {
#pragma unroll
            for (int j = 0; j < FP_PER; j += 2) {
                const ulonglong2 va = *reinterpret_cast<const ulonglong2*>(L + base + f0 + j);
                const ulonglong2 vb = *reinterpret_cast<const ulonglong2*>(L + base + f0 + j + sa);
                la[j] = va.x; la[j + 1] = va.y; lb[j] = vb.x; lb[j + 1] = vb.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j < FP_PER; ++j) {
                la[j] = in[j] ? L[base + (f0 + j) * sf] : 0ull;
                lb[j] = in[j] ? L[base + (f0 + j) * sf + sa] : 0ull;
            }
        }
        u64 a[FP_PER], b[FP_PER];
        bool emit[FP_PER];
#pragma unroll
        for (int j = 0; j < FP_PER; ++j) {
            emit[j] = in[j] && la[j] && lb[j];
            a[j] = emit[j] ? la[j] + off[ba_fix + bfj[j] * mul[fd]] : 0ull;
            b[j] = emit[j] ? lb[j] + off[bb_fix + bfj[j] * mul[fd]] : 0ull;
        }
        // the voxel before f0 along f: lane - 1's last pair, loaded by the first lane of a wave
        u64 qa = __shfl_up(a[FP_PER - 1], 1, 64), qb = __shfl_up(b[FP_PER - 1], 1, 64);
        if (lane == 0) {
            qa = qb = 0;
            if (hp) {
                const u64 xa = L[base + (f0 - 1) * sf], xb = L[base + (f0 - 1) * sf + sa];
                if (xa && xb) { qa = xa + off[ba_fix + bfp * mul[fd]]; qb = xb + off[bb_fix + bfp * mul[fd]]; }
            }
        }
        // the previous row (same f): in registers after the workgroup's first row
        if (row == row0 && row > 0) {
            const u32 pbi = (u32)(row - 1) / Br;
            const int64_t fa0 = k * mul[ax] + (int64_t)pbi * mul[rd], fb0 = fa0 + mul[ax];
#pragma unroll
            for (int j = 0; j < FP_PER; ++j) {
                pra[j] = prb[j] = 0;
                if (emit[j]) {
                    const int64_t ip = base - sr + (f0 + j) * sf;
                    const u64 ra = L[ip], rb = L[ip + sa];
                    if (ra && rb) { pra[j] = ra + off[fa0 + bfj[j] * mul[fd]]; prb[j] = rb + off[fb0 + bfj[j] * mul[fd]]; }
                }
            }
        } else if (row == row0) {
#pragma unroll
            for (int j = 0; j < FP_PER; ++j) pra[j] = prb[j] = 0;
        }
        u32 cnt = 0;
#pragma unroll
        for (int j = 0; j < FP_PER; ++j) {
            const u64 pva = j ? a[j - 1] : qa, pvb = j ? b[j - 1] : qb;
            if (emit[j] && ((pva == a[j] && pvb == b[j]) || (pra[j] == a[j] && prb[j] == b[j]))) emit[j] = false;
            pra[j] = a[j];                                     // this row is the next one's previous
            prb[j] = b[j];
            if (emit[j]) {
                mx = a[j] > mx ? a[j] : mx;
                mx = b[j] > mx ? b[j] : mx;
                if (bflag) bflag[ba_fix + bfj[j] * mul[fd]] = 1;      // block_faces.py:116-137 job flag
                ++cnt;
            }
        }
        // workgroup-exclusive scan of the per-thread counts
        u32 x = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { const u32 y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
        if (lane == 63) wcnt[wave] = x;
        __syncthreads();
        u32 wb = 0, tot = 0;
#pragma unroll
        for (int v = 0; v < FACE_PAIR_THREADS / 64; ++v) { const u32 c = wcnt[v]; wb += v < wave ? c : 0u; tot += c; }
        __syncthreads();
        if (nbuf + tot > (u32)FP_BUF) flush();
        u32 pos = nbuf + wb + x - cnt;
#pragma unroll
        for (int j = 0; j < FP_PER; ++j)
            if (emit[j]) { bufa[pos] = a[j]; bufb[pos] = b[j]; ++pos; }
        nbuf += tot;
    }
    __syncthreads();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { const u64 t = __shfl_xor(mx, o, 64); mx = t > mx ? t : mx; }
    if (lane == 0) wmax[wave] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long gm = 0;
        for (int v = 0; v < FACE_PAIR_THREADS / 64; ++v) gm = wmax[v] > gm ? wmax[v] : gm;
        if (gm) atomicMax(maxid, gm);
    }
    if (nbuf) flush();
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
// Grid (chunk of WRITE_CHUNK voxels, y, z): the row's block-row offsets from the grid, the x block
// from one 32-bit division per 16-B pair; each lane issues its WRITE_PER 16-B loads first (memory
// parallelism), then the offset / LUT gathers, then the stores -- background pairs are not
// rewritten (they stay 0).
constexpr int WRITE_THREADS = 256, WRITE_PER = 4, WRITE_CHUNK = 2 * WRITE_THREADS * WRITE_PER;

__global__ __launch_bounds__(WRITE_THREADS) void k_write_offsets(int64_t Y, int64_t X, int64_t bz, int64_t by,
                                                                 u32 bx, int64_t nby, int64_t nbx,
                                                                 u64* __restrict__ L, const u64* __restrict__ off,
                                                                 const u64* __restrict__ lut, u64 n_labels, u32* err) {
    const int64_t z = blockIdx.z, y = blockIdx.y;
    const u64* offr = off + ((z / bz) * nby + y / by) * nbx;
    u64* Lr = L + (z * Y + y) * X;
    const int64_t x0 = (int64_t)blockIdx.x * WRITE_CHUNK + 2 * (int64_t)threadIdx.x;
    bool bad = false;
    auto map = [&](u64 v, int64_t xx) -> u64 {
        if (!v) return 0ull;
        const u64 id = v + offr[(u32)xx / bx];
        if (id >= n_labels) { bad = true; return v; }
        return lut[id];
    };
    if ((X & 1) == 0) {
        ulonglong2 v[WRITE_PER];
#pragma unroll
        for (int j = 0; j < WRITE_PER; ++j) {
            const int64_t x = x0 + j * 2 * WRITE_THREADS;
            v[j] = x < X ? *reinterpret_cast<const ulonglong2*>(Lr + x) : make_ulonglong2(0ull, 0ull);
        }
#pragma unroll
        for (int j = 0; j < WRITE_PER; ++j) {
            const int64_t x = x0 + j * 2 * WRITE_THREADS;
            if (v[j].x | v[j].y) {
                v[j].x = map(v[j].x, x);
                v[j].y = map(v[j].y, x + 1);
            }
        }
#pragma unroll
        for (int j = 0; j < WRITE_PER; ++j) {
            const int64_t x = x0 + j * 2 * WRITE_THREADS;
            if (x < X && (v[j].x | v[j].y)) *reinterpret_cast<ulonglong2*>(Lr + x) = v[j];
        }
    } else {
        for (int j = 0; j < WRITE_PER; ++j)
            for (int q = 0; q < 2; ++q) {
                const int64_t x = x0 + j * 2 * WRITE_THREADS + q;
                if (x >= X) continue;
                const u64 v = Lr[x];
                if (v) Lr[x] = map(v, x);
            }
    }
    if (bad) atomicOr(err, 1u);
}

}  // namespace cc
