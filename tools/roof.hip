// tools/roof.hip -- HBM read / write ceilings on this box for the access shapes of the path
// (timing only, not part of the library).  Each variant streams the same bytes as C3:
//   rd_f4_uU      float4 per lane, U independent loads in flight per lane (grid-stride)
//   rd_tile_rzR   the tile walk of k_spec / k_block_stats: lane = x, one 256-B row per load
//                 instruction, R planes x 4 rows = 4R loads in flight per lane, 512-thread tiles
//   rd_tile4_rzR  the same tile walk with float4 per lane (16 lanes per 64-float row, 4 rows per
//                 load instruction), R planes x 4 row groups in flight
//   rd_tile4_nt_rzR  the same with non-temporal loads (k_spec's input loads)
//   wr_u2_uU      16-B uint64 pair stores per lane, U per lane per iteration
//   mix_wW_*      the non-temporal tile read plus W 4-B words stored per tile (k_spec: 1920)
// Run: tools/roof Z Y X [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

template <int U>
__global__ __launch_bounds__(256) void rd_f4(const float4* __restrict__ in, int64_t n4, float* out) {
    float acc = 0.f;
    const int64_t stride = (int64_t)gridDim.x * 256 * U;
    for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n4; b += stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = b + u * 256 < n4 ? in[b + u * 256] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w));
    }
    if (acc == 1234.5f) out[0] = acc;
}

// tiles of 16 x 32 x 64 voxels, one 512-thread workgroup per tile, wave w owns rows w + 8 b
template <int RZ>
__global__ __launch_bounds__(512) void rd_tile(const float* __restrict__ in, int64_t Y, int64_t X, int ntx, int nty,
                                               float* out) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
    const float* p = in + (((int64_t)tz * 16) * Y + ty * 32 + wave) * X + tx * 64 + lane;
    const int64_t sz = Y * X, sy = 8 * X;
    float mx = -1e30f;
#pragma unroll
    for (int z0 = 0; z0 < 16; z0 += RZ) {
        float v[RZ][4];
#pragma unroll
        for (int a = 0; a < RZ; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) v[a][b] = p[(z0 + a) * sz + b * sy];
#pragma unroll
        for (int a = 0; a < RZ; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) mx = fmaxf(mx, v[a][b]);
    }
    if (mx == 1234.5f) out[0] = mx;
}

// float4 lanes: lane l reads x = 4 (l % 16) .. + 3 of row group row 4 * (wave-slot) + l / 16
template <int RZ, bool NT = false>
__global__ __launch_bounds__(512) void rd_tile4(const float* __restrict__ in, int64_t Y, int64_t X, int ntx, int nty,
                                                float* out) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
    // wave w: rows y = 4 w + (lane / 16) of each plane (32 rows = 8 waves x 4)
    const float* p = in + (((int64_t)tz * 16) * Y + ty * 32 + 4 * wave + (lane >> 4)) * X + tx * 64 + 4 * (lane & 15);
    const int64_t sz = Y * X;
    float mx = -1e30f;
#pragma unroll
    for (int z0 = 0; z0 < 16; z0 += RZ) {
        float4 v[RZ];
#pragma unroll
        for (int a = 0; a < RZ; ++a) {
            if constexpr (NT) {          // non-temporal, as k_spec's input loads
                typedef float v4f __attribute__((ext_vector_type(4)));
                const v4f w = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p + (z0 + a) * sz));
                v[a] = float4{w.x, w.y, w.z, w.w};
            } else {
                v[a] = *reinterpret_cast<const float4*>(p + (z0 + a) * sz);
            }
        }
#pragma unroll
        for (int a = 0; a < RZ; ++a) mx = fmaxf(mx, fmaxf(fmaxf(v[a].x, v[a].y), fmaxf(v[a].z, v[a].w)));
    }
    if (mx == 1234.5f) out[0] = mx;
}

template <int U>
__global__ __launch_bounds__(256) void wr_u2(ulonglong2* __restrict__ out, int64_t n2) {
    const int64_t stride = (int64_t)gridDim.x * 256 * U;
    for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n2; b += stride)
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (b + u * 256 < n2) out[b + u * 256] = make_ulonglong2((unsigned long long)(b + u), 0);
}

// the k_pass2 shape: one 512-thread tile, each thread 16-B stores of (x, x+1) pairs of cube rows
__global__ __launch_bounds__(512) void wr_tile(unsigned long long* __restrict__ out, int64_t Y, int64_t X, int ntx,
                                               int nty) {
    const int t = blockIdx.x;
    const int tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
    for (int c = threadIdx.x; c < 4096; c += 512) {
        const int cz = c / 512, cy = (c / 32) % 16, cx = c % 32;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int z = 2 * cz + (d >> 1), y = 2 * cy + (d & 1);
            const int64_t idx = (((int64_t)tz * 16 + z) * Y + ty * 32 + y) * X + tx * 64 + 2 * cx;
            *reinterpret_cast<ulonglong2*>(out + idx) = make_ulonglong2((unsigned long long)c, (unsigned long long)d);
        }
    }
}

// the k_pass2 store shape over NT x-adjacent tiles per workgroup (NT * 512-B contiguous rows)
template <int NT>
__global__ __launch_bounds__(512) void wr_tile_w(unsigned long long* __restrict__ out, int64_t Y, int64_t X, int ntx,
                                                 int nty) {
    const int t = blockIdx.x;
    const int tx = t % (ntx / NT), ty = (t / (ntx / NT)) % nty, tz = t / ((ntx / NT) * nty);
    for (int c = threadIdx.x; c < 4096 * NT; c += 512) {
        const int cz = c / (512 * NT), cy = (c / (32 * NT)) % 16, cx = c % (32 * NT);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int z = 2 * cz + (d >> 1), y = 2 * cy + (d & 1);
            const int64_t idx = (((int64_t)tz * 16 + z) * Y + ty * 32 + y) * X + (int64_t)tx * 64 * NT + 2 * cx;
            *reinterpret_cast<ulonglong2*>(out + idx) = make_ulonglong2((unsigned long long)c, (unsigned long long)d);
        }
    }
}

// tile shape sweep: TZ x TY x 64 tiles (TZ * TY = 512 rows, 256 KB of uint64 per workgroup), the
// k_pass2 thread mapping (cube = 2 x 2 voxel rows x 2 voxels, 16-B stores); ZORD: tiles walked
// z-fastest instead of x-fastest
template <int TZ, int TY, bool ZORD = false>
__global__ __launch_bounds__(512) void wr_tile_s(unsigned long long* __restrict__ out, int64_t Y, int64_t X, int ntx,
                                                 int nty, int ntz) {
    const int t = blockIdx.x;
    int tx, ty, tz;
    if (ZORD) { tz = t % ntz; ty = (t / ntz) % nty; tx = t / (ntz * nty); }
    else { tx = t % ntx; ty = (t / ntx) % nty; tz = t / (ntx * nty); }
    constexpr int CYN = TY / 2, NC = (TZ / 2 > 0 ? TZ / 2 : 1) * CYN * 32;
    for (int c = threadIdx.x; c < NC; c += 512) {
        const int cz = c / (CYN * 32), cy = (c / 32) % CYN, cx = c % 32;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int z = (TZ == 1 ? 0 : 2 * cz + (d >> 1)), y = 2 * cy + (d & 1);
            if (TZ == 1 && (d >> 1)) continue;
            const int64_t idx = (((int64_t)tz * TZ + z) * Y + (int64_t)ty * TY + y) * X + tx * 64 + 2 * cx;
            *reinterpret_cast<ulonglong2*>(out + idx) = make_ulonglong2((unsigned long long)c, (unsigned long long)d);
        }
    }
}

// wr_tile_s plus k_pass2's per-tile bit-row read first (4 KB at bits + t * 512 in TILE-INDEX
// order, whatever order the workgroups walk the tiles in): is a z-ordered walk slow because of
// that read?  (BITSZ: the bit rows laid out in the walk's order instead)
template <bool ZORD, bool BITSZ>
__global__ __launch_bounds__(512) void wr_tile_bits(unsigned long long* __restrict__ out, const unsigned long long* __restrict__ bits,
                                                    int64_t Y, int64_t X, int ntx, int nty, int ntz) {
    const int t = blockIdx.x;
    int tx, ty, tz;
    if (ZORD) { tz = t % ntz; ty = (t / ntz) % nty; tx = t / (ntz * nty); }
    else { tx = t % ntx; ty = (t / ntx) % nty; tz = t / (ntx * nty); }
    const int64_t tile = BITSZ ? (int64_t)t : ((int64_t)tz * nty + ty) * ntx + tx;
    const unsigned long long b = bits[tile * 512 + threadIdx.x];
    __shared__ unsigned long long sb[512];
    sb[threadIdx.x] = b;
    __syncthreads();
    for (int c = threadIdx.x; c < 4096; c += 512) {
        const int cz = c / 512, cy = (c / 32) % 16, cx = c % 32;
        const unsigned long long v = sb[(c * 7) & 511];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int z = 2 * cz + (d >> 1), y = 2 * cy + (d & 1);
            const int64_t idx = (((int64_t)tz * 16 + z) * Y + ty * 32 + y) * X + tx * 64 + 2 * cx;
            *reinterpret_cast<ulonglong2*>(out + idx) = make_ulonglong2(v ^ (unsigned long long)c, (unsigned long long)d);
        }
    }
}

// read-side sweep: float4 lanes over TZ x TY x 64 tiles (k_spec's load shape)
template <int TZ, int TY>
__global__ __launch_bounds__(512) void rd_tile4_s(const float* __restrict__ in, int64_t Y, int64_t X, int ntx, int nty,
                                                  float* out) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
    float mx = -1e30f;
    // 512 rows of 64 floats; one load instruction = 4 rows (16 lanes each); wave w takes row groups w, w + 8, ...
    for (int gi = wave; gi < TZ * TY / 4; gi += 8) {
        const int row = gi * 4 + (lane >> 4), z = row / TY, y = row % TY;
        const float4 v = *reinterpret_cast<const float4*>(in + (((int64_t)tz * TZ + z) * Y + (int64_t)ty * TY + y) * X +
                                                          tx * 64 + 4 * (lane & 15));
        mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
    if (mx == 1234.5f) out[0] = mx;
}

template <class F>
static double time_ms(hipStream_t s, int iters, F&& f) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
    CHK(hipGetLastError());
    CHK(hipEventRecord(a, s));
    for (int i = 0; i < iters; ++i) f();
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

// k_spec's memory pattern without its compute: the non-temporal tile read (rd_tile4_nt, one plane
// in flight) plus W 4-byte words stored per tile after the read (BITS 1024 words + FACES 896 words
// = 1920 in k_spec), non-temporally (NT) or plainly: how much a side stream of stores costs the read
template <int W, bool NT>
__global__ __launch_bounds__(512) void mix_tile(const float* __restrict__ in, int64_t Y, int64_t X, int ntx, int nty,
                                                unsigned* __restrict__ side) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
    const float* p = in + (((int64_t)tz * 16) * Y + ty * 32 + 4 * wave + (lane >> 4)) * X + tx * 64 + 4 * (lane & 15);
    const int64_t sz = Y * X;
    float mx = -1e30f;
#pragma unroll
    for (int z = 0; z < 16; ++z) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        asm volatile("" ::: "memory");
        const v4f w = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p + z * sz));
        mx = fmaxf(mx, fmaxf(fmaxf(w.x, w.y), fmaxf(w.z, w.w)));
    }
    const unsigned v = __float_as_uint(mx);
    unsigned* q = side + (int64_t)t * W;
    for (int i = threadIdx.x; i < W; i += 512) {
        if (NT) __builtin_nontemporal_store(v + i, q + i);
        else q[i] = v + i;
    }
    if ((int)threadIdx.x >= W && v == 0x12345678u) q[0] = v;  // keeps every thread's loads live
}

// mix_tile with k_spec<mask>'s second input: a u8 mask read with plain 4-byte loads beside the
// non-temporal float4 loads (the masked pass's memory pattern: 5 B per voxel in, W words out).
template <int W>
__global__ __launch_bounds__(512) void mix_mask(const float* __restrict__ in, const unsigned* __restrict__ mask, int64_t Y,
                                                int64_t X, int ntx, int nty, unsigned* __restrict__ side) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
    const int64_t off = (((int64_t)tz * 16) * Y + ty * 32 + 4 * wave + (lane >> 4)) * X + tx * 64 + 4 * (lane & 15);
    const float* p = in + off;
    const unsigned* m = mask + off / 4;
    const int64_t sz = Y * X;
    float mx = -1e30f;
    unsigned mm = 0;
#pragma unroll
    for (int z = 0; z < 16; ++z) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        asm volatile("" ::: "memory");
        const v4f w = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p + z * sz));
        mm |= m[z * sz / 4];
        mx = fmaxf(mx, fmaxf(fmaxf(w.x, w.y), fmaxf(w.z, w.w)));
    }
    const unsigned v = __float_as_uint(mx) ^ mm;
    unsigned* q = side + (int64_t)t * W;
    for (int i = threadIdx.x; i < W; i += 512) __builtin_nontemporal_store(v + i, q + i);
    if ((int)threadIdx.x >= W && v == 0x12345678u) q[0] = v;
}

// Persistent form of mix_tile: G workgroups walk tiles t = k*G + g; each keeps the side words of
// E consecutive tiles in LDS and stores them together, so the chip's stores come in bunches
// between read stretches (no grid barrier: uniform work keeps the workgroups roughly in step).
template <int W, int E>
__global__ __launch_bounds__(512) void mix_epoch(const float* __restrict__ in, int64_t Y, int64_t X, int ntx, int nty,
                                                 int ntiles, unsigned* __restrict__ side) {
    __shared__ unsigned buf[E * W];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t sz = Y * X;
    int e = 0, t0 = blockIdx.x;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
        const float* p = in + (((int64_t)tz * 16) * Y + ty * 32 + 4 * wave + (lane >> 4)) * X + tx * 64 + 4 * (lane & 15);
        float mx = -1e30f;
#pragma unroll
        for (int z = 0; z < 16; ++z) {
            typedef float v4f __attribute__((ext_vector_type(4)));
            asm volatile("" ::: "memory");
            const v4f w = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p + z * sz));
            mx = fmaxf(mx, fmaxf(fmaxf(w.x, w.y), fmaxf(w.z, w.w)));
        }
        const unsigned v = __float_as_uint(mx);
        for (int i = threadIdx.x; i < W; i += 512) buf[e * W + i] = v + i;
        if (++e == E || t + (int)gridDim.x >= ntiles) {
            __syncthreads();
            for (int k = 0; k < e; ++k) {
                unsigned* q = side + (int64_t)(t0 + k * (int)gridDim.x) * W;
                for (int i = threadIdx.x; i < W; i += 512) __builtin_nontemporal_store(buf[k * W + i], q + i);
            }
            __syncthreads();
            e = 0;
            t0 = t + gridDim.x;
        }
    }
}

// Bounded grid barrier (thread 0 of each workgroup arrives and spins; gives up after ~2^20 polls and
// counts the give-up in tmo, so a non-resident grid skews a timing instead of hanging the device).
__device__ inline void grid_sync(unsigned* ctr, unsigned target, unsigned* tmo) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        atomicAdd(ctr, 1u);
        int spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++spins > (1 << 20)) {
                atomicAdd(tmo, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

// mix_epoch with chip-wide phases: every workgroup reads E tiles (side words into LDS), grid
// barrier, every workgroup stores its E tiles' words, grid barrier — the stores no longer share
// the memory with the read stream (G must be resident at once).
template <int W, int E>
__global__ __launch_bounds__(512) void mix_gbar(const float* __restrict__ in, int64_t Y, int64_t X, int ntx, int nty,
                                                int ntiles, unsigned* __restrict__ side, unsigned* ctr, unsigned* tmo) {
    __shared__ unsigned buf[E * W];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t sz = Y * X;
    const int G = gridDim.x, tpw = ntiles / G;
    unsigned nbar = 0;
    for (int k0 = 0; k0 < tpw; k0 += E) {
        const int ne = tpw - k0 < E ? tpw - k0 : E;
        for (int e = 0; e < ne; ++e) {
            const int t = (k0 + e) * G + blockIdx.x;
            const int tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
            const float* p = in + (((int64_t)tz * 16) * Y + ty * 32 + 4 * wave + (lane >> 4)) * X + tx * 64 + 4 * (lane & 15);
            float mx = -1e30f;
#pragma unroll
            for (int z = 0; z < 16; ++z) {
                typedef float v4f __attribute__((ext_vector_type(4)));
                asm volatile("" ::: "memory");
                const v4f w = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p + z * sz));
                mx = fmaxf(mx, fmaxf(fmaxf(w.x, w.y), fmaxf(w.z, w.w)));
            }
            const unsigned v = __float_as_uint(mx);
            for (int i = threadIdx.x; i < W; i += 512) buf[e * W + i] = v + i;
        }
        grid_sync(ctr, ++nbar * G, tmo);
        for (int e = 0; e < ne; ++e) {
            unsigned* q = side + (int64_t)((k0 + e) * G + blockIdx.x) * W;
            for (int i = threadIdx.x; i < W; i += 512) __builtin_nontemporal_store(buf[e * W + i], q + i);
        }
        grid_sync(ctr, ++nbar * G, tmo);
    }
}

// The side stores alone (no reads): what the 1920 words/tile would cost in a phase of their own.
template <int W>
__global__ __launch_bounds__(512) void side_only(unsigned* __restrict__ side) {
    unsigned* q = side + (int64_t)blockIdx.x * W;
    for (int i = threadIdx.x; i < W; i += 512) __builtin_nontemporal_store((unsigned)(blockIdx.x + i), q + i);
}

int main(int argc, char** argv) {
    const int64_t Z = argc > 1 ? atoll(argv[1]) : 1024, Y = argc > 2 ? atoll(argv[2]) : 2048,
                  X = argc > 3 ? atoll(argv[3]) : 2048;
    const int iters = argc > 4 ? atoi(argv[4]) : 10;
    const int64_t n = Z * Y * X;
    float* in;
    unsigned long long* out;
    float* dummy;
    CHK(hipMalloc(&in, n * 4));
    CHK(hipMalloc(&out, n * 8));
    CHK(hipMalloc(&dummy, 64));
    CHK(hipMemset(in, 0, n * 4));
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    const int ntx = (int)(X / 64), nty = (int)(Y / 32), ntz = (int)(Z / 16);
    const unsigned nt = (unsigned)ntx * nty * ntz;
    std::vector<std::pair<std::string, double>> r;
    const unsigned g = 256 * 16;
    r.push_back({"rd_f4_u1", time_ms(s, iters, [&] { rd_f4<1><<<g * 4, 256, 0, s>>>((const float4*)in, n / 4, dummy); })});
    r.push_back({"rd_f4_u2", time_ms(s, iters, [&] { rd_f4<2><<<g * 2, 256, 0, s>>>((const float4*)in, n / 4, dummy); })});
    r.push_back({"rd_f4_u4", time_ms(s, iters, [&] { rd_f4<4><<<g, 256, 0, s>>>((const float4*)in, n / 4, dummy); })});
    r.push_back({"rd_f4_u8", time_ms(s, iters, [&] { rd_f4<8><<<g, 256, 0, s>>>((const float4*)in, n / 4, dummy); })});
    r.push_back({"rd_f4_u8_g1k", time_ms(s, iters, [&] { rd_f4<8><<<1024, 256, 0, s>>>((const float4*)in, n / 4, dummy); })});
    r.push_back({"rd_tile_rz2", time_ms(s, iters, [&] { rd_tile<2><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile_rz4", time_ms(s, iters, [&] { rd_tile<4><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile_rz8", time_ms(s, iters, [&] { rd_tile<8><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile_rz16", time_ms(s, iters, [&] { rd_tile<16><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile4_rz2", time_ms(s, iters, [&] { rd_tile4<2><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile4_rz4", time_ms(s, iters, [&] { rd_tile4<4><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile4_rz8", time_ms(s, iters, [&] { rd_tile4<8><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile4_rz16", time_ms(s, iters, [&] { rd_tile4<16><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile4_nt_rz1", time_ms(s, iters, [&] { rd_tile4<1, true><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    r.push_back({"rd_tile4_nt_rz4", time_ms(s, iters, [&] { rd_tile4<4, true><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, dummy); })});
    // read + side stores per tile (the side buffer is the start of `out`: nt * 1920 words)
#define MIX(W, NT, NAME) r.push_back({NAME, time_ms(s, iters, [&] { mix_tile<W, NT><<<nt, 512, 0, s>>>(in, Y, X, ntx, nty, (unsigned*)out); })});
    MIX(0, true, "mix_w0")
    MIX(128, true, "mix_w128_nt")
    MIX(256, true, "mix_w256_nt")
    MIX(512, true, "mix_w512_nt")
    MIX(1024, true, "mix_w1024_nt")
    MIX(1472, true, "mix_w1472_nt")
    MIX(1920, true, "mix_w1920_nt")
    MIX(1920, false, "mix_w1920_plain")
#undef MIX
#define EP(E, G, NAME) r.push_back({NAME, time_ms(s, iters, [&] { mix_epoch<1920, E><<<G, 512, 0, s>>>(in, Y, X, ntx, nty, (int)nt, (unsigned*)out); })});
    EP(1, 512, "epoch_e1_g512")
    EP(4, 512, "epoch_e4_g512")
    EP(8, 512, "epoch_e8_g512")
    EP(4, 1024, "epoch_e4_g1024")
    EP(8, 1024, "epoch_e8_g1024")
#undef EP
    {
        unsigned* mask;
        CHK(hipMalloc(&mask, n));
        CHK(hipMemset(mask, 1, n));
        r.push_back({"mask_rd_w0", time_ms(s, iters, [&] { mix_mask<0><<<nt, 512, 0, s>>>(in, mask, Y, X, ntx, nty, (unsigned*)out); })});
        r.push_back({"mask_mix_w1920", time_ms(s, iters, [&] { mix_mask<1920><<<nt, 512, 0, s>>>(in, mask, Y, X, ntx, nty, (unsigned*)out); })});
        CHK(hipFree(mask));
    }
    unsigned* bar;
    CHK(hipMalloc(&bar, 16));
    CHK(hipMemset(bar, 0, 16));
#define GB(E, G, NAME)                                                                                               \
    {                                                                                                               \
        r.push_back({NAME, time_ms(s, iters, [&] {                                                                  \
                         CHK(hipMemsetAsync(bar, 0, 4, s));                                                         \
                         mix_gbar<1920, E><<<G, 512, 0, s>>>(in, Y, X, ntx, nty, (int)nt, (unsigned*)out, bar, bar + 1); \
                     })});                                                                                          \
        unsigned h[2];                                                                                              \
        CHK(hipMemcpy(h, bar, 8, hipMemcpyDeviceToHost));                                                           \
        r.push_back({std::string(NAME) + "_tmo", (double)h[1]});                                                    \
        CHK(hipMemset(bar, 0, 16));                                                                                 \
    }
    if (std::getenv("ROOF_GBAR")) {  // measured in r05_roof_mix_gbar_fastbox.txt; 6-9 ms each
        GB(8, 256, "gbar_e8_g256")
        GB(16, 256, "gbar_e16_g256")
        GB(8, 512, "gbar_e8_g512")
    }
#undef GB
    r.push_back({"side_only_w1920", time_ms(s, iters, [&] { side_only<1920><<<nt, 512, 0, s>>>((unsigned*)out); })});
    r.push_back({"side_only_w1024", time_ms(s, iters, [&] { side_only<1024><<<nt, 512, 0, s>>>((unsigned*)out); })});
    r.push_back({"wr_u2_u1", time_ms(s, iters, [&] { wr_u2<1><<<g * 8, 256, 0, s>>>((ulonglong2*)out, n / 2); })});
    r.push_back({"wr_u2_u4", time_ms(s, iters, [&] { wr_u2<4><<<g * 2, 256, 0, s>>>((ulonglong2*)out, n / 2); })});
    r.push_back({"wr_u2_u8", time_ms(s, iters, [&] { wr_u2<8><<<g, 256, 0, s>>>((ulonglong2*)out, n / 2); })});
    r.push_back({"wr_tile", time_ms(s, iters, [&] { wr_tile<<<nt, 512, 0, s>>>(out, Y, X, ntx, nty); })});
    r.push_back({"wr_tile_w2", time_ms(s, iters, [&] { wr_tile_w<2><<<nt / 2, 512, 0, s>>>(out, Y, X, ntx, nty); })});
    r.push_back({"wr_tile_w4", time_ms(s, iters, [&] { wr_tile_w<4><<<nt / 4, 512, 0, s>>>(out, Y, X, ntx, nty); })});
    const int64_t nrow = (Y / 64) * 0 + 1;
    (void)nrow;
#define WS(TZ, TY, ZO, NAME)                                                                                        \
    r.push_back({NAME, time_ms(s, iters, [&] {                                                                      \
                     wr_tile_s<TZ, TY, ZO><<<nt, 512, 0, s>>>(out, Y, X, ntx, (int)(Y / TY), (int)(Z / TZ));        \
                 })});
    WS(16, 32, false, "wr_s16x32")
    WS(16, 32, true, "wr_s16x32_zord")
    WS(8, 64, false, "wr_s8x64")
    WS(4, 128, false, "wr_s4x128")
    WS(2, 256, false, "wr_s2x256")
    WS(1, 512, false, "wr_s1x512")
    {
        unsigned long long* bits;
        CHK(hipMalloc(&bits, (size_t)nt * 512 * 8));
        CHK(hipMemset(bits, 0, (size_t)nt * 512 * 8));
        r.push_back({"wr_bits_lin", time_ms(s, iters, [&] { wr_tile_bits<false, false><<<nt, 512, 0, s>>>(out, bits, Y, X, ntx, nty, (int)(Z / 16)); })});
        r.push_back({"wr_bits_zord", time_ms(s, iters, [&] { wr_tile_bits<true, false><<<nt, 512, 0, s>>>(out, bits, Y, X, ntx, nty, (int)(Z / 16)); })});
        r.push_back({"wr_bits_zord_zbits", time_ms(s, iters, [&] { wr_tile_bits<true, true><<<nt, 512, 0, s>>>(out, bits, Y, X, ntx, nty, (int)(Z / 16)); })});
        CHK(hipFree(bits));
    }
#define RS(TZ, TY, NAME)                                                                                            \
    r.push_back({NAME, time_ms(s, iters, [&] { rd_tile4_s<TZ, TY><<<nt, 512, 0, s>>>(in, Y, X, ntx, (int)(Y / TY), dummy); })});
    RS(16, 32, "rd_s16x32")
    RS(8, 64, "rd_s8x64")
    RS(4, 128, "rd_s4x128")
    RS(1, 512, "rd_s1x512")
    std::printf("{\"shape\": [%lld, %lld, %lld]", (long long)Z, (long long)Y, (long long)X);
    for (auto& kv : r) std::printf(", \"%s\": %.4f", kv.first.c_str(), kv.second);
    std::printf("}\n");
    for (auto& kv : r)
        std::printf("# %-16s %7.3f ms  %6.0f GB/s\n", kv.first.c_str(), kv.second,
                    (kv.first[0] == 'r' ? 4.0 : 8.0) * n / kv.second / 1e6);
    return 0;
}
