// cc_prefilter.hip -- input preparation before the labelling (included at the end of cc_lib.hip).
//
// Multi-channel input (`channel` of BlockComponents / Threshold): the reference copies the selected
// channels of a 4-D (C, Z, Y, X) dataset into a stack of the dataset's dtype and averages it with
// np.mean(axis=0) (block_components.py:150-159, threshold.py:139-148) before vu.normalize casts to
// float32 (volume_utils.py:99).  numpy reduces over the outer axis element by element in list
// order; the accumulator is float32 for float32 input and float64 otherwise, and the sum is divided
// by the channel count in that type.  The mean is elementwise, so one streaming kernel produces the
// float32 volume the labelling reads: (n_sel * sizeof(T) + 4) B/voxel, HBM-bound.

namespace cc {

constexpr int CHAN_MAX = 64;
struct ChanList {
    int32_t n;
    int32_t c[CHAN_MAX];
};

template <typename T> struct MeanAcc { using type = double; };
template <> struct MeanAcc<float> { using type = float; };

template <typename T, int V> struct alignas(V * sizeof(T)) VecT { T v[V]; };

// V consecutive voxels per lane (one 4..16-byte load per selected channel), grid-stride over
// vector groups; the tail (n % V voxels) is done by the first lanes.
template <typename T, int V>
__global__ __launch_bounds__(256) void k_channel_mean(const T* __restrict__ in, int64_t n, ChanList cl,
                                                      float* __restrict__ out) {
    using A = typename MeanAcc<T>::type;
    const A cnt = (A)cl.n;
    const int64_t ng = n / V;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t g = tid; g < ng; g += stride) {
        A acc[V];
        {
            const VecT<T, V> x = *(const VecT<T, V>*)(in + (int64_t)cl.c[0] * n + g * V);
#pragma unroll
            for (int k = 0; k < V; ++k) acc[k] = (A)x.v[k];
        }
        for (int j = 1; j < cl.n; ++j) {
            const VecT<T, V> x = *(const VecT<T, V>*)(in + (int64_t)cl.c[j] * n + g * V);
#pragma unroll
            for (int k = 0; k < V; ++k) acc[k] = acc[k] + (A)x.v[k];
        }
        VecT<float, V> r;
#pragma unroll
        for (int k = 0; k < V; ++k) r.v[k] = (float)(acc[k] / cnt);
        *(VecT<float, V>*)(out + g * V) = r;
    }
    for (int64_t i = ng * V + tid; i < n; i += stride) {
        A acc = (A)in[(int64_t)cl.c[0] * n + i];
        for (int j = 1; j < cl.n; ++j) acc = acc + (A)in[(int64_t)cl.c[j] * n + i];
        out[i] = (float)(acc / cnt);
    }
}

template <typename T>
static void launch_channel_mean(cc_ctx* c, const void* in, int64_t n, const ChanList& cl, float* out) {
    // 16-byte loads when every channel plane and the output stay 16-byte aligned
    constexpr int V = 16 / sizeof(T) < 4 ? 4 : 16 / sizeof(T);
    const bool vec = ((uintptr_t)in % (V * sizeof(T)) == 0) && ((uintptr_t)out % (V * sizeof(float)) == 0) &&
                     (n % V == 0);
    const int64_t work = vec ? n / V : n;
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(1, (work + 255) / 256), 256 * 16);
    hipStream_t s = cstream(c);
    launch(c, "k_channel_mean", [&] {
        if (vec) k_channel_mean<T, V><<<grid, 256, 0, s>>>((const T*)in, n, cl, out);
        else k_channel_mean<T, 1><<<grid, 256, 0, s>>>((const T*)in, n, cl, out);
    });
}

}  // namespace cc

extern "C" {

int cc_channel_mean(cc_ctx* c, const void* in_dev, int dtype, const int64_t shape4[4], const int64_t* channels,
                    int64_t n_channels, float* out_dev) {
    CC_TRY({
        CC_REQUIRE(c && in_dev && shape4 && channels && out_dev, "NULL argument");
        CC_REQUIRE(n_channels >= 1 && n_channels <= CHAN_MAX, "1 .. 64 channels");
        for (int a = 0; a < 4; ++a) CC_REQUIRE(shape4[a] >= 1, "bad shape");
        ChanList cl;
        cl.n = (int32_t)n_channels;
        for (int64_t j = 0; j < n_channels; ++j) {
            CC_REQUIRE(channels[j] >= 0 && channels[j] < shape4[0], "channel out of range");
            cl.c[j] = (int32_t)channels[j];
        }
        const int64_t n = shape4[1] * shape4[2] * shape4[3];
        HIP_OK(hipSetDevice(c->device));
        switch (dtype) {
            case CC_DTYPE_FLOAT32: launch_channel_mean<float>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_FLOAT64: launch_channel_mean<double>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_UINT8: launch_channel_mean<uint8_t>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_INT8: launch_channel_mean<int8_t>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_UINT16: launch_channel_mean<uint16_t>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_INT16: launch_channel_mean<int16_t>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_UINT32: launch_channel_mean<uint32_t>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_INT32: launch_channel_mean<int32_t>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_UINT64: launch_channel_mean<uint64_t>(c, in_dev, n, cl, out_dev); break;
            case CC_DTYPE_INT64: launch_channel_mean<int64_t>(c, in_dev, n, cl, out_dev); break;
            default: CC_REQUIRE(false, "unsupported dtype");
        }
        sync(c);
    });
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// sigma_prefilter (block_components.py:161-163, threshold.py:151-153): per block
//   vu.normalize -> vu.apply_filter(., 'gaussianSmoothing', sigma) -> vu.normalize
// The reference filters each block on its own (no halo).  Its filter is fastfilters' or, when
// fastfilters is absent, vigra.filters.gaussianSmoothing (volume_utils.py:13-18, 80-94); neither
// library is available here, so the arithmetic below restates vigra's separable Gaussian
// (Kernel1D::initGaussian + separableConvolveMultiArray with BORDER_TREATMENT_REFLECT) in float32
// as oracle/oracle.py:gaussian_smooth_blocks does: taps g(x) = norm * exp(x^2 * (-0.5/s/s)) for
// x = -r..r, r = (int)(3 sigma + 0.5) (>= 1), divided by their sum; axes z, y, x in turn, each
// output sum_i k[x - i] * src[reflect(i)] accumulated from 0 in increasing i with separate float32
// multiply and add (no FMA: hipcc contracts a * b + c by default, so the sums run under
// `fp contract(off)`); float32 between the axes.  Parity with vigra / fastfilters is
// unpinned.  The second normalize is the labelling path's own.
//
// Layout: three streaming passes over the volume (z with the first normalize folded into the
// loads, then y, then x); each workgroup stages its lines with the halo (reflected inside the
// block) in LDS.  Traffic 8 B/voxel per pass (24 in all) + the block statistics read.
// ------------------------------------------------------------------------------------------
namespace cc {

constexpr int GS_RMAX = 64;
struct GaussTaps {
    int32_t r;
    float k[2 * GS_RMAX + 1];      // k[j] = tap of offset j - r
};
// tiles of one axis: outputs [a0, a0 + n) of the block segment [b0, b0 + w) along the axis
struct AxSeg {
    int32_t a0, b0, w, n;
    int32_t blk, pad[3];           // block index along the axis
};
struct NormP {                     // vu.normalize of one block: y = x - mn; if (m > 0) y = y / m
    float mn, m;
    int32_t nan, pad;
};
constexpr int GS_ZY_OUT = 64;      // outputs per z / y tile (x: 64 lanes)
constexpr int GS_X_OUT = 256;      // outputs per x tile (one row per wave)
constexpr int GS_U = 8;            // z / y lines loaded per wave before their LDS stores
constexpr int GS_UX = 5;           // x: (256 + 2 r) / 64 <= 5 loads per lane for r <= 32

__global__ void k_norm_params(int64_t nb, const u32* smin, const u32* smax, const u32* sflag, NormP* np) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    NormP p;
    p.mn = __uint_as_float(ord2f(smin[b]));
    const float mx = __uint_as_float(ord2f(smax[b]));
    // numpy: max(x - mn) is NaN when some x - mn is (x = mn = +-inf), else fl(mx - mn)
    p.m = isinf(p.mn) ? __uint_as_float(0x7FC00000u) : mx - p.mn;
    p.nan = (int32_t)(sflag[b] & 1u);
    p.pad = 0;
    np[b] = p;
}

__device__ __forceinline__ float gs_norm(float x, const NormP& p) {
    if (p.nan) return __uint_as_float(0x7FC00000u);
    float y = x - p.mn;
    if (p.m > 0.0f) y = y / p.m;
    return y;
}

__device__ __forceinline__ int gs_reflect(int rel, int w) {
    rel = rel < 0 ? -rel : rel;
    return rel >= w ? 2 * (w - 1) - rel : rel;
}

// z (AX = 0) or y (AX = 1) lines: 64 x-adjacent lines x GS_ZY_OUT outputs per workgroup, at a fixed
// y (AX = 0) or z (AX = 1).  NORM: the first pass normalizes every loaded value with its block's
// parameters.
template <int AX, bool NORM>
__global__ __launch_bounds__(256) void k_gauss_zy(const float* __restrict__ in, float* __restrict__ out, int64_t Z,
                                                  int64_t Y, int64_t X, int64_t by, int64_t bx, int nby, int nbx,
                                                  const AxSeg* __restrict__ segs, int64_t other, int64_t nxt,
                                                  const NormP* __restrict__ np, GaussTaps tp) {
    extern __shared__ float gbuf[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t id = blockIdx.x;
    const int64_t xt = id % nxt, rest = id / nxt;
    const int64_t o = rest % other, sg = rest / other;
    const AxSeg S = segs[sg];
    const int r = tp.r;
    const int64_t x = xt * 64 + lane;
    const bool xin = x < X;
    const int64_t xs = xin ? x : X - 1;
    NormP P{0.f, 0.f, 0, 0};
    if (NORM) {       // AX = 0: the segment's z block, the tile's y block, the lane's x block
        static_assert(!NORM || AX == 0, "the first (normalizing) pass runs along z");
        P = np[((int64_t)S.blk * nby + o / by) * nbx + xs / bx];
    }
    // GS_U lines in flight per wave (one load at a time, each waited for before the LDS store,
    // left the passes latency-bound at 2.7-4.2 TB/s)
    const int np_ = S.n + 2 * r;
    for (int p0 = wave; p0 < np_; p0 += 4 * GS_U) {
        float v[GS_U];
#pragma unroll
        for (int u = 0; u < GS_U; ++u) {
            const int p = p0 + 4 * u;
            const int64_t c = S.b0 + gs_reflect(S.a0 - S.b0 - r + (p < np_ ? p : np_ - 1), S.w);
            v[u] = in[AX == 0 ? (c * Y + o) * X + xs : (o * Y + c) * X + xs];
        }
#pragma unroll
        for (int u = 0; u < GS_U; ++u) {
            const int p = p0 + 4 * u;
            if (p < np_) gbuf[p * 64 + lane] = NORM ? gs_norm(v[u], P) : v[u];
        }
    }
    __syncthreads();
    if (!xin) return;
    for (int q = wave; q < S.n; q += 4) {
#pragma clang fp contract(off)
        float sum = 0.0f;
        for (int j = 0; j <= 2 * r; ++j) { const float t = tp.k[2 * r - j] * gbuf[(q + j) * 64 + lane]; sum = sum + t; }
        const int64_t c = S.a0 + q;
        out[AX == 0 ? (c * Y + o) * X + x : (o * Y + c) * X + x] = sum;
    }
}

// z (AX = 0) or y (AX = 1) lines without LDS: one wave per (segment, row o, 256 x-adjacent
// columns), a lane owns 4 columns (float4) and walks its segment's outputs with the 2R + 1 taps'
// window in registers (R <= GS_WIN_RMAX, X % 4 == 0); 8 outputs' new values are loaded before
// they are used (8 float4 loads in flight per lane).  Same sums, same order as k_gauss_zy.
constexpr int GS_WIN_RMAX = 8, GS_WIN_CH = 8;
template <int AX, int R, bool NORM>
__global__ __launch_bounds__(64) void k_gauss_win(const float* __restrict__ in, float* __restrict__ out, int64_t Y,
                                                  int64_t X, int64_t by, int64_t bx, int nby, int nbx,
                                                  const AxSeg* __restrict__ segs, int64_t other, int64_t nxc,
                                                  const NormP* __restrict__ np, GaussTaps tp) {
    const int lane = threadIdx.x;
    const int64_t id = blockIdx.x;
    const int64_t xc = id % nxc, rest = id / nxc;
    const int64_t o = rest % other, sg = rest / other;
    const AxSeg S = segs[sg];
    const int64_t x = (xc * 64 + lane) * 4;
    if (x >= X) return;
    NormP P[4];
    if (NORM) {
        static_assert(!NORM || AX == 0, "the first (normalizing) pass runs along z");
#pragma unroll
        for (int c = 0; c < 4; ++c) P[c] = np[((int64_t)S.blk * nby + o / by) * nbx + (x + c) / bx];
    }
    auto at = [&](int p) -> float4 {                 // p-th value of the window sequence (reflected)
        const int64_t cpos = S.b0 + gs_reflect(S.a0 - S.b0 - R + p, S.w);
        float4 v = *reinterpret_cast<const float4*>(in + (AX == 0 ? (cpos * Y + o) * X + x : (o * Y + cpos) * X + x));
        if (NORM) { v.x = gs_norm(v.x, P[0]); v.y = gs_norm(v.y, P[1]); v.z = gs_norm(v.z, P[2]); v.w = gs_norm(v.w, P[3]); }
        return v;
    };
    float4 w[2 * R + 1];
#pragma unroll
    for (int j = 0; j < 2 * R; ++j) w[j] = at(j);
    for (int q0 = 0; q0 < S.n; q0 += GS_WIN_CH) {
        float4 nv[GS_WIN_CH];
#pragma unroll
        for (int u = 0; u < GS_WIN_CH; ++u) nv[u] = q0 + u < S.n ? at(q0 + u + 2 * R) : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < GS_WIN_CH; ++u) {
            if (q0 + u >= S.n) break;
            w[2 * R] = nv[u];
            float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int j = 0; j <= 2 * R; ++j) {
#pragma clang fp contract(off)
                const float k = tp.k[2 * R - j];
                sum.x = sum.x + k * w[j].x; sum.y = sum.y + k * w[j].y;
                sum.z = sum.z + k * w[j].z; sum.w = sum.w + k * w[j].w;
            }
            const int64_t c = S.a0 + q0 + u;
            *reinterpret_cast<float4*>(out + (AX == 0 ? (c * Y + o) * X + x : (o * Y + c) * X + x)) = sum;
#pragma unroll
            for (int j = 0; j < 2 * R; ++j) w[j] = w[j + 1];
        }
    }
}

// x lines: one row per wave, GS_X_OUT outputs of one block segment per workgroup row
__global__ __launch_bounds__(256) void k_gauss_x(const float* __restrict__ in, float* __restrict__ out, int64_t rows,
                                                 int64_t X, const AxSeg* __restrict__ segs, GaussTaps tp) {
    extern __shared__ float gbuf[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = tp.r;
    const AxSeg S = segs[blockIdx.y];
    const int64_t row = (int64_t)blockIdx.x * 4 + wave;
    const bool ok = row < rows;                   // wave-uniform
    float* b = gbuf + wave * (GS_X_OUT + 2 * GS_RMAX);
    const float* src = in + (ok ? row : 0) * X;
    if (ok) {
        const int np_ = S.n + 2 * r;
        for (int p0 = lane; p0 < np_; p0 += 64 * GS_UX) {
            float v[GS_UX];
#pragma unroll
            for (int u = 0; u < GS_UX; ++u) {
                const int p = p0 + 64 * u;
                v[u] = src[S.b0 + gs_reflect(S.a0 - S.b0 - r + (p < np_ ? p : np_ - 1), S.w)];
            }
#pragma unroll
            for (int u = 0; u < GS_UX; ++u)
                if (p0 + 64 * u < np_) b[p0 + 64 * u] = v[u];
        }
    }
    __syncthreads();
    if (!ok) return;
    for (int q = lane; q < S.n; q += 64) {
#pragma clang fp contract(off)
        float sum = 0.0f;
        for (int j = 0; j <= 2 * r; ++j) { const float t = tp.k[2 * r - j] * b[q + j]; sum = sum + t; }
        out[row * X + S.a0 + q] = sum;
    }
}

// x lines with 16-B accesses (X and the x block a multiple of 4, 16-B aligned rows): the segment's
// own values are one float4 per lane into LDS (the 2r reflected halo values scalar), each lane
// computes 4 consecutive outputs and stores them as one float4.  Same sums, same order.
__global__ __launch_bounds__(256) void k_gauss_x4(const float* __restrict__ in, float* __restrict__ out, int64_t rows,
                                                  int64_t X, const AxSeg* __restrict__ segs, GaussTaps tp) {
    extern __shared__ float gbuf[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = tp.r;
    const AxSeg S = segs[blockIdx.y];
    const int64_t row = (int64_t)blockIdx.x * 4 + wave;
    const bool ok = row < rows;                   // wave-uniform
    float* b = gbuf + wave * (GS_X_OUT + 2 * GS_RMAX);
    const float* src = in + (ok ? row : 0) * X;
    if (ok) {
        if (4 * lane < S.n) {
            const float4 v = *reinterpret_cast<const float4*>(src + S.a0 + 4 * lane);
            b[r + 4 * lane] = v.x; b[r + 4 * lane + 1] = v.y; b[r + 4 * lane + 2] = v.z; b[r + 4 * lane + 3] = v.w;
        }
        for (int h = lane; h < 2 * r; h += 64) {                      // halo: p in [0, r) and [n + r, n + 2r)
            const int p = h < r ? h : S.n + h;
            b[p] = src[S.b0 + gs_reflect(S.a0 - S.b0 - r + p, S.w)];
        }
    }
    __syncthreads();
    if (!ok || 4 * lane >= S.n) return;
    float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* bq = b + 4 * lane;
    for (int j = 0; j <= 2 * r; ++j) {
#pragma clang fp contract(off)
        const float k = tp.k[2 * r - j];
        sum.x = sum.x + k * bq[j]; sum.y = sum.y + k * bq[j + 1];
        sum.z = sum.z + k * bq[j + 2]; sum.w = sum.w + k * bq[j + 3];
    }
    *reinterpret_cast<float4*>(out + row * X + S.a0 + 4 * lane) = sum;
}

}  // namespace cc

namespace cc {

// vigra Kernel1D<float>::initGaussian(sigma, 1.0) restated (see above): float arithmetic, expf
static int gauss_taps(double sigma, GaussTaps& t) {
    int radius = (int)(3.0 * sigma + 0.5);
    if (radius == 0) radius = 1;
    if (radius > GS_RMAX) return -1;
    const float s = (float)sigma;
    const float sigma2 = -0.5f / s / s;
    const float norm = (float)(1.0 / (std::sqrt(2.0 * M_PI) * (double)s));
    float sum = 0.0f;
    float x = -(float)radius;
    for (int i = 0; i <= 2 * radius; ++i, x += 1.0f) {
        const float x2 = x * x;
        t.k[i] = norm * std::exp(x2 * sigma2);
    }
    for (int i = 0; i <= 2 * radius; ++i) sum += t.k[i];
    const float f = 1.0f / sum;
    for (int i = 0; i <= 2 * radius; ++i) t.k[i] = t.k[i] * f;
    for (int i = 2 * radius + 1; i <= 2 * GS_RMAX; ++i) t.k[i] = 0.0f;
    t.r = radius;
    return radius;
}

// the register-window z and y passes for taps radius R
struct WinArgs {
    const float* in; float* A; float* B;
    int64_t Y, X, Z, by, bx;
    int nby, nbx;
    const AxSeg* sz; const AxSeg* sy;
    int64_t gz, gy, nxc;
    const NormP* np;
};
template <int R>
static void gauss_win_passes(cc_ctx* c, const WinArgs& w, const GaussTaps& tp) {
    hipStream_t s = cstream(c);
    launch(c, "k_gauss_z", [&] {
        k_gauss_win<0, R, true><<<(unsigned)w.gz, 64, 0, s>>>(w.in, w.A, w.Y, w.X, w.by, w.bx, w.nby, w.nbx, w.sz, w.Y,
                                                              w.nxc, w.np, tp);
    });
    launch(c, "k_gauss_y", [&] {
        k_gauss_win<1, R, false><<<(unsigned)w.gy, 64, 0, s>>>(w.A, w.B, w.Y, w.X, w.by, w.bx, w.nby, w.nbx, w.sy, w.Z,
                                                               w.nxc, w.np, tp);
    });
}

// tiles of `out_per` outputs inside each block segment of an axis of length n, blocks of bs
static void axis_segs(int64_t n, int64_t bs, int out_per, std::vector<AxSeg>& v) {
    for (int64_t b0 = 0, bi = 0; b0 < n; b0 += bs, ++bi) {
        const int64_t w = std::min(bs, n - b0);
        for (int64_t a0 = b0; a0 < b0 + w; a0 += out_per) {
            AxSeg S{};
            S.a0 = (int32_t)a0; S.b0 = (int32_t)b0; S.w = (int32_t)w;
            S.n = (int32_t)std::min<int64_t>(out_per, b0 + w - a0);
            S.blk = (int32_t)bi;
            v.push_back(S);
        }
    }
}

}  // namespace cc

extern "C" {

int cc_gaussian_taps(double sigma, float* taps, int cap) {
    CC_TRY({
        CC_REQUIRE(sigma > 0 && taps, "sigma must be > 0");
        GaussTaps t;
        const int r = gauss_taps(sigma, t);
        CC_REQUIRE(r > 0, "sigma too large (kernel radius > 64)");
        CC_REQUIRE(cap >= 2 * r + 1, "taps buffer too small");
        for (int i = 0; i <= 2 * r; ++i) taps[i] = t.k[i];
        return r;
    });
}

int cc_gaussian_smooth_blocks(cc_ctx* c, const float* in, const int64_t shape[3], const int64_t block_shape[3],
                              double sigma, float* out) {
    CC_TRY({
        CC_REQUIRE(c && in && out && shape && block_shape, "NULL argument");
        CC_REQUIRE(sigma > 0, "sigma must be > 0");
        GaussTaps tp;
        const int r = gauss_taps(sigma, tp);
        CC_REQUIRE(r > 0, "sigma too large (kernel radius > 64)");
        for (int a = 0; a < 3; ++a) {
            CC_REQUIRE(shape[a] >= 1 && block_shape[a] >= 1, "bad shape / block_shape");
            CC_REQUIRE(shape[a] < (1ll << 31), "axis too long");
            // vigra convolveLine: "kernel longer than line" unless every line (block extent) > r
            const int64_t last = shape[a] - (shape[a] - 1) / block_shape[a] * block_shape[a];
            CC_REQUIRE(std::min(block_shape[a], shape[a]) > r && last > r,
                       "sigma_prefilter: kernel longer than a block line (block extent <= 3 sigma)");
        }
        HIP_OK(hipSetDevice(c->device));
        const int64_t Z = shape[0], Y = shape[1], X = shape[2], n = Z * Y * X;
        hipStream_t s = cstream(c);
        // block statistics (ordered min / max, NaN flag) -> normalize parameters
        RunState& st = state(c);
        st = RunState();
        st.hg = make_geom(shape, block_shape, 0);
        upload_geom(c, st.hg);
        Geom& g = st.hg.g;
        const int64_t nt = g.n_tiles, nb = g.n_blocks;
        c->bstat.ensure(nb * 3 * sizeof(u32));
        u32* smin = c->bstat.as<u32>();
        u32* smax = smin + nb;
        u32* sflag = smax + nb;
        HIP_OK(hipMemsetAsync(smin, 0xFF, nb * sizeof(u32), s));
        HIP_OK(hipMemsetAsync(smax, 0x00, 2 * nb * sizeof(u32), s));
        launch(c, "k_block_stats", [&] { k_block_stats<<<(unsigned)nt, NTHREADS, 0, s>>>(g, in, smin, smax, sflag); });
        // register-window z / y passes (k_gauss_win) when the taps fit and rows are 16-B aligned;
        // else the LDS-staged k_gauss_zy
        const bool win = r <= GS_WIN_RMAX && X % 4 == 0 && ((uintptr_t)in | (uintptr_t)out) % 16 == 0;
        std::vector<AxSeg> sz, sy, sx;
        axis_segs(Z, block_shape[0], win ? 64 : GS_ZY_OUT, sz);
        axis_segs(Y, block_shape[1], win ? 128 : GS_ZY_OUT, sy);
        axis_segs(X, block_shape[2], GS_X_OUT, sx);
        CC_REQUIRE(sx.size() < 65536, "too many x segments");
        const size_t nseg = sz.size() + sy.size() + sx.size();
        c->gs_tab.ensure(nseg * sizeof(AxSeg) + nb * sizeof(NormP));
        AxSeg* dseg = c->gs_tab.as<AxSeg>();
        NormP* np = (NormP*)(dseg + nseg);
        static_assert(sizeof(AxSeg) % sizeof(int32_t) == 0, "AxSeg as int32 words");
        c->h_gs.resize(nseg * sizeof(AxSeg) / sizeof(int32_t));    // kept alive until the stream has read it
        {
            char* h = reinterpret_cast<char*>(c->h_gs.data());
            std::memcpy(h, sz.data(), sz.size() * sizeof(AxSeg));
            std::memcpy(h + sz.size() * sizeof(AxSeg), sy.data(), sy.size() * sizeof(AxSeg));
            std::memcpy(h + (sz.size() + sy.size()) * sizeof(AxSeg), sx.data(), sx.size() * sizeof(AxSeg));
        }
        HIP_OK(hipMemcpyAsync(dseg, c->h_gs.data(), nseg * sizeof(AxSeg), hipMemcpyHostToDevice, s));
        launch(c, "k_norm_params", [&] { k_norm_params<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(nb, smin, smax, sflag, np); });
        c->gs1.ensure(n * sizeof(float));
        c->gs2.ensure(n * sizeof(float));
        float* A = c->gs1.as<float>();
        float* B = c->gs2.as<float>();
        const int nby = (int)g.nb[1], nbx = (int)g.nb[2];
        if (win) {
            const int64_t nxc = (X / 4 + 63) / 64;
            const int64_t gz = (int64_t)sz.size() * Y * nxc, gy = (int64_t)sy.size() * Z * nxc;
            CC_REQUIRE(gz < (1ll << 31) && gy < (1ll << 31), "volume too large for the z / y pass grid");
            const WinArgs wa{in, A, B, Y, X, Z, block_shape[1], block_shape[2], nby, nbx, dseg,
                             dseg + sz.size(), gz, gy, nxc, np};
            switch (r) {
                case 1: gauss_win_passes<1>(c, wa, tp); break;
                case 2: gauss_win_passes<2>(c, wa, tp); break;
                case 3: gauss_win_passes<3>(c, wa, tp); break;
                case 4: gauss_win_passes<4>(c, wa, tp); break;
                case 5: gauss_win_passes<5>(c, wa, tp); break;
                case 6: gauss_win_passes<6>(c, wa, tp); break;
                case 7: gauss_win_passes<7>(c, wa, tp); break;
                default: gauss_win_passes<8>(c, wa, tp); break;
            }
        } else {
            const int64_t nxt = (X + 63) / 64;
            const size_t lds_zy = (size_t)(GS_ZY_OUT + 2 * r) * 64 * sizeof(float);
            const int64_t grid_z = (int64_t)sz.size() * Y * nxt, grid_y = (int64_t)sy.size() * Z * nxt;
            CC_REQUIRE(grid_z < (1ll << 31) && grid_y < (1ll << 31), "volume too large for the z / y pass grid");
            launch(c, "k_gauss_z", [&] {
                k_gauss_zy<0, true><<<(unsigned)grid_z, 256, lds_zy, s>>>(in, A, Z, Y, X, block_shape[1], block_shape[2],
                                                                          nby, nbx, dseg, Y, nxt, np, tp);
            });
            launch(c, "k_gauss_y", [&] {
                k_gauss_zy<1, false><<<(unsigned)grid_y, 256, lds_zy, s>>>(A, B, Z, Y, X, block_shape[1], block_shape[2],
                                                                           nby, nbx, dseg + sz.size(), Z, nxt, np, tp);
            });
        }
        {
            const int64_t rows = Z * Y, gx = (rows + 3) / 4;
            CC_REQUIRE(gx < (1ll << 31), "volume too large for the x pass grid");
            const size_t lds_x = (size_t)4 * (GS_X_OUT + 2 * GS_RMAX) * sizeof(float);
            const bool x4 = X % 4 == 0 && block_shape[2] % 4 == 0 && ((uintptr_t)out % 16) == 0;
            launch(c, "k_gauss_x", [&] {
                if (x4)
                    k_gauss_x4<<<dim3((unsigned)gx, (unsigned)sx.size()), 256, lds_x, s>>>(B, out, rows, X,
                                                                                        dseg + sz.size() + sy.size(), tp);
                else
                    k_gauss_x<<<dim3((unsigned)gx, (unsigned)sx.size()), 256, lds_x, s>>>(B, out, rows, X,
                                                                                       dseg + sz.size() + sy.size(), tp);
            });
        }
        sync(c);
        st.stage = 0;
    });
}

}  // extern "C"
