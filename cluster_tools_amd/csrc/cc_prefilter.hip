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
    hipStream_t s = c->stream;
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
