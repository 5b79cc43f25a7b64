// cc_prims.hip -- the library's own device primitives: exclusive scan, LSD radix sort (keys or
// key/value pairs, any bit range), select-unique and select-flagged.
//
// Why not hipcub / rocprim: their dispatch instantiates every tuning configuration of every
// algorithm used (944 of the code object's 1041 kernels, 1.3 MB of kernel metadata), and the HIP
// runtime loads the whole code object on the library's first launch: 25-27 ms that every
// one-shot drop-in job (one process, one call) paid before its first kernel ran
// (profiles/r03_c1_cold.json, r03_cold_probe.json).  Every sort here is small (root lists of
// the fallback path, seam pairs, the distinct ids of relabel): a few hundred thousand keys, far
// from where onesweep tuning matters.
//
// Layout: 256-thread workgroups (4 waves of 64).  Radix sort: 8-bit digits, per pass
//   k_rs_hist    per-workgroup digit histograms of a 2048-key tile, digit-major [d][wg]
//   scan         exclusive scan of the 256 x nwg histogram (= each tile's first slot per digit)
//   k_rs_scatter the tile in 8 rounds of 256 keys in index order; a key's rank among equal
//                digits of its wave from 8 ballots, the waves' counts prefixed per digit in LDS
//                (stable: rounds, waves and lanes are visited in index order)
// Scan: tiles of 4096 (16 per thread): per-tile sums -> one-workgroup scan of the sums ->
// each tile rescanned with its carry.
namespace cc {
namespace prims {
// one copy of the primitives per translation unit of the library (cc_lib.hip, cc_aux.hip): the
// inline namespace keeps their kernels' symbols apart
#ifndef CC_PRIMS_NS
#define CC_PRIMS_NS core
#endif
inline namespace CC_PRIMS_NS {

constexpr int PT = 256;                 // threads per workgroup
constexpr int PW = PT / 64;             // waves
constexpr int SC_ITEMS = 16;
constexpr int SC_TILE = PT * SC_ITEMS;  // scan tile
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = PT * RS_ITEMS;  // radix-sort tile
constexpr int RADIX = 256;
static_assert(PT == RADIX, "k_rs_scatter maps one thread to each digit");

struct NoVal {};

template <class T>
__device__ __forceinline__ T shfl_up_t(T x, int o) {
    if constexpr (sizeof(T) == 8) {
        const u32 lo = (u32)__shfl_up((int)(u32)x, o, 64), hi = (u32)__shfl_up((int)(u32)((u64)x >> 32), o, 64);
        return (T)(((u64)hi << 32) | lo);
    } else {
        return (T)__shfl_up((int)x, o, 64);
    }
}

// exclusive scan of one value per thread over the workgroup; *total = the sum
template <class T>
__device__ __forceinline__ T wg_excl_scan(T v, T* sh, T* total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    T x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = shfl_up_t(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    T base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < PW; ++w) {
        const T s = sh[w];
        if (w < wave) base += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// per-tile sums
template <class T>
__global__ __launch_bounds__(PT) void k_scan_reduce(const T* __restrict__ in, int64_t n, T* part) {
    __shared__ T sh[PW];
    const int64_t base = (int64_t)blockIdx.x * SC_TILE;
    T s = 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const int64_t i = base + j * PT + threadIdx.x;
        if (i < n) s += in[i];
    }
    T tot;
    wg_excl_scan(s, sh, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// exclusive scan of a tile, starting from carry (part[wg], or 0); in == out allowed
template <class T>
__device__ __forceinline__ T scan_tile(const T* in, T* out, int64_t base, int64_t n, T carry, T* tile, T* sh) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const int64_t i = base + j * PT + tid;
        tile[j * PT + tid] = i < n ? in[i] : (T)0;
    }
    __syncthreads();
    T v[SC_ITEMS], s = 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) { v[j] = tile[tid * SC_ITEMS + j]; s += v[j]; }
    T tot;
    T run = carry + wg_excl_scan(s, sh, &tot);
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) { tile[tid * SC_ITEMS + j] = run; run += v[j]; }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const int64_t i = base + j * PT + tid;
        if (i < n) out[i] = tile[j * PT + tid];
    }
    __syncthreads();
    return carry + tot;
}

template <class T>
__global__ __launch_bounds__(PT) void k_scan_down(const T* in, T* out, int64_t n, const T* __restrict__ part) {
    __shared__ T tile[SC_TILE];
    __shared__ T sh[PW];
    scan_tile(in, out, (int64_t)blockIdx.x * SC_TILE, n, part ? part[blockIdx.x] : (T)0, tile, sh);
}

// one workgroup: exclusive scan of in[0, m) into out (the tile sums, in place; or a whole short
// array: one launch instead of three)
template <class T>
__global__ __launch_bounds__(PT) void k_scan_single(const T* in, T* out, int64_t m) {
    __shared__ T tile[SC_TILE];
    __shared__ T sh[PW];
    T carry = 0;
    for (int64_t b = 0; b < m; b += SC_TILE) carry = scan_tile(in, out, b, m, carry, tile, sh);
}
constexpr int64_t SC_SINGLE_MAX = 2 * SC_TILE;      // arrays up to this length: one workgroup

template <class K>
__global__ __launch_bounds__(PT) void k_rs_hist(const K* __restrict__ kin, int64_t n, int shift, u32 mask, int64_t nwg,
                                                u32* hist) {
    __shared__ u32 h[RADIX];
    const int tid = threadIdx.x;
    h[tid] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll
    for (int j = 0; j < RS_ITEMS; ++j) {
        const int64_t i = base + j * PT + tid;
        if (i < n) atomicAdd(&h[(u32)(kin[i] >> shift) & mask], 1u);
    }
    __syncthreads();
    hist[(int64_t)tid * nwg + blockIdx.x] = h[tid];
}

template <class K, class V>
__global__ __launch_bounds__(PT) void k_rs_scatter(const K* __restrict__ kin, K* __restrict__ kout,
                                                   const V* __restrict__ vin, V* __restrict__ vout, int64_t n,
                                                   int shift, u32 mask, int64_t nwg, const u32* __restrict__ hoff) {
    constexpr bool HASV = !std::is_same<V, NoVal>::value;
    __shared__ u32 run[RADIX];
    __shared__ u32 wc[PW][RADIX];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    run[tid] = hoff[(int64_t)tid * nwg + blockIdx.x];
    const int64_t base = (int64_t)blockIdx.x * RS_TILE;
    const u64 lt = (1ull << lane) - 1;
    for (int j = 0; j < RS_ITEMS; ++j) {
        const int64_t i = base + j * PT + tid;
        const bool valid = i < n;
        const K k = valid ? kin[i] : (K)0;
        V v{};
        if constexpr (HASV) { if (valid) v = vin[i]; }
        const u32 d = (u32)(k >> shift) & mask;
        u64 peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const u64 bb = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? bb : ~bb;
        }
#pragma unroll
        for (int q = 0; q < PW; ++q) wc[q][tid] = 0;
        __syncthreads();
        const u32 rank = (u32)__popcll(peers & lt);
        if (valid && rank == 0) wc[w][d] = (u32)__popcll(peers);
        __syncthreads();
        {
            u32 r = run[tid];
#pragma unroll
            for (int q = 0; q < PW; ++q) { const u32 c = wc[q][tid]; wc[q][tid] = r; r += c; }
            run[tid] = r;
        }
        __syncthreads();
        if (valid) {
            const u32 pos = wc[w][d] + rank;
            kout[pos] = k;
            if constexpr (HASV) vout[pos] = v;
        }
        __syncthreads();
    }
}

template <class T>
__global__ void k_flag_unique(const T* __restrict__ in, int64_t n, u32* f) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) f[i] = (i == 0 || in[i] != in[i - 1]) ? 1u : 0u;
}
__global__ void k_flag_u8(const u8* __restrict__ fl, int64_t n, u32* f) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) f[i] = fl[i] ? 1u : 0u;
}
// keep element i when its flag is set (UNIQUE: flag recomputed from the sorted input); pos =
// exclusive scan of the flags; nsel = the number kept
template <class T, bool UNIQUE>
__global__ void k_compact(const T* __restrict__ in, const u8* __restrict__ fl, const u32* __restrict__ pos, int64_t n,
                          T* __restrict__ out, int* nsel) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool keep = UNIQUE ? (i == 0 || in[i] != in[i - 1]) : fl[i] != 0;
    if (keep) out[pos[i]] = in[i];
    if (i == n - 1) *nsel = (int)(pos[i] + (keep ? 1u : 0u));
}

// ---- one-workgroup sort + unique of up to SU_MAX u64 keys in LDS ----------------------------
// The seam schedule sorts a few hundred to a few thousand keys per slab (unique seam pairs, the
// distinct ids of all seams); the multi-kernel sort is launch-bound there (3 kernels per 8-bit
// pass), so one 1024-thread workgroup does it all in LDS: the key bound (largest key) -> passes,
// per pass a digit histogram (LDS atomics), its scan, and the stable scatter in rounds of 1024
// keys (ranks among equal digits from 8 ballots per wave, wave counts prefixed per digit), then
// the unique keys compacted in order.
constexpr int SU_T = 1024, SU_W = SU_T / 64, SU_MAX = 8192;
struct SortSmallLDS {
    u64 a[SU_MAX], b[SU_MAX];
    u32 wc[SU_W][RADIX];
    u32 run[RADIX];
    u64 red[SU_W];
    u32 sh[SU_W];
};

// sorts L.a[0, n) (result in *res, which is L.a or L.b), returns nothing; keys < 2^bits
__device__ __forceinline__ u64* su_sort(SortSmallLDS& L, int n, int bits) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 lt = (1ull << lane) - 1;
    u64* src = L.a;
    u64* dst = L.b;
    for (int shift = 0; shift < bits; shift += 8) {
        const u32 mask = (1u << min(8, bits - shift)) - 1;
        if (tid < RADIX) L.run[tid] = 0;
        __syncthreads();
        for (int i = tid; i < n; i += SU_T) atomicAdd(&L.run[(u32)(src[i] >> shift) & mask], 1u);
        __syncthreads();
        if (w == 0) {                              // exclusive scan of the 256 digit counts
            u32 v[4], sum = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) { v[j] = L.run[4 * lane + j]; sum += v[j]; }
            u32 x = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) { const u32 y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
            u32 r = x - sum;
#pragma unroll
            for (int j = 0; j < 4; ++j) { L.run[4 * lane + j] = r; r += v[j]; }
        }
        __syncthreads();
        for (int r0 = 0; r0 < n; r0 += SU_T) {
            const int i = r0 + tid;
            const bool valid = i < n;
            const u64 k = valid ? src[i] : 0ull;
            const u32 d = (u32)(k >> shift) & mask;
            u64 peers = __ballot(valid);
#pragma unroll
            for (int bb = 0; bb < 8; ++bb) {
                const u64 q = __ballot((d >> bb) & 1u);
                peers &= ((d >> bb) & 1u) ? q : ~q;
            }
            for (int j = tid; j < SU_W * RADIX; j += SU_T) (&L.wc[0][0])[j] = 0;
            __syncthreads();
            const u32 rank = (u32)__popcll(peers & lt);
            if (valid && rank == 0) L.wc[w][d] = (u32)__popcll(peers);
            __syncthreads();
            if (tid < RADIX) {
                u32 r = L.run[tid];
                for (int q = 0; q < SU_W; ++q) { const u32 c = L.wc[q][tid]; L.wc[q][tid] = r; r += c; }
                L.run[tid] = r;
            }
            __syncthreads();
            if (valid) dst[L.wc[w][d] + rank] = k;
            __syncthreads();
        }
        u64* t = src; src = dst; dst = t;
    }
    return src;
}

// largest of L.a[0, n) over the workgroup
__device__ __forceinline__ u64 su_max(SortSmallLDS& L, int n) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u64 m = 0;
    for (int i = tid; i < n; i += SU_T) m = L.a[i] > m ? L.a[i] : m;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { const u64 t = __shfl_xor(m, o, 64); m = t > m ? t : m; }
    if (lane == 0) L.red[w] = m;
    __syncthreads();
    m = 0;
    for (int q = 0; q < SU_W; ++q) m = L.red[q] > m ? L.red[q] : m;
    __syncthreads();
    return m;
}

// unique keys of the sorted k[0, n) in order: emit(position, key); returns the count
template <class EMIT>
__device__ __forceinline__ int su_unique(SortSmallLDS& L, const u64* k, int n, EMIT&& emit) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int carry = 0;
    for (int r0 = 0; r0 < n; r0 += SU_T) {
        const int i = r0 + tid;
        const u32 f = (i < n && (i == 0 || k[i] != k[i - 1])) ? 1u : 0u;
        const u64 bal = __ballot(f);
        if (lane == 0) L.sh[w] = (u32)__popcll(bal);
        __syncthreads();
        u32 before = 0, tot = 0;
        for (int q = 0; q < SU_W; ++q) { const u32 c = L.sh[q]; before += q < w ? c : 0u; tot += c; }
        if (f) emit(carry + (int)(before + (u32)__popcll(bal & ((1ull << lane) - 1))), k[i]);
        carry += (int)tot;
        __syncthreads();
    }
    return carry;
}

// sorted distinct (a, b) pairs of pa / pb [0, n) (n <= SU_MAX, every id < 2^nb) -> pairs
// ([m][2], at most cap written; qa / qb, if given, get them too), *nsel = m
__global__ __launch_bounds__(SU_T) void k_pairs_sort_unique_small(const u64* __restrict__ pa, const u64* __restrict__ pb,
                                                                  int n, int nb, u64* pairs, int64_t cap, u64* qa,
                                                                  u64* qb, int* nsel) {
    __shared__ SortSmallLDS L;
    for (int i = threadIdx.x; i < n; i += SU_T) L.a[i] = (pa[i] << nb) | pb[i];
    __syncthreads();
    const u64* k = su_sort(L, n, 2 * nb);
    const u64 lo = (1ull << nb) - 1;
    const int m = su_unique(L, k, n, [&](int pos, u64 v) {
        const u64 a = v >> nb, b = v & lo;
        if (pairs && pos < cap) { pairs[2 * pos] = a; pairs[2 * pos + 1] = b; }
        if (qa) { qa[pos] = a; qb[pos] = b; }
    });
    if (threadIdx.x == 0) *nsel = m;
}

// The seam map of cc_shard_finish in one workgroup (2 n <= SU_MAX ids; the multi-kernel form is
// phase_map's: sort, unique, pairs -> indices, iota, unions, resolve, map = 7+ launches): U = the
// sorted distinct ids of the n pairs, a union-find over indices into U in LDS (the smaller index
// wins, so a component's root is its smallest id), V[i] = U[root(i)]; *m_out = |U|.
__global__ __launch_bounds__(SU_T) void k_seam_map_small(const u64* __restrict__ pairs, int n, u64* U, u64* V,
                                                         int* m_out) {
    __shared__ SortSmallLDS L;
    const int n2 = 2 * n, tid = threadIdx.x;
    for (int i = tid; i < n2; i += SU_T) L.a[i] = pairs[i];
    __syncthreads();
    const u64 mx = su_max(L, n2);
    int bits = 0;
    while (bits < 64 && (mx >> bits)) ++bits;
    u64* k = su_sort(L, n2, bits);
    u64* ub = k == L.a ? L.b : L.a;                  // distinct ids; k's buffer becomes the parents
    const int m = su_unique(L, k, n2, [&](int pos, u64 v) { ub[pos] = v; U[pos] = v; });
    __syncthreads();
    u32* par = reinterpret_cast<u32*>(k);
    for (int i = tid; i < m; i += SU_T) par[i] = (u32)i;
    __syncthreads();
    auto index_of = [&](u64 v) -> u32 {              // v is in ub[0, m)
        int lo = 0, hi = m - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (ub[mid] < v) lo = mid + 1; else hi = mid;
        }
        return (u32)lo;
    };
    for (int i = tid; i < n; i += SU_T) lunion(par, index_of(pairs[2 * i]), index_of(pairs[2 * i + 1]));
    __syncthreads();
    for (int i = tid; i < m; i += SU_T) V[i] = ub[lfind_ro(as_lds(par), (u32)i)];
    if (tid == 0) *m_out = m;
}

// ---- host side: temporaries carved from one caller buffer (the context's cub_tmp) ----------
struct Carve {
    char* p;
    size_t off = 0;
    template <class T>
    T* take(int64_t n) {
        off = (off + 255) & ~(size_t)255;
        T* r = (T*)(p ? p + off : nullptr);
        off += (size_t)std::max<int64_t>(n, 1) * sizeof(T);
        return r;
    }
};

inline unsigned nblk(int64_t n, int64_t per) { return (unsigned)std::max<int64_t>(1, (n + per - 1) / per); }

template <class T>
size_t scan_tmp_bytes(int64_t n) {
    Carve cv{nullptr};
    if (n > SC_SINGLE_MAX) cv.take<T>((n + SC_TILE - 1) / SC_TILE);
    return cv.off + 256;
}

// exclusive prefix sum of in[0, n) into out (in == out allowed)
template <class T>
void scan_excl(const T* in, T* out, int64_t n, char* tmp, hipStream_t s) {
    if (n <= 0) return;
    if (n <= SC_SINGLE_MAX) {
        k_scan_single<T><<<1, PT, 0, s>>>(in, out, n);
    } else {
        Carve cv{tmp};
        const int64_t m = (n + SC_TILE - 1) / SC_TILE;
        T* part = cv.take<T>(m);
        k_scan_reduce<T><<<(unsigned)m, PT, 0, s>>>(in, n, part);
        k_scan_single<T><<<1, PT, 0, s>>>(part, part, m);
        k_scan_down<T><<<(unsigned)m, PT, 0, s>>>(in, out, n, part);
    }
    HIP_OK(hipGetLastError());
}

template <class K, class V>
size_t sort_tmp_bytes(int64_t n) {
    Carve cv{nullptr};
    const int64_t nwg = (n + RS_TILE - 1) / RS_TILE;
    cv.take<K>(n);
    if constexpr (!std::is_same<V, NoVal>::value) cv.take<V>(n);
    cv.take<u32>(RADIX * nwg);
    const size_t a = cv.off;
    return a + scan_tmp_bytes<u32>(RADIX * nwg) + 256;
}

// stable LSD radix sort of keys bits [b0, b1) (values follow); kin / vin are left untouched
template <class K, class V>
void sort_pairs(const K* kin, K* kout, const V* vin, V* vout, int64_t n, int b0, int b1, DevBuf& tmpbuf, hipStream_t s) {
    constexpr bool HASV = !std::is_same<V, NoVal>::value;
    if (n <= 0) return;
    CC_REQUIRE(n < (1LL << 31), "too many keys for one sort");
    tmpbuf.ensure(sort_tmp_bytes<K, V>(n));
    Carve cv{(char*)tmpbuf.p};
    const int64_t nwg = (n + RS_TILE - 1) / RS_TILE;
    K* kalt = cv.take<K>(n);
    V* valt = HASV ? cv.take<V>(n) : nullptr;
    u32* hist = cv.take<u32>(RADIX * nwg);
    char* stmp = (char*)tmpbuf.p + ((cv.off + 255) & ~(size_t)255);
    const int passes = b1 > b0 ? (b1 - b0 + 7) / 8 : 0;
    if (passes == 0) {
        HIP_OK(hipMemcpyAsync(kout, kin, n * sizeof(K), hipMemcpyDeviceToDevice, s));
        if constexpr (HASV) HIP_OK(hipMemcpyAsync(vout, vin, n * sizeof(V), hipMemcpyDeviceToDevice, s));
        return;
    }
    const K* ks = kin;
    const V* vs = vin;
    for (int p = 0; p < passes; ++p) {
        K* kd = ((passes - 1 - p) % 2 == 0) ? kout : kalt;
        V* vd = ((passes - 1 - p) % 2 == 0) ? vout : valt;
        const int shift = b0 + 8 * p;
        const int bits = std::min(8, b1 - shift);
        const u32 mask = (1u << bits) - 1;
        k_rs_hist<K><<<(unsigned)nwg, PT, 0, s>>>(ks, n, shift, mask, nwg, hist);
        HIP_OK(hipGetLastError());
        scan_excl<u32>(hist, hist, RADIX * nwg, stmp, s);
        k_rs_scatter<K, V><<<(unsigned)nwg, PT, 0, s>>>(ks, kd, vs, vd, n, shift, mask, nwg, hist);
        HIP_OK(hipGetLastError());
        ks = kd;
        vs = vd;
    }
}

template <class K>
void sort_keys(const K* kin, K* kout, int64_t n, int b0, int b1, DevBuf& tmp, hipStream_t s) {
    sort_pairs<K, NoVal>(kin, kout, nullptr, nullptr, n, b0, b1, tmp, s);
}

// out = the first element of every run of equal elements of the sorted in[0, n); *nsel (device) = count
template <class T>
void select_unique(const T* in, T* out, int* nsel, int64_t n, DevBuf& tmpbuf, hipStream_t s) {
    if (n <= 0) { HIP_OK(hipMemsetAsync(nsel, 0, sizeof(int), s)); return; }
    Carve cv{nullptr};
    cv.take<u32>(n);
    tmpbuf.ensure(cv.off + scan_tmp_bytes<u32>(n) + 256);
    Carve c2{(char*)tmpbuf.p};
    u32* pos = c2.take<u32>(n);
    char* stmp = (char*)tmpbuf.p + ((c2.off + 255) & ~(size_t)255);
    k_flag_unique<T><<<nblk(n, 256), 256, 0, s>>>(in, n, pos);
    HIP_OK(hipGetLastError());
    scan_excl<u32>(pos, pos, n, stmp, s);
    k_compact<T, true><<<nblk(n, 256), 256, 0, s>>>(in, nullptr, pos, n, out, nsel);
    HIP_OK(hipGetLastError());
}

// out = in[i] for every i with flags[i] != 0, in order; *nsel (device) = count
template <class T>
void select_flagged(const T* in, const u8* flags, T* out, int* nsel, int64_t n, DevBuf& tmpbuf, hipStream_t s) {
    if (n <= 0) { HIP_OK(hipMemsetAsync(nsel, 0, sizeof(int), s)); return; }
    Carve cv{nullptr};
    cv.take<u32>(n);
    tmpbuf.ensure(cv.off + scan_tmp_bytes<u32>(n) + 256);
    Carve c2{(char*)tmpbuf.p};
    u32* pos = c2.take<u32>(n);
    char* stmp = (char*)tmpbuf.p + ((c2.off + 255) & ~(size_t)255);
    k_flag_u8<<<nblk(n, 256), 256, 0, s>>>(flags, n, pos);
    HIP_OK(hipGetLastError());
    scan_excl<u32>(pos, pos, n, stmp, s);
    k_compact<T, false><<<nblk(n, 256), 256, 0, s>>>(in, flags, pos, n, out, nsel);
    HIP_OK(hipGetLastError());
}

// exclusive scan with the temporaries in tmpbuf
template <class T>
void scan_excl(const T* in, T* out, int64_t n, DevBuf& tmpbuf, hipStream_t s) {
    tmpbuf.ensure(scan_tmp_bytes<T>(n));
    scan_excl<T>(in, out, n, (char*)tmpbuf.p, s);
}

}  // namespace CC_PRIMS_NS
}  // namespace prims
}  // namespace cc
