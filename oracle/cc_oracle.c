/*
 * cc_oracle.c -- CPU restatement of cluster_tools' ThresholdedComponentsWorkflow
 * (reference v0.3.3).  TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke()
 * and the cpu_baseline leg of bench.py load this library.  It is the checker and
 * the side-by-side CPU baseline ("port"), never the product path.
 *
 * Parity pin: tests/test_oracle_golden.py checks this file against the golden
 * vectors produced by the reference's own job functions (tests/golden/make_golden.py).
 *
 * Stage by stage (all citations relative to /root/reference):
 *   1. block_components  cluster_tools/thresholded_components/block_components.py:143-233,236-291
 *        normalize        cluster_tools/utils/volume_utils.py:98-105
 *        threshold        block_components.py:166-173 (threshold cast to float32)
 *        mask             block_components.py:194-197,225
 *        label            skimage.morphology.label(input_) (block_components.py:179): 26-connectivity,
 *                         labels 1..n in raster first-occurrence order (scikit-image 0.18.3, not vendored)
 *        value            n+1, or 0 for a block without foreground (block_components.py:175-182)
 *   2. merge_offsets     merge_offsets.py:104-120 (exclusive cumsum of values, n_labels = off[-1]+v[-1]+1)
 *   3. block_faces       block_faces.py:87-137 + volume_utils.py:187-236 (upper neighbours,
 *                        1-voxel face slabs, pairs where both labels != 0, + block offsets)
 *   4. merge_assignments merge_assignments.py:105-130 (union-find over arange(n_labels)).
 *                        nifty's boost_ufd is not vendored; we use the min-id representative,
 *                        which gives the same partition.  The empty-job quirk
 *                        (merge_assignments.py:115-123 with block_faces.py:169-176) is emulated
 *                        when quirk_n_jobs > 0.
 *   5. write             cluster_tools/write/write.py:185-202 (seg[seg!=0] += off; seg = lut[seg]),
 *                        maxId = lut.max() (write.py:281-289).
 *
 * Threading mirrors target='local': n_jobs workers, job j owns block_list[j::n_jobs]
 * (cluster_tools/cluster_tasks.py:331).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math: the f32 arithmetic
 * must be IEEE like numpy's).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------- */
/* synthetic boundary map (same definition as oracle/synth.py)               */
/* ------------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

#define PITCH 32
#define NOISE_SALT 0x5851F42D4C957F2DULL

static inline int64_t fdiv(int64_t a, int64_t b) { /* floor division, b > 0 */
    int64_t q = a / b;
    return (a % b != 0 && a < 0) ? q - 1 : q;
}

/* q, and in *dither the 16-bit dither of the continuous variant (bits 16..31 of the noise hash) */
static uint8_t boundary_q_at(int64_t z, int64_t y, int64_t x, uint64_t seed, uint32_t* dither) {
    int64_t cz = fdiv(z, PITCH), cy = fdiv(y, PITCH), cx = fdiv(x, PITCH);
    int64_t d1 = (int64_t)1 << 62, d2 = (int64_t)1 << 62;
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                int64_t nz = cz + dz, ny = cy + dy, nx = cx + dx;
                uint64_t key = ((uint64_t)(nz + 1) << 42) | ((uint64_t)(ny + 1) << 21) | (uint64_t)(nx + 1);
                uint64_t h = splitmix64(seed ^ key);
                int64_t sz = nz * PITCH + (int64_t)(h & 31);
                int64_t sy = ny * PITCH + (int64_t)((h >> 5) & 31);
                int64_t sx = nx * PITCH + (int64_t)((h >> 10) & 31);
                int64_t d = (z - sz) * (z - sz) + (y - sy) * (y - sy) + (x - sx) * (x - sx);
                if (d < d1) { d2 = d1; d1 = d; }
                else if (d < d2) { d2 = d; }
            }
    int64_t m = 255 - (d2 - d1);
    if (m < 0) m = 0;
    uint64_t vkey = ((uint64_t)z << 42) | ((uint64_t)y << 21) | (uint64_t)x;
    uint64_t nh = splitmix64((seed + NOISE_SALT) ^ vkey);
    int64_t n = (int64_t)(nh % 33) - 16;
    *dither = (uint32_t)((nh >> 16) & 0xFFFF);
    int64_t q = m + n;
    if (q < 0) q = 0;
    if (q > 255) q = 255;
    return (uint8_t)q;
}

typedef struct {
    float* out; uint8_t* outq;
    int64_t Z, Y, X, oz, oy, ox; uint64_t seed; int tid, nt, dither;
} gen_arg_t;

static void* gen_worker(void* p) {
    gen_arg_t* a = (gen_arg_t*)p;
    for (int64_t z = a->tid; z < a->Z; z += a->nt)
        for (int64_t y = 0; y < a->Y; ++y)
            for (int64_t x = 0; x < a->X; ++x) {
                uint32_t d;
                uint8_t q = boundary_q_at(z + a->oz, y + a->oy, x + a->ox, a->seed, &d);
                int64_t i = (z * a->Y + y) * a->X + x;
                /* quantized: q / 256; continuous (dither): (q * 2^16 + d) / 2^24, exact in float32 */
                if (a->out) a->out[i] = a->dither ? (float)((uint32_t)q * 65536u + d) / 16777216.0f : (float)q / 256.0f;
                if (a->outq) a->outq[i] = q;
            }
    return NULL;
}

/* out (float32) and/or outq (uint8 q) may be NULL; dither != 0: the continuous variant. */
void oracle_boundary_map(float* out, uint8_t* outq, int64_t Z, int64_t Y, int64_t X,
                         int64_t oz, int64_t oy, int64_t ox, uint64_t seed, int n_threads, int dither) {
    if (n_threads < 1) n_threads = 1;
    pthread_t th[256];
    gen_arg_t args[256];
    if (n_threads > 256) n_threads = 256;
    for (int t = 0; t < n_threads; ++t) {
        args[t] = (gen_arg_t){out, outq, Z, Y, X, oz, oy, ox, seed, t, n_threads, dither};
        pthread_create(&th[t], NULL, gen_worker, &args[t]);
    }
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------------- */
/* block grid (nifty.tools.blocking, C-order ids, roi begin 0)               */
/* ------------------------------------------------------------------------- */
typedef struct {
    int64_t shape[3], bs[3], nb[3], n_blocks;
} grid_t;

static void grid_init(grid_t* g, const int64_t* shape, const int64_t* bs) {
    g->n_blocks = 1;
    for (int a = 0; a < 3; ++a) {
        g->shape[a] = shape[a];
        g->bs[a] = bs[a];
        g->nb[a] = (shape[a] + bs[a] - 1) / bs[a];
        g->n_blocks *= g->nb[a];
    }
}

static void block_box(const grid_t* g, int64_t b, int64_t* beg, int64_t* end) {
    int64_t c[3];
    c[2] = b % g->nb[2];
    c[1] = (b / g->nb[2]) % g->nb[1];
    c[0] = b / (g->nb[2] * g->nb[1]);
    for (int a = 0; a < 3; ++a) {
        beg[a] = c[a] * g->bs[a];
        end[a] = beg[a] + g->bs[a];
        if (end[a] > g->shape[a]) end[a] = g->shape[a];
    }
}

/* getNeighborId(b, axis, lower=False): upper neighbour or -1 */
static int64_t upper_neighbor(const grid_t* g, int64_t b, int axis) {
    int64_t c[3];
    c[2] = b % g->nb[2];
    c[1] = (b / g->nb[2]) % g->nb[1];
    c[0] = b / (g->nb[2] * g->nb[1]);
    c[axis] += 1;
    if (c[axis] >= g->nb[axis]) return -1;
    return (c[0] * g->nb[1] + c[1]) * g->nb[2] + c[2];
}

/* ------------------------------------------------------------------------- */
/* stage 1: normalize + threshold + 26-conn label, per block                 */
/* ------------------------------------------------------------------------- */
enum { MODE_GREATER = 0, MODE_LESS = 1, MODE_EQUAL = 2 };

typedef struct {
    const float* in; const uint8_t* mask; uint64_t* labels; const grid_t* g;
    float thr; int mode; int job, n_jobs; uint64_t* values;
} bc_arg_t;

static inline uint32_t uf_find32(uint32_t* p, uint32_t x) {
    while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
    return x;
}

static inline void uf_union32(uint32_t* p, uint32_t a, uint32_t b) {
    a = uf_find32(p, a);
    b = uf_find32(p, b);
    if (a == b) return;
    if (a < b) p[b] = a; else p[a] = b;
}

#define NOFG 0xFFFFFFFFu

static void* block_components_worker(void* varg) {
    bc_arg_t* A = (bc_arg_t*)varg;
    const grid_t* g = A->g;
    const int64_t Y = g->shape[1], X = g->shape[2];
    uint32_t* par = NULL;
    size_t cap = 0;
    for (int64_t b = A->job; b < g->n_blocks; b += A->n_jobs) {
        int64_t beg[3], end[3];
        block_box(g, b, beg, end);
        const int64_t bz = end[0] - beg[0], by = end[1] - beg[1], bx = end[2] - beg[2];
        const size_t nv = (size_t)(bz * by * bx);
        if (nv > cap) { free(par); par = (uint32_t*)malloc(nv * sizeof(uint32_t)); cap = nv; }
#define GIDX(z, y, x) (((beg[0] + (z)) * Y + (beg[1] + (y))) * X + (beg[2] + (x)))
        /* mask: block skipped when the mask is empty (block_components.py:194-197) */
        if (A->mask) {
            int any = 0;
            for (int64_t z = 0; z < bz && !any; ++z)
                for (int64_t y = 0; y < by && !any; ++y)
                    for (int64_t x = 0; x < bx; ++x)
                        if (A->mask[GIDX(z, y, x)]) { any = 1; break; }
            if (!any) { A->values[b] = 0; continue; }
        }
        /* normalize (volume_utils.py:98-105): numpy min/max propagate NaN */
        float mn = INFINITY; int has_nan = 0;
        for (int64_t z = 0; z < bz; ++z)
            for (int64_t y = 0; y < by; ++y)
                for (int64_t x = 0; x < bx; ++x) {
                    float v = A->in[GIDX(z, y, x)];
                    if (v != v) has_nan = 1;
                    else if (v < mn) mn = v;
                }
        if (has_nan) mn = NAN;
        float m = -INFINITY; int m_nan = 0;
        for (int64_t z = 0; z < bz; ++z)
            for (int64_t y = 0; y < by; ++y)
                for (int64_t x = 0; x < bx; ++x) {
                    float v = A->in[GIDX(z, y, x)] - mn;
                    if (v != v) m_nan = 1;
                    else if (v > m) m = v;
                }
        if (m_nan) m = NAN;
        const int divide = (m > 0.0f);
        /* threshold (+mask) into par: foreground -> own index, background -> NOFG */
        int64_t n_fg = 0;
        for (int64_t z = 0; z < bz; ++z)
            for (int64_t y = 0; y < by; ++y)
                for (int64_t x = 0; x < bx; ++x) {
                    float v = A->in[GIDX(z, y, x)] - mn;
                    if (divide) v = v / m;
                    int fg = A->mode == MODE_GREATER ? (v > A->thr)
                           : A->mode == MODE_LESS ? (v < A->thr) : (v == A->thr);
                    if (A->mask && !A->mask[GIDX(z, y, x)]) fg = 0;
                    uint32_t i = (uint32_t)((z * by + y) * bx + x);
                    par[i] = fg ? i : NOFG;
                    n_fg += fg;
                }
        if (n_fg == 0) { A->values[b] = 0; continue; }  /* block NOT written */
        /* 26-connectivity union-find, link larger root under smaller: root = first voxel */
        for (int64_t z = 0; z < bz; ++z)
            for (int64_t y = 0; y < by; ++y)
                for (int64_t x = 0; x < bx; ++x) {
                    uint32_t i = (uint32_t)((z * by + y) * bx + x);
                    if (par[i] == NOFG) continue;
                    for (int dz = -1; dz <= 0; ++dz)
                        for (int dy = -1; dy <= 1; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                if (dz == 0 && (dy > 0 || (dy == 0 && dx >= 0))) continue;
                                int64_t nz = z + dz, ny = y + dy, nx = x + dx;
                                if (nz < 0 || ny < 0 || ny >= by || nx < 0 || nx >= bx) continue;
                                uint32_t j = (uint32_t)((nz * by + ny) * bx + nx);
                                if (par[j] != NOFG) uf_union32(par, i, j);
                            }
                }
        /* raster-order labels 1..n (first occurrence), written to ds_out[bb] */
        uint64_t n = 0;
        for (int64_t z = 0; z < bz; ++z)
            for (int64_t y = 0; y < by; ++y)
                for (int64_t x = 0; x < bx; ++x) {
                    uint32_t i = (uint32_t)((z * by + y) * bx + x);
                    uint64_t* out = &A->labels[GIDX(z, y, x)];
                    if (par[i] == NOFG) { *out = 0; continue; }
                    uint32_t r = uf_find32(par, i);
                    if (r == i) *out = ++n;
                    else {
                        int64_t rz = r / (by * bx), ry = (r / bx) % by, rx = r % bx;
                        *out = A->labels[GIDX(rz, ry, rx)];
                    }
                }
        A->values[b] = n + 1;
#undef GIDX
    }
    free(par);
    return NULL;
}

/* ------------------------------------------------------------------------- */
/* stage 3: face pairs                                                      */
/* ------------------------------------------------------------------------- */
typedef struct {
    const uint64_t* labels; const grid_t* g; const uint64_t* offsets; const uint8_t* empty;
    int job, n_jobs;
    uint64_t* pairs; size_t n_pairs, cap;
} bf_arg_t;

static void push_pair(bf_arg_t* A, uint64_t a, uint64_t b) {
    if (A->n_pairs == A->cap) {
        A->cap = A->cap ? 2 * A->cap : 1024;
        A->pairs = (uint64_t*)realloc(A->pairs, A->cap * 2 * sizeof(uint64_t));
    }
    A->pairs[2 * A->n_pairs] = a;
    A->pairs[2 * A->n_pairs + 1] = b;
    A->n_pairs++;
}

static void* block_faces_worker(void* varg) {
    bf_arg_t* A = (bf_arg_t*)varg;
    const grid_t* g = A->g;
    const int64_t Y = g->shape[1], X = g->shape[2];
    for (int64_t b = A->job; b < g->n_blocks; b += A->n_jobs) {
        if (A->empty[b]) continue;                               /* block_faces.py:118-120 */
        int64_t beg[3], end[3];
        block_box(g, b, beg, end);
        for (int axis = 0; axis < 3; ++axis) {
            int64_t nb = upper_neighbor(g, b, axis);
            if (nb < 0 || A->empty[nb]) continue;                /* volume_utils.py:228-233 */
            const uint64_t oa = A->offsets[b], ob = A->offsets[nb];
            /* face: a's extent, axis slab [end-1, end+1) (volume_utils.py:204-206) */
            int64_t lo[3], hi[3];
            for (int d = 0; d < 3; ++d) { lo[d] = beg[d]; hi[d] = end[d]; }
            lo[axis] = end[axis] - 1; hi[axis] = end[axis];
            int64_t step = axis == 0 ? Y * X : axis == 1 ? X : 1;
            for (int64_t z = lo[0]; z < hi[0]; ++z)
                for (int64_t y = lo[1]; y < hi[1]; ++y)
                    for (int64_t x = lo[2]; x < hi[2]; ++x) {
                        int64_t i = (z * Y + y) * X + x;
                        uint64_t la = A->labels[i], lb = A->labels[i + step];
                        if (la != 0 && lb != 0) push_pair(A, la + oa, lb + ob);
                    }
        }
    }
    return NULL;
}

/* ------------------------------------------------------------------------- */
/* stage 5: write                                                            */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint64_t* labels; const grid_t* g; const uint64_t* offsets; const uint8_t* empty;
    const uint64_t* lut; int job, n_jobs;
} wr_arg_t;

static void* write_worker(void* varg) {
    wr_arg_t* A = (wr_arg_t*)varg;
    const grid_t* g = A->g;
    const int64_t Y = g->shape[1], X = g->shape[2];
    for (int64_t b = A->job; b < g->n_blocks; b += A->n_jobs) {
        if (A->empty[b]) continue;                               /* write.py:219 */
        int64_t beg[3], end[3];
        block_box(g, b, beg, end);
        const uint64_t off = A->offsets[b];
        for (int64_t z = beg[0]; z < end[0]; ++z)
            for (int64_t y = beg[1]; y < end[1]; ++y)
                for (int64_t x = beg[2]; x < end[2]; ++x) {
                    uint64_t* s = &A->labels[(z * Y + y) * X + x];
                    if (*s) *s = A->lut[*s + off];               /* write.py:199-200 */
                }
    }
    return NULL;
}

static uint64_t uf_find64(uint64_t* p, uint64_t x) {
    while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
    return x;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/*
 * Whole path.  labels_out receives the final uint64 labels (min-id representatives of
 * the reference's id space).  Optional outputs may be NULL:
 *   local_out      block-local labels after stage 1 (skimage numbering, 0 outside)
 *   values_out     per block n_i+1 or 0                              [n_blocks]
 *   offsets_out    merge_offsets' offsets                            [n_blocks]
 *   lut_out        assignments LUT, written if lut_cap >= n_labels   [n_labels]
 *   stage_s        wall seconds of the 5 stages                      [5]
 * quirk_n_jobs > 0 emulates block_faces with that many jobs and the empty-job quirk.
 * Returns 0, or <0 on bad arguments / allocation failure.
 */
int oracle_label_volume(const float* in, const uint8_t* mask, const int64_t* shape,
                        const int64_t* block_shape, double threshold, int mode, int n_threads,
                        uint64_t* labels_out, uint64_t* local_out, uint64_t* values_out,
                        uint64_t* offsets_out, uint64_t* n_labels_out, uint64_t* lut_out,
                        int64_t lut_cap, uint64_t* max_id_out, int quirk_n_jobs,
                        double* stage_s) {
    if (!in || !labels_out || !shape || !block_shape) return -1;
    if (mode < 0 || mode > 2) return -2;
    for (int a = 0; a < 3; ++a)
        if (shape[a] < 1 || block_shape[a] < 1) return -3;
    if (block_shape[0] * block_shape[1] * block_shape[2] >= (int64_t)NOFG) return -4;
    grid_t g;
    grid_init(&g, shape, block_shape);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    const int64_t nb = g.n_blocks;
    const int64_t nvox = shape[0] * shape[1] * shape[2];
    double t0 = now_s(), t1, t2, t3, t4, t5;

    /* stage 1 */
    uint64_t* values = (uint64_t*)calloc(nb, sizeof(uint64_t));
    int n_jobs = (int)(nb < n_threads ? nb : n_threads);
    pthread_t th[256];
    {
        bc_arg_t args[256];
        memset(labels_out, 0, (size_t)nvox * sizeof(uint64_t));   /* fill value of the n5 dataset */
        for (int j = 0; j < n_jobs; ++j) {
            args[j] = (bc_arg_t){in, mask, labels_out, &g, (float)threshold, mode, j, n_jobs, values};
            pthread_create(&th[j], NULL, block_components_worker, &args[j]);
        }
        for (int j = 0; j < n_jobs; ++j) pthread_join(th[j], NULL);
    }
    if (local_out) memcpy(local_out, labels_out, (size_t)nvox * sizeof(uint64_t));
    t1 = now_s();

    /* stage 2: merge_offsets.py:109-120 */
    uint64_t* offsets = (uint64_t*)malloc(nb * sizeof(uint64_t));
    uint8_t* empty = (uint8_t*)malloc(nb);
    uint64_t acc = 0;
    for (int64_t b = 0; b < nb; ++b) {
        offsets[b] = acc;
        acc += values[b];
        empty[b] = values[b] == 0;
    }
    const uint64_t n_labels = offsets[nb - 1] + values[nb - 1] + 1;
    t2 = now_s();

    /* stage 3 */
    int n_bf = quirk_n_jobs > 0 ? (int)(nb < quirk_n_jobs ? nb : quirk_n_jobs) : n_jobs;
    bf_arg_t* bf = (bf_arg_t*)calloc(n_bf, sizeof(bf_arg_t));
    for (int j0 = 0; j0 < n_bf; j0 += 256) {
        int cnt = n_bf - j0 < 256 ? n_bf - j0 : 256;
        for (int j = 0; j < cnt; ++j) {
            bf[j0 + j] = (bf_arg_t){labels_out, &g, offsets, empty, j0 + j, n_bf, NULL, 0, 0};
            pthread_create(&th[j], NULL, block_faces_worker, &bf[j0 + j]);
        }
        for (int j = 0; j < cnt; ++j) pthread_join(th[j], NULL);
    }
    t3 = now_s();

    /* stage 4 */
    uint64_t* par = (uint64_t*)malloc(n_labels * sizeof(uint64_t));
    if (!par) return -5;
    for (uint64_t i = 0; i < n_labels; ++i) par[i] = i;
    int have = 1;
    if (quirk_n_jobs > 0)
        for (int j = 0; j < n_bf; ++j) have &= bf[j].n_pairs > 0;   /* all(ass.size ...) */
    if (have)
        for (int j = 0; j < n_bf; ++j)
            for (size_t k = 0; k < bf[j].n_pairs; ++k) {
                uint64_t a = uf_find64(par, bf[j].pairs[2 * k]);
                uint64_t b = uf_find64(par, bf[j].pairs[2 * k + 1]);
                if (a < b) par[b] = a; else if (b < a) par[a] = b;
            }
    uint64_t max_id = 0;
    for (uint64_t i = 0; i < n_labels; ++i) {
        par[i] = uf_find64(par, i);
        if (par[i] > max_id) max_id = par[i];
    }
    for (int j = 0; j < n_bf; ++j) free(bf[j].pairs);
    free(bf);
    t4 = now_s();

    /* stage 5 */
    {
        wr_arg_t args[256];
        for (int j = 0; j < n_jobs; ++j) {
            args[j] = (wr_arg_t){labels_out, &g, offsets, empty, par, j, n_jobs};
            pthread_create(&th[j], NULL, write_worker, &args[j]);
        }
        for (int j = 0; j < n_jobs; ++j) pthread_join(th[j], NULL);
    }
    t5 = now_s();

    if (values_out) memcpy(values_out, values, nb * sizeof(uint64_t));
    if (offsets_out) memcpy(offsets_out, offsets, nb * sizeof(uint64_t));
    if (n_labels_out) *n_labels_out = n_labels;
    if (lut_out && lut_cap >= (int64_t)n_labels) memcpy(lut_out, par, n_labels * sizeof(uint64_t));
    if (max_id_out) *max_id_out = max_id;
    if (stage_s) {
        stage_s[0] = t1 - t0; stage_s[1] = t2 - t1; stage_s[2] = t3 - t2;
        stage_s[3] = t4 - t3; stage_s[4] = t5 - t4;
    }
    free(par); free(values); free(offsets); free(empty);
    return 0;
}

int64_t oracle_n_blocks(const int64_t* shape, const int64_t* block_shape) {
    grid_t g;
    grid_init(&g, shape, block_shape);
    return g.n_blocks;
}

/* ------------------------------------------------------------------------- */
/* canonical relabel (the parity contract, BASELINE north_star): first        */
/* occurrence in C order -> 1, 2, ...; 0 stays 0.  Same result as oracle.py's */
/* numpy canon(), in one pass with an open-addressing hash (large volumes).   */
/* Returns the number of distinct non-zero ids, or -1 if it exceeds 2^32-2.    */
/* ------------------------------------------------------------------------- */
int64_t oracle_canon_u64(const uint64_t* in, int64_t n, uint32_t* out) {
    int64_t cap = 1 << 16;
    uint64_t* key = (uint64_t*)calloc((size_t)cap, sizeof(uint64_t));
    uint32_t* val = (uint32_t*)malloc((size_t)cap * sizeof(uint32_t));
    if (!key || !val) { free(key); free(val); return -1; }
    int64_t used = 0;
    uint64_t prev = 0;
    uint32_t prev_v = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t v = in[i];
        if (v == 0) { out[i] = 0; continue; }
        if (v == prev && prev_v) { out[i] = prev_v; continue; }   /* runs are the common case */
        if (2 * (used + 1) > cap) {                                /* grow x2, rehash */
            int64_t nc = 2 * cap;
            uint64_t* nk = (uint64_t*)calloc((size_t)nc, sizeof(uint64_t));
            uint32_t* nv = (uint32_t*)malloc((size_t)nc * sizeof(uint32_t));
            if (!nk || !nv) { free(nk); free(nv); free(key); free(val); return -1; }
            for (int64_t j = 0; j < cap; ++j)
                if (key[j]) {
                    uint64_t h = splitmix64(key[j]) & (uint64_t)(nc - 1);
                    while (nk[h]) h = (h + 1) & (uint64_t)(nc - 1);
                    nk[h] = key[j]; nv[h] = val[j];
                }
            free(key); free(val);
            key = nk; val = nv; cap = nc;
        }
        uint64_t h = splitmix64(v) & (uint64_t)(cap - 1);
        while (key[h] && key[h] != v) h = (h + 1) & (uint64_t)(cap - 1);
        if (!key[h]) {
            if (used >= 0xFFFFFFFELL) { free(key); free(val); return -1; }
            key[h] = v; val[h] = (uint32_t)(++used);
        }
        out[i] = prev_v = val[h];
        prev = v;
    }
    free(key); free(val);
    return used;
}
