/*
 * cc_mi355x.h -- C ABI of the MI355X thresholded connected-components library
 * (libcc_mi355x.so, built from the HIP sources in cluster_tools_amd/csrc for gfx950).
 *
 * Drop-in boundary for cluster_tools' ThresholdedComponentsWorkflow (reference v0.3.3).
 * The reference has no native boundary of its own: its five stages are Python job
 * functions run as `python <tmp>/<task>.py <tmp>/<task>_job_<i>.config`
 * (cluster_tools/cluster_tasks.py:529-543).  Each entry point below replaces the
 * compute of one of those job functions (or all five, fused); the Python host shell
 * (package cluster_tools_amd.thresholded_components) keeps the task classes, configs,
 * tmp artefacts and log tokens and calls these through ctypes.  See INTEGRATION.md.
 *
 * Conventions
 *   - status: 0 = ok, < 0 = error; cc_last_error() returns the message of the last
 *     failure on the calling thread.  The Python binding raises RuntimeError.
 *   - volumes are C-order (Z, Y, X); shape/block_shape are int64[3] host arrays.
 *   - the _dev pointers are device pointers (hipMalloc / torch CUDA tensors); the
 *     _host entry points take host pointers and copy.
 *   - mode: 0 = 'greater', 1 = 'less', 2 = 'equal'  (block_components.py:41,166-173).
 *     threshold is cast to float32, as numpy does for `float32_array OP python_float`.
 *   - one cc_ctx per GPU; a ctx is not thread-safe; all work is enqueued on the
 *     ctx's stream (cc_set_stream) and the call returns when it is complete.
 *   - output label semantics: the reference id space (block offset + skimage label,
 *     merge_offsets.py:115-120, block_faces.py:108-109) with the union-find
 *     representative = the smallest id of each component.  The reference uses
 *     nifty's boost_ufd representative instead; the partition is identical and
 *     maxId (= n_labels - 1) is identical.
 */
#ifndef CC_MI355X_H
#define CC_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cc_ctx cc_ctx;

/* Results of one labelling run (host copy of the small artefacts). */
typedef struct {
    int64_t  n_blocks;      /* blocks_in_volume(shape, block_shape)           */
    uint64_t n_labels;      /* merge_offsets.py:120                            */
    uint64_t max_id;        /* write.py:281-289 (attrs['maxId'])               */
    uint64_t n_components;  /* number of distinct non-zero output labels      */
    uint64_t n_block_components; /* sum over blocks of n_i (block-local comps) */
    uint64_t n_relabelled_tiles; /* tiles whose speculated foreground interval was not exact and
                                    were labelled again (instrumentation; results never depend on it) */
    uint64_t identity_lut;  /* 1 if CC_OPT_EMPTY_JOB_QUIRK found an empty face job: no block-face
                               merge, the LUT is the identity (merge_assignments.py:115-123) */
} cc_result;

/* sizeof(cc_result) as built: a binding checks its struct against it before passing one
 * (ctypes: assert ctypes.sizeof(_Res) == cc_result_size()).  No GPU needed. */
int64_t     cc_result_size(void);

/* --- context ----------------------------------------------------------- */
int         cc_create(int device, cc_ctx** out);
void        cc_destroy(cc_ctx* ctx);
const char* cc_last_error(void);
/* use an existing hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL (the default)
 * -> the null stream */
int         cc_set_stream(cc_ctx* ctx, void* hip_stream);
/* library version string, e.g. "cc_mi355x 0.2 gfx950 src=0123456789abcdef": src = SHA-256 prefix of
 * the sources (csrc/ files, this header) the library was built from (binary provenance, build.py) */
const char* cc_version(void);

/* --- fused path: block_components -> merge_offsets -> block_faces ->
 *     merge_assignments -> write, all on the device.
 * Replaces: block_components  cluster_tools/thresholded_components/block_components.py:236-291
 *           merge_offsets     cluster_tools/thresholded_components/merge_offsets.py:83-131
 *           block_faces       cluster_tools/thresholded_components/block_faces.py:140-177
 *           merge_assignments cluster_tools/thresholded_components/merge_assignments.py:88-141
 *           write (offsets)   cluster_tools/write/write.py:185-220,292-387
 * in_dev     float32 [Z*Y*X]
 * mask_dev   uint8 [Z*Y*X] or NULL (nonzero = inside, block_components.py:194,225)
 * labels_dev uint64 [Z*Y*X] final labels (0 = background)
 * res        may be NULL
 * Device volumes (here and in every entry below) are read / written with vector accesses of up to
 * 16 B wherever their rows allow, so each base must be aligned like its rows: to the largest power
 * of two <= 16 dividing the row's bytes (X * element size).  Any hipMalloc / torch allocation and
 * any z-slab view of one is; a view at an odd element offset may not be, and is refused with an
 * error (-1, cc_last_error) instead of being read.
 */
int cc_label_volume(cc_ctx* ctx, const float* in_dev, const uint8_t* mask_dev,
                    const int64_t shape[3], const int64_t block_shape[3],
                    double threshold, int mode, uint64_t* labels_dev, cc_result* res);

/* Same with host buffers (copies in and out; the PCIe-inclusive path). */
int cc_label_volume_host(cc_ctx* ctx, const float* in_host, const uint8_t* mask_host,
                         const int64_t shape[3], const int64_t block_shape[3],
                         double threshold, int mode, uint64_t* labels_host, cc_result* res);

/* Artefacts of the last cc_label_volume* call, copied to host:
 *   block values v_i = n_i + 1 or 0   (connected_components_offsets_<job>.json values,
 *                                      block_components.py:175-182,286-290)
 *   offsets                           (cc_offsets.json 'offsets', merge_offsets.py:115-117)
 *   lut[n_labels]                     (the 'assignments' dataset, merge_assignments.py:136-139)
 * Each returns the number of elements written, or <0 (error / cap too small). */
int64_t cc_get_block_values(cc_ctx* ctx, uint64_t* out_host, int64_t cap);
int64_t cc_get_offsets(cc_ctx* ctx, uint64_t* out_host, int64_t cap);
int64_t cc_get_lut(cc_ctx* ctx, uint64_t* out_host, int64_t cap);

/* --- stage-level entry points (each a single reference job's compute) ---------- */

/* block_components (block_components.py:143-291): block-local 26-connected labels in
 * skimage numbering (1..n_i, raster first occurrence) written to labels_dev (0 outside),
 * and values_host[n_blocks] = n_i + 1 or 0. */
int cc_block_components(cc_ctx* ctx, const float* in_dev, const uint8_t* mask_dev,
                        const int64_t shape[3], const int64_t block_shape[3],
                        double threshold, int mode, uint64_t* labels_dev,
                        uint64_t* values_host, int64_t n_blocks);

/* Threshold task (thresholded_components/threshold.py:131-171, _threshold_block): per
 * reference block normalize (volume_utils.py:98-105) then `> / < / ==` threshold (float32), the
 * result as uint8 0/1 of the same shape.  in_dev / out_dev are device pointers (C-order).
 * Multi-channel input: cc_channel_mean first. */
int cc_threshold(cc_ctx* ctx, const float* in_dev, const int64_t shape[3], const int64_t block_shape[3],
                 double threshold, int mode, uint8_t* out_dev);

/* Multi-channel input (the `channel` parameter of BlockComponents / Threshold,
 * block_components.py:150-159, threshold.py:139-148): out_dev[Z*Y*X] (float32) = the mean of the
 * listed channels of in_dev (C, Z, Y, X) = shape4, in list order (repeats allowed), computed as
 * np.mean(stack, axis=0) in the reference: sequential sum over the list, float32 accumulation and
 * division for float32 input, float64 for every other dtype, then the cast to float32 of
 * vu.normalize (volume_utils.py:99).  The result feeds cc_label_volume / cc_threshold. */
#define CC_DTYPE_FLOAT32 0
#define CC_DTYPE_FLOAT64 1
#define CC_DTYPE_UINT8   2
#define CC_DTYPE_INT8    3
#define CC_DTYPE_UINT16  4
#define CC_DTYPE_INT16   5
#define CC_DTYPE_UINT32  6
#define CC_DTYPE_INT32   7
#define CC_DTYPE_UINT64  8
#define CC_DTYPE_INT64   9
int cc_channel_mean(cc_ctx* ctx, const void* in_dev, int dtype, const int64_t shape4[4],
                    const int64_t* channels, int64_t n_channels, float* out_dev);

/* sigma_prefilter (block_components.py:161-163, threshold.py:151-153): out_dev = per block of
 * block_shape, gaussianSmoothing(normalize(block), sigma) with the block's own borders (reflected,
 * no halo), as float32; the labelling / threshold entry points then apply the second normalize.
 * The filter restates vigra.filters.gaussianSmoothing (the reference's fallback when fastfilters is
 * absent): taps of Kernel1D::initGaussian in float32 (radius (int)(3 sigma + 0.5)), separable
 * z -> y -> x, BORDER_TREATMENT_REFLECT, float32 sums without FMA (parity with vigra unpinned).
 * Error when a block line is not longer than the radius (vigra: "kernel longer than line") or the
 * radius exceeds 64.  in_dev and out_dev may alias.  cc_gaussian_taps writes the 2r + 1 taps and
 * returns r. */
int cc_gaussian_smooth_blocks(cc_ctx* ctx, const float* in_dev, const int64_t shape[3],
                              const int64_t block_shape[3], double sigma, float* out_dev);
int cc_gaussian_taps(double sigma, float* taps, int cap);

/* Masks of another shape than the volume (block_components.py:274-275 -> volume_utils.py:174-184:
 * elf ResizedVolume(mask, shape, order=0)): out_dev = rows z0 .. z0 + nz of the mask resized to
 * shape by nearest neighbour, src(c) = floor((c + 0.5) * m / S) per axis (skimage resize(order=0)
 * of the whole mask), as uint8 0 / 1; mask_dev is the (mZ, mY, mX) uint8 mask, out_dev nz*Y*X
 * bytes.  The result is the mask argument of the labelling entry points.  elf is absent: the
 * reference resizes each block's crop, whose rounding this does not restate (parity unpinned). */
int cc_resize_mask_nearest(cc_ctx* ctx, const uint8_t* mask_dev, const int64_t mshape[3], const int64_t shape[3],
                           int64_t z0, int64_t nz, uint8_t* out_dev);

/* merge_offsets (merge_offsets.py:104-120): exclusive scan of values; writes offsets
 * and empty flags; returns n_labels through *n_labels. Host arrays. */
int cc_merge_offsets(const uint64_t* values_host, int64_t n_blocks, uint64_t* offsets_host,
                     uint8_t* empty_host, uint64_t* n_labels);

/* block_faces (block_faces.py:87-177): from block-local labels (device) and offsets
 * (host), the deduplicated face pairs (label_a + off_a, label_b + off_b), sorted
 * lexicographically like np.unique(axis=0).  Writes at most cap pairs to pairs_host
 * ([cap][2]); returns the number of pairs (may exceed cap: call again with a larger cap).
 * block_has_pairs_host (nullable, n_blocks bytes): 1 for every block with a pair on one of its
 * upper faces (the block's face job emits it; used for the empty-job emulation). */
int64_t cc_block_faces(cc_ctx* ctx, const uint64_t* labels_dev, const int64_t shape[3],
                       const int64_t block_shape[3], const uint64_t* offsets_host,
                       uint64_t* pairs_host, int64_t cap, uint8_t* block_has_pairs_host);

/* merge_assignments (merge_assignments.py:105-130): union-find over ids 0..n_labels-1
 * merged by pairs (host, [n_pairs][2]); lut_host[n_labels] = min id of each set. */
int cc_merge_assignments(cc_ctx* ctx, const uint64_t* pairs_host, int64_t n_pairs,
                         uint64_t n_labels, uint64_t* lut_host);

/* write with offsets (write.py:185-220): per non-empty block, seg[seg!=0] += off;
 * seg = lut[seg], in place on labels_dev.  offsets/lut are host arrays. */
int cc_write(cc_ctx* ctx, uint64_t* labels_dev, const int64_t shape[3],
             const int64_t block_shape[3], const uint64_t* offsets_host,
             const uint64_t* lut_host, uint64_t n_labels);

/* --- z-slab sharding (multi-GPU, one process and one cc_ctx per GPU) ----------------------
 * The volume is split along z at block faces; rank r labels slab r.  Collective schedule
 * (cluster_tools_amd/distributed.py, RCCL over xGMI):
 *   cc_shard_begin   local stages up to the per-slab block offsets; returns the slab's sum of
 *                    block values (merge_offsets.py:115-120 restricted to the slab)
 *   [allgather of the sums -> id_base = sum over the slabs below]
 *   cc_shard_assign  global ids (offsets + id_base) and the slab's 6-connected block-face unions
 *   cc_shard_planes  bottom / top voxel planes as component ids (Y*X uint64 each, NULL = skip);
 *                    enqueued on the ctx's stream, returns without waiting (order by stream)
 *   [send top plane to rank r+1; rank r+1 forms the seam pairs with cc_seam_pairs;
 *    allgather of all seam pairs]
 *   cc_shard_finish  replicated union-find over all seam pairs, LUT, final labels.
 * cc_get_lut then returns the slab's part of the LUT (ids id_base .. id_base + sum). */
int cc_shard_begin(cc_ctx* ctx, const float* in_dev, const uint8_t* mask_dev,
                   const int64_t slab_shape[3], const int64_t block_shape[3], double threshold,
                   int mode, int64_t z_offset, uint64_t* sum_values);
int cc_shard_assign(cc_ctx* ctx, uint64_t id_base);
int cc_shard_planes(cc_ctx* ctx, uint64_t* bottom_dev, uint64_t* top_dev);
/* unique (upper[i], lower[i]) pairs with both non-zero, sorted; writes min(cap, count) pairs
 * ([n][2] uint64, device) and returns the count */
int64_t cc_seam_pairs(cc_ctx* ctx, const uint64_t* upper_dev, const uint64_t* lower_dev, int64_t n,
                      uint64_t* pairs_dev, int64_t cap);
int cc_shard_finish(cc_ctx* ctx, const uint64_t* pairs_dev, int64_t n_pairs, uint64_t* labels_dev,
                    cc_result* res);
/* The top plane in the compact form sent over xGMI (half the bytes of cc_shard_planes' top):
 * uint32 id - id_base + 1, 0 = background (requires the slab's sum of block values < 2^32 - 2),
 * and cc_seam_pairs on it, given the sending slab's id_base. */
int cc_shard_top_plane32(cc_ctx* ctx, uint32_t* top32_dev);
int64_t cc_seam_pairs32(cc_ctx* ctx, const uint32_t* upper32_dev, uint64_t upper_id_base,
                        const uint64_t* lower_dev, int64_t n, uint64_t* pairs_dev, int64_t cap);
/* The top plane as one uint32 per 2x2 cube of the global cube grid, ceil(Y/2) x ceil(X/2):
 * (id - id_base + 1) << 4 | the cube's 4 voxel bits ((y & 1) * 2 + (x & 1)), 0 = background; a
 * quarter of the voxel plane's bytes.  Needs even block_shape[1:] (or one block along the axis)
 * and the slab's sum of block values < 2^28 - 2.  cc_seam_pairs_cubes32 forms the seam pairs
 * from it (upper) and this slab's uint64 bottom plane (lower, Y x X). */
int cc_shard_top_cubes32(cc_ctx* ctx, uint32_t* cubes_dev);
int64_t cc_seam_pairs_cubes32(cc_ctx* ctx, const uint32_t* upper_cubes_dev, uint64_t upper_id_base,
                              const uint64_t* lower_dev, int64_t Y, int64_t X, uint64_t* pairs_dev,
                              int64_t cap);

/* One-read-back schedule of the z-slab shards (distributed.py's default).  The same collective
 * schedule as above, but nothing comes back to the host until cc_shard_dev_finish: counts, the
 * id base and the seam pairs stay in device memory between the collectives, which the caller
 * runs on the ctx's stream (RCCL allgather / point-to-point on device buffers).
 *   cc_shard_dev_begin      local stages; the slab's sum of block values -> sum_dev (1 uint64)
 *   [allgather sum_dev -> sums_dev[world]]
 *   cc_shard_dev_assign     id base = sum of sums_dev[0 .. rank) on the device; block-face unions
 *   cc_shard_dev_top_cubes  the top plane in the cube form of cc_shard_top_cubes32 (even
 *                           block_shape[1:] required)
 *   [send it to rank + 1]
 *   cc_shard_dev_seam_pairs hdr_pairs_dev[cap + 1][2]: row 0 = (pair count, redo flags), then up to
 *                           cap seam pairs (upper id, lower id) of this slab's bottom face against
 *                           the slab below's cube plane (upper_cubes_dev NULL on rank 0: header only)
 *   [allgather hdr_pairs_dev -> all_dev[world][cap + 1][2]]
 *   cc_shard_dev_finish     replicated union-find over every slab's pairs, LUT, final labels; the
 *                           step's ONE host read-back.  status_host[4] = redo flags, the largest
 *                           pair count of a slab, the global n_labels, this slab's id base.  Redo
 *                           flags != 0 (identical on every rank: computed from the allgathered
 *                           headers and sums) mean an optimistic bound did not hold -- more seam
 *                           pairs than cap (8), ids beyond the 28-bit cube form (4), more roots than
 *                           the context's root arrays (2), a block needing the global-stitch
 *                           fallback (1), a tile's block-face pair list overflowing (16) -- and the
 *                           caller relabels this step with the schedule
 *                           above (cc_shard_begin ...), which sizes everything from read-backs. */
/* 1 when this context can run the schedule above, 0 when it must use the host-synchronised one:
 * CC_FAST=0 in the environment, CC_FRONT_CHUNKS > 1, CC_DEBUG_GLOBAL_STITCH or the empty-job quirk
 * option (cc_shard_dev_begin fails on such a context).  Callers decide the schedule from it on
 * every rank alike (distributed.py takes the minimum over the ranks). */
int cc_shard_dev_ok(cc_ctx* ctx);
int cc_shard_dev_begin(cc_ctx* ctx, const float* in_dev, const uint8_t* mask_dev, const int64_t slab_shape[3],
                       const int64_t block_shape[3], double threshold, int mode, int64_t z_offset,
                       uint64_t* sum_dev);
int cc_shard_dev_assign(cc_ctx* ctx, const uint64_t* sums_dev, int rank, int world);
int cc_shard_dev_top_cubes(cc_ctx* ctx, uint32_t* cubes_dev);
int cc_shard_dev_seam_pairs(cc_ctx* ctx, const uint32_t* upper_cubes_dev, const uint64_t* sums_dev, int rank,
                            uint64_t* hdr_pairs_dev, int64_t cap);
int cc_shard_dev_finish(cc_ctx* ctx, const uint64_t* all_dev, int world, int64_t cap, const uint64_t* sums_dev,
                        uint64_t* labels_dev, cc_result* res, uint64_t* status_host);

/* --- z-slab sharding with RCCL inside the library (cc_comm.hip) ----------------------------
 * Replaces the reference's job pool for this path (cluster_tools/cluster_tasks.py:529-551: the
 * block_components / block_faces / write jobs of a ProcessPool exchanging offsets and face
 * assignments through files) for a plain C / ctypes caller: one process (or thread) per GPU,
 * each owning the z-slab [z_offset, z_offset + slab_depth) of the volume (slab boundaries on
 * block faces); the one-read-back schedule above with its three exchanges as RCCL collectives
 * on the context's stream (the communicator's own stream when the context has none), and the
 * host-synchronised schedule (uint64 seam planes) when a step's status asks for it.  Results are
 * those of cc_label_volume on the whole volume (labels of this slab; res->n_labels global).
 *   cc_comm_unique_id   the RCCL bootstrap id (128 bytes), made on one rank and handed to all
 *   cc_comm_create      one rank's communicator (ncclCommInitRank: collective over the ranks)
 *   cc_comm_info        out[8]: world, rank, last schedule (1 one-read-back, 0 synchronised,
 *                       -1 none), RF_* redo flags of the last one-read-back attempt, seam-pair
 *                       capacity, aborted (0/1), calls, 0
 * Every call of cc_label_volume_sharded is collective: it begins with an agreement over the ranks
 * (arguments, volume, slab tiling in rank order), so a bad argument on ANY rank makes every rank
 * return -1 and the communicator stays usable.  An error after the agreement aborts the
 * communicator (ncclCommAbort) so peers blocked in a collective return too (every host wait is
 * bounded by CC_COMM_TIMEOUT seconds, default 300); an aborted communicator refuses further calls
 * and must be destroyed.  Ordering: with no stream set on the context the call runs on the
 * communicator's stream, after the work queued on the null stream and before the null stream's
 * later work.
 * RCCL is opened on first use (an RCCL already in the process, e.g. torch's, is reused;
 * CC_RCCL_PATH overrides). */
typedef struct cc_comm cc_comm;
int  cc_comm_unique_id(void* id_out, int64_t cap);
int  cc_comm_create(const void* id, int world, int rank, int device, cc_comm** out);
int  cc_comm_info(const cc_comm* comm, int64_t* out);
void cc_comm_destroy(cc_comm* comm);
int  cc_label_volume_sharded(cc_ctx* ctx, cc_comm* comm, const float* slab_dev, const uint8_t* mask_dev,
                             const int64_t global_shape[3], int64_t z_offset, int64_t slab_depth,
                             const int64_t block_shape[3], double threshold, int mode,
                             uint64_t* labels_dev, cc_result* res);

/* --- synthetic benchmark input (oracle/synth.py is its restatement) ---
 * dither = 0: q / 256 (quantized); dither = 1: (q * 2^16 + 16-bit hash dither) / 2^24, the
 * continuous variant (block extremes and threshold crossings no longer on a 2^-8 grid). */
int cc_generate_boundary_map(cc_ctx* ctx, float* out_dev, const int64_t shape[3],
                             const int64_t origin[3], uint64_t seed, int dither);

/* --- instrumentation ---------------------------------------------------------- */
/* Per-kernel HIP-event timing on the stream each kernel runs on: enable = 0 off, 1 every launch
 * (one event pair per launch), 2 only the volume-sized kernels k_spec and k_pass2 (what bench.py
 * keeps on inside its timed region). */
int cc_set_profiling(cc_ctx* ctx, int enable);
/* Accumulated per-kernel totals since the last reset: name list as "k1,k2,...",
 * and for each: launch count and total milliseconds.  Returns number of kernels. */
int cc_get_profile(cc_ctx* ctx, char* names, int names_cap, int64_t* counts, double* total_ms,
                   int cap);
int cc_reset_profile(cc_ctx* ctx);
/* Options.  CC_OPT_EMPTY_JOB_QUIRK = max_jobs (0 = off, the default): reproduce the reference's
 * empty-job branch -- block_faces job j owns blocks j :: min(n_blocks, max_jobs)
 * (cluster_tasks.py:301-335); if any job has no face pair (it saves [], block_faces.py:169-176),
 * merge_assignments drops every merge and writes the identity LUT (merge_assignments.py:115-123).
 * Fused single-volume path only. */
#define CC_OPT_EMPTY_JOB_QUIRK 1
/* CC_OPT_WS_PRENORMALIZED = 1: cc_watershed_from_seeds takes its input as the already normalized
 * block values (4-D input: the output of cc_normalize_channels) instead of normalizing each block
 * itself; 0 (the default) normalizes (3-D input, watershed_from_seeds.py:138). */
#define CC_OPT_WS_PRENORMALIZED 2
int cc_set_option(cc_ctx* ctx, int option, int64_t value);
/* Test hook: CC_DEBUG_GLOBAL_STITCH routes every block's intra-block seams through the global
 * union-find fallback instead of the per-block LDS path (both must give identical results). */
#define CC_DEBUG_GLOBAL_STITCH 1
int cc_set_debug(cc_ctx* ctx, int flags);

/* --- segmentation evaluation ------------------------------------------------
 * EvaluationWorkflow (evaluation/evaluation_workflow.py:46-84): overlaps of seg with gt per block
 * of the evaluation grid (node_labels/block_node_labels.py:133-166: a block whose seg sums to 0 is
 * skipped; voxels with gt == ignore_label are not counted when use_ignore), then the contingency
 * table and the measures (evaluation/measures.py:81-162; a = gt sizes, b = seg sizes).
 * seg_dev / gt_dev: uint64 device volumes (C-order, 8-byte aligned).  Ids: seg < 2^31,
 * gt < 2^32 - 1 (error otherwise).  vi_* in bits (log2). */
typedef struct {
    uint64_t n_points;            /* measures.py:113                               */
    uint64_t n_pairs;             /* contingency-table entries (seg id, gt id)      */
    uint64_t n_seg_ids;           /* distinct seg ids counted (b_dict)              */
    uint64_t n_gt_ids;            /* distinct gt ids counted (a_dict)               */
    double   vi_split;            /* H(seg | gt)                                    */
    double   vi_merge;            /* H(gt | seg)                                    */
    double   adapted_rand_error;  /* 1 - 2 P R / (P + R)                            */
    double   rand_index;          /* 1 - (sum a^2 + sum b^2 - 2 sum p^2) / N^2       */
    double   sum_sq_pairs, sum_sq_gt, sum_sq_seg;
} cc_eval_result;

/* status CC_ERR_ID_RANGE: an id beyond the key packing (seg >= 2^31 or gt >= 2^32 - 1); relabel
 * the volumes consecutively (cc_relabel_consecutive) and call again */
#define CC_ERR_ID_RANGE (-3)
int cc_evaluate(cc_ctx* ctx, const uint64_t* seg_dev, const uint64_t* gt_dev, const int64_t shape[3],
                const int64_t block_shape[3], int use_ignore, uint64_t ignore_label, cc_eval_result* out);
/* contingency table of the last cc_evaluate (unordered); returns its size (copies min(size, cap)) */
int64_t cc_get_overlaps(cc_ctx* ctx, uint64_t* seg_ids, uint64_t* gt_ids, uint64_t* counts, int64_t cap);

/* --- consecutive relabelling --------------------------------------------------
 * RelabelWorkflow (relabel/relabel_workflow.py:10-60; find_labeling.py:84-120): the sorted unique
 * ids of labels_dev get new ids start, start + 1, ... (start = 0 when id 0 occurs, else 1); the
 * volume mapped into out_dev (may alias labels_dev).  n uint64 device elements.  Returns the
 * number of unique ids and start; copies the sorted unique ids to uniques_host (nullable) -- the
 * old ids of the assignment table, new id = index + start.  If uniques_host is given and
 * cap < n_unique, only n_unique / start are returned and out_dev is NOT written (safe for in-place
 * calls: call again with cap >= n_unique).  Id 2^64-1 is reserved (error). */
int cc_relabel_consecutive(cc_ctx* ctx, const uint64_t* labels_dev, uint64_t* out_dev, int64_t n,
                           uint64_t* n_unique, uint64_t* start_label, uint64_t* uniques_host, int64_t cap);

/* Seeded watershed per block (watershed/watershed_from_seeds.py:143-273, the WatershedFromSeeds
 * task of ThresholdAndWatershedWorkflow, thresholded_components_workflow.py:107-144): the seeds
 * (uint64 ids < 2^32 - 1, 0 = none; e.g. the thresholded components) grow over the input
 * normalized per block (volume_utils.py:98-105), 6-connected inside each block (no halo).  The
 * reference calls vu.watershed, which its volume_utils does not define (parity unpinned):
 * cost(v) = min over paths from a seed of the max normalized value on the path (seed excluded),
 * label(v) = the smallest label among the neighbours an optimal path can come through
 * (max(cost(u), f(v)) == cost(v)); 0 where no seed of the block reaches v.  mask_dev (optional,
 * uint8, same shape): the input is 1.0 outside the mask and the output 0 there
 * (_ws_block_masked).  out_dev may be seeds_dev (in place, as the workflow writes).  *rounds
 * (optional): relaxation rounds run. */
int cc_watershed_from_seeds(cc_ctx* ctx, const float* in_dev, const uint64_t* seeds_dev, const uint8_t* mask_dev,
                            const int64_t shape[3], const int64_t block_shape[3], uint64_t* out_dev,
                            int64_t* rounds);
/* 4-D (channel) input of the watershed (_read_data, watershed_from_seeds.py:127-139): in_dev =
 * the selected channels (n_channels, Z, Y, X) as float32 (the reference's normalize casts first);
 * per block of block_shape the 4-D block is normalized as one array (vu.normalize, one min / max
 * over all its channels, volume_utils.py:98-105), then aggregated over the channels in order:
 * agg 0 = np.mean (float32 sequential sum, then / n_channels), 1 = np.max, 2 = np.min (NaN
 * propagates).  out_dev (Z, Y, X) float32: the watershed's input with CC_OPT_WS_PRENORMALIZED. */
int cc_normalize_channels(cc_ctx* ctx, const float* in_dev, int64_t n_channels, const int64_t shape[3],
                          const int64_t block_shape[3], int agg, float* out_dev);

#ifdef __cplusplus
}
#endif
#endif /* CC_MI355X_H */
