// cc_aux.hip -- second translation unit of libcc_mi355x.so: segmentation evaluation
// (cc_eval.hip), consecutive relabelling (cc_relabel.hip), the channel / Gaussian prefilter
// (cc_prefilter.hip) and the seeded watershed (cc_watershed.hip), with their C-ABI entries.
//
// A unit of its own because the HIP runtime loads a code object whole, every kernel of it, at
// the first launch from it: kept apart, the ~60 kernels here (the prefilter's 40 template
// instances alone) are loaded only by the jobs that use them, and a one-shot labelling job's
// first call loads the labelling path's code object only (profiles/r04_cold_split.jsonl: the
// first cc_label_volume of a fresh process 5.3 -> 3.9-4.1 ms, dlopen 0.87 -> 0.5 ms).
#include "cc_rows.hpp"
#include "cc_ctx.hpp"
#define CC_PRIMS_NS aux
#include "cc_prims.hip"

namespace cc {
inline namespace aux {
// per-block statistics of the normalisation steps (this unit's copy of cc_kernels.hip's kernel)
__global__ __launch_bounds__(NTHREADS) void k_block_stats(Geom g, const float* __restrict__ in,
                                                          u32* smin, u32* smax, u32* sflag) {
    __shared__ u32 red[3][NTHREADS / 64];
    stats_tile(g, tile_info(g, blockIdx.x), in, smin, smax, sflag, red);
}
}  // namespace aux
}  // namespace cc

#include "cc_eval.hip"
#include "cc_relabel.hip"
#include "cc_prefilter.hip"
#include "cc_watershed.hip"
