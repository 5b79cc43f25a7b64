// cc_host.hpp -- host-side helpers shared by the library (cc_lib.hip) and the kernel
// ablation harness (tools/ablate.hip): error type, block grid + tile tables.
#pragma once
#include <cstdint>
#include <initializer_list>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "cc_common.hpp"

namespace cc {

struct CCError {
    std::string msg;
};

#define HIP_OK(expr)                                                                           \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            throw CCError{std::string(#expr) + ": " + hipGetErrorString(e_)};                  \
    } while (0)

#define CC_REQUIRE(cond, msg)                                                                  \
    do {                                                                                       \
        if (!(cond)) throw CCError{msg};                                                       \
    } while (0)

// A device volume is read / written with vector accesses of up to 16 B wherever its rows allow
// them, so its base must be aligned like its rows: to the largest power of two <= 16 dividing the
// row's bytes (16 B for rows of a multiple of 16 bytes).  Any hipMalloc / torch allocation is, and
// so is a z-slab view of one; a view at an odd element offset may not be.
inline void require_row_aligned(const void* p, int64_t row_bytes) {
    const int64_t need = row_bytes > 0 ? std::min<int64_t>(16, row_bytes & -row_bytes) : 16;
    CC_REQUIRE(((uintptr_t)p % (uintptr_t)need) == 0,
               "device buffer not " + std::to_string(need) + "-byte aligned (its rows are)");
}

// Block grid + tile tables (tiles tiled from each block's origin).
struct HostGeom {
    Geom g;
    std::vector<int32_t> tab;  // [3][3][nt] packed
    int64_t nvox;
};

static HostGeom make_geom(const int64_t shape[3], const int64_t block_shape[3], int64_t zoff) {
    HostGeom hg;
    Geom& g = hg.g;
    std::memset(&g, 0, sizeof(g));
    const int T[3] = {TZ, TY, TX};
    std::vector<int32_t> st[3], ln[3], bk[3];
    int maxlen[3] = {0, 0, 0};
    for (int a = 0; a < 3; ++a) {
        CC_REQUIRE(shape[a] >= 1 && shape[a] < (1LL << 31), "shape must be in [1, 2^31)");
        CC_REQUIRE(block_shape[a] >= 1, "block_shape must be >= 1");
        const int64_t nb = (shape[a] + block_shape[a] - 1) / block_shape[a];
        g.nb[a] = (int32_t)nb;
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t b0 = b * block_shape[a], b1 = std::min(b0 + block_shape[a], shape[a]);
            for (int64_t s = b0; s < b1; s += T[a]) {
                const int l = (int)std::min<int64_t>(T[a], b1 - s);
                st[a].push_back((int32_t)s);
                ln[a].push_back(l);
                bk[a].push_back((int32_t)b);
                maxlen[a] = std::max(maxlen[a], l);
            }
        }
        g.nt[a] = (int32_t)st[a].size();
    }
    g.Z = shape[0]; g.Y = shape[1]; g.X = shape[2];
    g.gY = shape[1]; g.gX = shape[2];
    g.zoff = zoff;
    g.n_tiles = (int64_t)g.nt[0] * g.nt[1] * g.nt[2];
    g.n_blocks = (int64_t)g.nb[0] * g.nb[1] * g.nb[2];
    g.cap = ((maxlen[0] + 1) / 2) * ((maxlen[1] + 1) / 2) * ((maxlen[2] + 1) / 2);
    hg.nvox = shape[0] * shape[1] * shape[2];
    CC_REQUIRE((uint64_t)g.n_tiles * (uint64_t)g.cap < 0xFFFFFFF0ull,
               "too many tiles x cubes for 32-bit node ids (block shape too small for this volume)");
    CC_REQUIRE(g.n_blocks < (1LL << (64 - KEY_BITS)), "too many blocks");
    CC_REQUIRE((uint64_t)(zoff + shape[0]) * (uint64_t)shape[1] * (uint64_t)shape[2] < (1ull << KEY_BITS),
               "volume too large (>= 2^36 voxels)");
    CC_REQUIRE(g.n_tiles < (1LL << 31), "too many tiles");
    for (int a = 0; a < 3; ++a) {
        hg.tab.insert(hg.tab.end(), st[a].begin(), st[a].end());
        hg.tab.insert(hg.tab.end(), ln[a].begin(), ln[a].end());
        hg.tab.insert(hg.tab.end(), bk[a].begin(), bk[a].end());
    }
    for (int a = 0; a < 3; ++a) {          // block -> first tile, tile count
        std::vector<int32_t> b0(g.nb[a], 0), bn(g.nb[a], 0);
        for (int i = (int)bk[a].size() - 1; i >= 0; --i) { b0[bk[a][i]] = i; bn[bk[a][i]] += 1; }
        hg.tab.insert(hg.tab.end(), b0.begin(), b0.end());
        hg.tab.insert(hg.tab.end(), bn.begin(), bn.end());
    }
    return hg;
}

// point the Geom's table pointers into a device copy of hg.tab
static void bind_geom_tables(HostGeom& hg, int32_t* base) {
    int64_t off = 0;
    for (int a = 0; a < 3; ++a) {
        const int n = hg.g.nt[a];
        hg.g.tstart[a] = base + off;
        hg.g.tlen[a] = base + off + n;
        hg.g.tblk[a] = base + off + 2 * n;
        off += 3 * n;
    }
    for (int a = 0; a < 3; ++a) {
        const int n = hg.g.nb[a];
        hg.g.bt0[a] = base + off;
        hg.g.btn[a] = base + off + n;
        off += 2 * n;
    }
}


}  // namespace cc
