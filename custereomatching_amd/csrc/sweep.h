// Shared geometry of the sliding-window ("sweep") kernels.
#pragma once
#include "common.h"

namespace custma {

constexpr int TW = 16;  // camera (own-image) columns per workgroup

// Kernel sizes with a compile-time sweep instantiation (register-resident
// column sums need a static trip count).  Other odd sizes up to
// CUSTMA_MAX_KERNEL run on the exact kernel.
#define CUSTMA_SWEEP_KS(X) X(1) X(3) X(5) X(7) X(9) X(11) X(13) X(15)

struct SweepGrid {
    int nChunk;  // disparity-diagonal chunks per column tile
    int nTile;   // column tiles of TW
    int nBand;   // row bands
    int TH;      // rows per band
    int NL;      // lanes (diagonals) per workgroup = blockDim.x
};

struct DispPartial {
    float* best;     // [nChunk][HV][WO]
    float* second;   // [nChunk][HV][WO]
    int32_t* index;  // [nChunk][HV][WO] layout index s of best, -1 if none
};

inline SweepGrid sweep_grid(const Geo& g) {
    SweepGrid sg;
    if (g.layout == CUSTMA_LAYOUT_WINDOW) {
        const int64_t nd = (int64_t)g.D + 1;
        int nw = (int)cdiv(nd, 64);
        if (nw > 5) nw = 4;
        sg.NL = 64 * nw;
        sg.nChunk = (int)cdiv(nd, sg.NL);
    } else {
        sg.NL = 256;
        sg.nChunk = (int)cdiv(g.W + TW - 1, sg.NL);
    }
    sg.nTile = (int)cdiv(g.WO, TW);
    sg.TH = 64;
    // keep >= ~4 workgroups per CU on small problems
    while (sg.TH > 8 && (int64_t)sg.nTile * sg.nChunk * cdiv(g.HV(), sg.TH) < 2048) sg.TH /= 2;
    sg.nBand = (int)cdiv(g.HV(), sg.TH);
    return sg;
}

inline int64_t sweep_blocks(const SweepGrid& sg) { return (int64_t)sg.nBand * sg.nTile * sg.nChunk; }

hipError_t launch_disp_partials(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                                DispPartial part, hipStream_t s);

}  // namespace custma
