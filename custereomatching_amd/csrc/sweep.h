// Shared geometry of the sliding-window ("sweep") kernels.
#pragma once
#include <stdlib.h>

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
    int NL;      // lanes per workgroup = blockDim.x
    int TD;      // diagonals per lane (forward sweep); a chunk covers TD * NL diagonals
};

struct DispPartial {
    float* best;     // [nChunk][HV][WO]
    float* second;   // [nChunk][HV][WO]
    int32_t* index;  // [nChunk][HV][WO] layout index s of best, -1 if none
};

// Lane / chunk geometry.  td_max = 2 for the forward sweep (two diagonals
// per lane), 1 for the backward.  The diagonal range of a column tile is
// split into chunks of TD * NL; the choice minimises idle lanes.
inline SweepGrid sweep_grid(const Geo& g, int td_max = 1) {
    SweepGrid sg;
    const int64_t nd = g.layout == CUSTMA_LAYOUT_WINDOW ? (int64_t)g.D + 1 : g.W + TW - 1;
    // cost = diagonal slots launched, discounted for two diagonals per lane (half the LDS
    // bytes per voxel) and penalised for single-wave workgroups
    double best = 1e300;
    sg.NL = 256; sg.TD = 1;
    // tuning overrides (benchmarking only): CUSTMA_SWEEP_TD, CUSTMA_SWEEP_NW
    const char* etd = getenv("CUSTMA_SWEEP_TD");
    const char* enw = getenv("CUSTMA_SWEEP_NW");
    const int td_fix = etd ? atoi(etd) : 0, nw_fix = enw ? atoi(enw) : 0;
    for (int td = 1; td <= td_max; ++td)
        for (int nw = 1; nw <= (g.layout == CUSTMA_LAYOUT_WINDOW ? 5 : 4); ++nw) {
            if ((td_fix && td != td_fix) || (nw_fix && nw != nw_fix)) continue;
            const int64_t per = (int64_t)64 * nw * td;
            const double cost = (double)(cdiv(nd, per) * per) * (td == 2 ? 0.8 : 1.0) * (nw == 1 ? 1.1 : 1.0);
            if (cost < best) { best = cost; sg.NL = 64 * nw; sg.TD = td; }
        }
    sg.nChunk = (int)cdiv(nd, (int64_t)sg.NL * sg.TD);
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
