// Driver of the statistics-kernel emulation (tests/test_stats_emulated.py): reads two fp32 images and
// a case from argv, runs custma::launch_stats on the host, writes every output array.
// usage: stats_emu <in.bin> <out.bin> H W k mode rows h_lo h_hi
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "common.h"

int main(int argc, char** argv) {
    if (argc != 10) return 2;
    const int64_t H = atoll(argv[3]), W = atoll(argv[4]);
    const int k = atoi(argv[5]), mode = atoi(argv[6]), rows = atoi(argv[7]);
    const int64_t n = H * W;
    std::vector<float> img(2 * n), shift(2);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(img.data(), 4, 2 * n, f) != (size_t)(2 * n) || fread(shift.data(), 4, 2, f) != 2) return 3;
    fclose(f);
    custma::Geo g;
    memset(&g, 0, sizeof g);
    g.H = H; g.W = W; g.k = k; g.r = k / 2; g.layout = CUSTMA_LAYOUT_WINDOW; g.D = 0; g.WO = W; g.DO = 1;
    g.h_lo = atoll(argv[8]);
    g.h_hi = atoll(argv[9]);
    // outputs pre-filled with a NaN pattern: an element a mode must not write stays NaN
    std::vector<float> mean(2 * n, NAN), sq(2 * n, NAN), sqt(2 * n, NAN), prep(6 * n, NAN);
    std::vector<double> box(2 * n, NAN);
    custma::Stats st[2];
    for (int i = 0; i < 2; ++i) st[i] = custma::Stats{mean.data() + i * n, sq.data() + i * n, box.data() + i * n,
                                                      sqt.data() + i * n};
    const int e = custma::launch_stats(img.data(), img.data() + n, CUSTMA_F32, g, st[0], st[1], nullptr, mode,
                                       prep.data(), shift.data(), rows);
    if (e) return 4;
    f = fopen(argv[2], "wb");
    if (!f) return 5;
    fwrite(mean.data(), 4, 2 * n, f);
    fwrite(sq.data(), 4, 2 * n, f);
    fwrite(box.data(), 8, 2 * n, f);
    fwrite(sqt.data(), 4, 2 * n, f);
    fwrite(prep.data(), 4, 6 * n, f);
    fclose(f);
    return 0;
}
