"""Oracle checks of large window-layout problems on haloed (row x column) tiles -- test
infrastructure (the fp64 oracle, oracle/zncc_oracle.c, on a crop)."""
from oracle import oracle as O


def tile_backward(g, cam, proj, k, D, h0, h1, c0, wc):
    """fp64 oracle gradients of image rows [h0, h1) on the columns a [h0-2r, h1+2r) x [c0, c0+wc)
    crop of a window-layout problem determines exactly: a crop voxel (h, w, s) is the image's
    voxel (h, c0 + w, s) wherever both patches stay inside the crop (or meet the image's own
    edges) and the voxel's camera column is inside the crop's window volume (< c0 + wc - D), so
    camera columns [c0 + 2r, c0 + wc - D - 2r) and projector columns [c0 + D + 2r, c0 + wc - D - 2r)
    (no margin at an image edge) only see exact voxels.
    Returns the two gradient tiles and their global column ranges."""
    H, W = cam.shape
    r = k // 2
    a0, a1 = max(0, h0 - 2 * r), min(H, h1 + 2 * r)
    e = c0 + wc
    gt = g[a0:a1, c0:e - D]
    gt = gt.cpu().numpy() if hasattr(gt, "cpu") else gt
    rc, rp = O.backward_f64(gt, cam[a0:a1, c0:e], proj[a0:a1, c0:e], k, layout=O.WINDOW, D=D)
    lo = c0 if c0 == 0 else c0 + 2 * r
    hi_c = W if e == W else e - D - 2 * r
    lo_p = c0 if c0 == 0 else c0 + D + 2 * r
    hi_p = W if e == W else e - D - 2 * r
    return (rc[h0 - a0:h1 - a0, lo - c0:hi_c - c0], rp[h0 - a0:h1 - a0, lo_p - c0:hi_p - c0],
            (lo, hi_c), (lo_p, hi_p))
