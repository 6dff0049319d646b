"""Offline (CPU) analysis of the wrong weight-gradient partials captured by tools/diag_wgrad_capture.py:
every wrong (run, slice) partial is fit, by least squares, as a sum of single staging loads that returned
zero -- one load = one row m of the slice (step m // 32, chunk (m % 32) // 8, row i = m % 8) over one
16-lane group of columns (a B k-tile) or over the dY columns (A).  A residual ~1e-6 of the error means the
partial is explained exactly.  Used for DESIGN.md section 4, "The k_wgrad_rect zeros".

  python tools/diag_wgrad_fit.py gpurun_out/r05/capture_wg_soff2.npz [N_SHOW]
"""
import sys

import numpy as np


def main(path, nshow=12):
    z = np.load(path)
    N, K, rows = int(z["N"]), int(z["K"]), int(z["rows"])
    slices = list(z["slices"])
    nst = rows // 32
    print(f"{path}: {len(z['bad_run'])} bad partials kept, slices {slices}, rows per slice {rows}")
    for b in range(min(nshow, len(z["bad_run"]))):
        i = slices.index(z["bad_slice"][b])
        dy, x = z["dy_rows"][i].astype(np.float64), z["x_rows"][i].astype(np.float64)
        got = z["bad_part"][b].astype(np.float64)
        err = got - dy.T @ x
        bad = np.abs(err) > 1e-5 * np.abs(dy.T @ x).max()
        tiles = sorted(set((np.nonzero(bad.any(0))[0] // 16).tolist()))
        out = []
        if len(tiles) <= 4:  # B loads: per k-tile, which rows of which chunk lost their value
            for t in tiles:
                cols = slice(16 * t, 16 * t + 16)
                e = err[:, cols].ravel()
                best = None
                for c in range(4):
                    ms = [32 * st + 8 * c + r for st in range(nst) for r in range(8)]
                    basis = np.array([-np.outer(dy[m], x[m, cols]).ravel() for m in ms]).T
                    coef, *_ = np.linalg.lstsq(basis, e, rcond=None)
                    res = np.abs(basis @ coef - e).max() / np.abs(e).max()
                    if best is None or res < best[0]:
                        best = (res, c, [(ms[k] // 32, ms[k] % 8, round(float(coef[k]), 3))
                                         for k in np.nonzero(np.abs(coef) > 0.05)[0]])
                out.append(f"B k-tile {t}: chunk {best[1]}, zeroed (step, row, coef) {best[2]}, residual {best[0]:.1e}")
        else:  # A loads (dY, all columns): rows of chunk 3 (lanes 48-63 of wave 0)
            e = err.ravel()
            best = None
            for c in range(4):
                ms = [32 * st + 8 * c + r for st in range(nst) for r in range(8)]
                basis = np.array([-np.outer(dy[m], x[m]).ravel() for m in ms]).T
                coef, *_ = np.linalg.lstsq(basis, e, rcond=None)
                res = np.abs(basis @ coef - e).max() / np.abs(e).max()
                if best is None or res < best[0]:
                    best = (res, c, [(ms[k] // 32, ms[k] % 8, round(float(coef[k]), 3))
                                     for k in np.nonzero(np.abs(coef) > 0.05)[0]])
            out.append(f"A: chunk {best[1]}, zeroed (step, row, coef) {best[2]}, residual {best[0]:.1e}")
        print(f"run {z['bad_run'][b]} slice {z['bad_slice'][b]}: " + "; ".join(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
