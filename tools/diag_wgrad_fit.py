"""Offline (CPU) analysis of the wrong weight-gradient partials captured by tools/diag_wgrad_capture.py:
for every bad (run, slice), which output elements are wrong, and which per-step / per-8-row-chunk
contributions of the kernel's own arithmetic explain the error (least squares per 16-column tile).

  python tools/diag_wgrad_fit.py gpurun_out/r05/capture_x2_40000x6x264.npz
"""
import sys

import numpy as np


def x2_split(v, s):
    """The kernel's P_X2 operand split: hi = RN16(v s), lo = RN16(2^11 (v s - hi))."""
    vs = (v.astype(np.float32) * np.float32(s)).astype(np.float32)
    hi = vs.astype(np.float16).astype(np.float32)
    lo = ((vs - hi) * np.float32(2048)).astype(np.float16).astype(np.float32)
    return hi.astype(np.float64), lo.astype(np.float64)


def main(path):
    z = np.load(path)
    N, K, rows, s = int(z["N"]), int(z["K"]), int(z["rows"]), float(z["dscale"])
    slices = list(z["slices"])
    print(f"{path}: {len(z['bad_run'])} bad partials, slices {slices}, rows per slice {rows}")
    for b, (run, sl) in enumerate(zip(z["bad_run"], z["bad_slice"])):
        i = slices.index(sl)
        dy, x = z["dy_rows"][i], z["x_rows"][i]
        ah, al = x2_split(dy, s)
        bh, bl = x2_split(x, 1.0)
        nst = (rows + 31) // 32
        # the kernel's contribution of every 8-row chunk: hh part and cross part (x 2^-11), scaled by 1/s
        chunks_hh = np.stack([ah[8 * c:8 * c + 8].T @ bh[8 * c:8 * c + 8] for c in range(4 * nst)]) / s
        chunks_x = np.stack([(al[8 * c:8 * c + 8].T @ bh[8 * c:8 * c + 8] + ah[8 * c:8 * c + 8].T @ bl[8 * c:8 * c + 8])
                             for c in range(4 * nst)]) * (2.0 ** -11) / s
        model = chunks_hh.sum(0) + chunks_x.sum(0)
        got = z["bad_part"][b].astype(np.float64)
        err = got - model
        scale = np.abs(model).max()
        bad = np.abs(err) > 1e-5 * scale
        tiles = sorted(set((np.nonzero(bad.any(0))[0] // 16).tolist()))
        nrows = sorted(set(np.nonzero(bad.any(1))[0].tolist()))
        print(f"\nrun {run} slice {sl}: max |err| / max |model| {np.abs(err).max() / scale:.3e}, "
              f"{bad.sum()} wrong of {N * K}; n rows {nrows[:12]}{'...' if len(nrows) > 12 else ''} "
              f"({len(nrows)}), k-tiles {tiles}")
        good_err = np.abs(z['good_part'][i].astype(np.float64) - model).max() / scale
        print(f"   the first run's partial of this slice vs the model: {good_err:.2e}")
        for t in tiles[:6]:
            cols = slice(16 * t, min(K, 16 * t + 16))
            e = err[:, cols].ravel()
            # err = sum_j alpha_j * (chunk j contribution), hh and cross parts separately
            basis = np.concatenate([chunks_hh[:, :, cols].reshape(4 * nst, -1),
                                    chunks_x[:, :, cols].reshape(4 * nst, -1)])
            coef, *_ = np.linalg.lstsq(basis.T, e, rcond=None)
            res = np.abs(basis.T @ coef - e).max() / np.abs(e).max()
            big = [(("hh" if j < 4 * nst else "x") + f" step {(j % (4 * nst)) // 4} chunk {j % 4}", round(c, 3))
                   for j, c in enumerate(coef) if abs(c) > 0.05]
            print(f"   tile {t}: err fit by chunk contributions, residual {res:.3f}: {big[:12]}")
            # err = (tile t' contribution - tile t contribution) of one step: a fragment of another tile
            for tp in range(-(-K // 16)):
                if tp == t:
                    continue
                cp = slice(16 * tp, min(K, 16 * tp + 16))
                if cp.stop - cp.start != cols.stop - cols.start:
                    continue
                for st in range(nst):
                    cand = (chunks_hh[4 * st:4 * st + 4].sum(0) + chunks_x[4 * st:4 * st + 4].sum(0))
                    d = (cand[:, cp] - cand[:, cols]).ravel()
                    r = np.abs(d - e).max() / np.abs(e).max()
                    if r < 0.05:
                        print(f"   tile {t}: err = step {st}'s B of tile {tp} in place of its own (residual {r:.3f})")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
