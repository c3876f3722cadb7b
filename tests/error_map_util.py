"""Host-side pieces of the error-map CDF update shared by the error-map tests: the image
CDF normalisation the reference runs on the CPU (src/testbed_nerf.cu:2553-2567) and a
numpy restatement of construct_cdf_2d / construct_cdf_1d (:1493-1546)."""
import numpy as np

MIN_PDF = np.float32(0.01)
MIN_PMF = np.float32(0.1)


def build_cdf_numpy(err):
    """err: [n_images][ry][rx] f32 -> (cdf_x_cond_y, cdf_y, cdf_img unnormalised)."""
    err = np.asarray(err, np.float32)
    n, ry, rx = err.shape
    cx = np.cumsum(err + np.float32(1e-10), axis=2, dtype=np.float32)
    row = cx[:, :, -1].copy()
    norm = (np.float32(1.0) / row)[:, :, None]
    xs = (np.arange(1, rx + 1, dtype=np.float32) / np.float32(rx))[None, None, :]
    cx = (np.float32(1.0) - MIN_PDF) * cx * norm + MIN_PDF * xs
    cy = np.cumsum(row, axis=1, dtype=np.float32)
    tot = cy[:, -1].copy()
    ys = (np.arange(1, ry + 1, dtype=np.float32) / np.float32(ry))[None, :]
    cy = (np.float32(1.0) - MIN_PDF) * cy * (np.float32(1.0) / tot)[:, None] + MIN_PDF * ys
    return cx.astype(np.float32), cy.astype(np.float32), tot.astype(np.float32)


def normalise_image_cdf(totals):
    """pmf_img and the normalised image CDF from the per-image totals (CPU step of the reference)."""
    totals = np.asarray(totals, np.float32)
    n = totals.size
    cum = np.float32(0.0)
    cdf = np.zeros(n, np.float32)
    for i in range(n):
        cum = np.float32(cum + totals[i])
        cdf[i] = cum
    norm = np.float32(1.0) / cum
    pmf = (np.float32(1.0) - MIN_PMF) * totals * norm + MIN_PMF / np.float32(n)
    cdf = (np.float32(1.0) - MIN_PMF) * cdf * norm + MIN_PMF * np.arange(1, n + 1, dtype=np.float32) / np.float32(n)
    return pmf.astype(np.float32), cdf.astype(np.float32)
