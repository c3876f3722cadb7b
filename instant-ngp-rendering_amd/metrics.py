"""Image error metrics of the reference's evaluation harness (scripts/common.py:49,139-263,
used by scripts/run.py:210-268): PSNR from MSE, a 5-tap Gaussian SSIM on luminance, and
the relative/absolute error maps.  Numpy only; parity with the reference implementation
is pinned by tests/golden/metrics.npz (tests/golden/make_metric_golden.py).
FLIP is not provided (not part of the path's evaluation: run.py reports PSNR and SSIM).
"""
import numpy as np
from scipy.ndimage import convolve1d

# 5-tap separable Gaussian the reference SSIM blurs with (scripts/common.py:190-193)
_SSIM_TAPS = np.array([0.120078, 0.233881, 0.292082, 0.233881, 0.120078])
_C1, _C2 = 0.01 ** 2, 0.03 ** 2


def mse2psnr(mse):
    return -10.0 * np.log(mse) / np.log(10.0)


def srgb_to_linear(x):
    x = np.asarray(x)
    return np.where(x > 0.04045, np.power((x + 0.055) / 1.055, 2.4), x / 12.92)


def linear_to_srgb(x):
    x = np.asarray(x)
    return np.where(x > 0.0031308, 1.055 * np.power(x, 1.0 / 2.4) - 0.055, 12.92 * x)


def luminance(img):
    return 0.2126 * img[..., 0] + 0.7152 * img[..., 1] + 0.0722 * img[..., 2]


def _blur(x):
    return convolve1d(convolve1d(x, _SSIM_TAPS, axis=0), _SSIM_TAPS, axis=1)


def ssim_map(img, ref):
    """Per-pixel SSIM of the luminances (inputs clipped to [0, 1] by the caller)."""
    a, b = luminance(img), luminance(ref)
    ma, mb = _blur(a), _blur(b)
    va = _blur(a * a) - ma * ma
    vb = _blur(b * b) - mb * mb
    cov = _blur(a * b) - ma * mb
    return ((2.0 * ma * mb + _C1) / (ma * ma + mb * mb + _C1)) * ((2.0 * cov + _C2) / (va + vb + _C2))


def _trimmed_mean(x, skip=1e-6):
    x = np.sort(x.ravel())
    k = int(skip * x.size)
    return x[k:x.size - k].mean()


def error_map(metric, img, ref):
    img = np.where(np.isfinite(img), img, 0.0)
    img = np.maximum(img, 0.0)
    if metric == "MAE":
        return np.abs(img - ref)
    if metric == "MAPE":
        return np.abs(img - ref) / (1e-2 + ref)
    if metric == "SMAPE":
        return np.abs(img - ref) / (1e-2 + (ref + img) / 2.0)
    if metric == "MSE":
        return (img - ref) ** 2
    if metric == "MScE":
        return (np.clip(img, 0.0, 1.0) - np.clip(ref, 0.0, 1.0)) ** 2
    if metric == "MRSE":
        return (img - ref) ** 2 / (1e-2 + ref ** 2)
    if metric == "MtRSE":
        return _trimmed_mean((img - ref) ** 2 / (1e-2 + ref ** 2))
    if metric == "MRScE":
        ic, rc = np.clip(img, 0, 100), np.clip(ref, 0, 100)
        return (ic - rc) ** 2 / (1e-2 + rc ** 2)
    if metric == "SSIM":
        return ssim_map(np.clip(img, 0.0, 1.0), np.clip(ref, 0.0, 1.0))
    raise ValueError(f"Unknown metric: {metric}.")


def compute_error(metric, img, ref):
    m = np.asarray(error_map(metric, np.array(img, copy=True), np.asarray(ref)))
    m = np.where(np.isfinite(m), m, 0.0)
    if m.ndim == 3:
        m = m.mean(axis=2)
    return float(np.mean(m))


def psnr_ssim(image_linear, ref_linear):
    """The run.py test-set metric pair on sRGB-clamped RGB (scripts/run.py:248-253)."""
    a = np.clip(linear_to_srgb(image_linear[..., :3]), 0.0, 1.0)
    r = np.clip(linear_to_srgb(ref_linear[..., :3]), 0.0, 1.0)
    mse = compute_error("MSE", a, r)
    return mse2psnr(mse), compute_error("SSIM", a, r), mse
