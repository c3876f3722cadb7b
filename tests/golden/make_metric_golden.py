"""Golden vectors for the evaluation metrics, computed by the reference's own
scripts/common.py (imported read-only from /root/reference in the build container;
`imageio` is not installed here, so a stub module stands in for it -- the metric code
never touches it).  Output: tests/golden/metrics.npz (inputs and expected values).

    python tests/golden/make_metric_golden.py
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SCRIPTS = "/root/reference/scripts"
# MtRSE is left out: the reference compute_error() fails on its scalar map (item assignment)
METRICS = ["MAE", "MAPE", "SMAPE", "MSE", "MScE", "MRSE", "MRScE", "SSIM"]


def main():
    sys.modules.setdefault("imageio", types.ModuleType("imageio"))
    sys.path.insert(0, REF_SCRIPTS)
    import common  # noqa: E402  (reference scripts/common.py)

    rng = np.random.default_rng(71)
    imgs, refs = [], []
    for k in range(4):
        h, w = 23 + 5 * k, 31 + 3 * k
        ref = rng.uniform(0, 1, (h, w, 3)).astype(np.float32)
        img = np.clip(ref + rng.normal(0, 0.05 * (k + 1), ref.shape), -0.1, 1.2).astype(np.float32)
        if k == 3:
            img[0, 0, 0] = np.nan  # non-finite pixels are zeroed by the metric
        imgs.append(img)
        refs.append(ref)
    out = {}
    for k, (img, ref) in enumerate(zip(imgs, refs)):
        out[f"img{k}"] = img
        out[f"ref{k}"] = ref
        for m in METRICS:
            out[f"{m}_{k}"] = np.float64(common.compute_error(m, img.copy(), ref.copy()))
        a = np.clip(common.linear_to_srgb(np.nan_to_num(img)), 0.0, 1.0)
        r = np.clip(common.linear_to_srgb(ref), 0.0, 1.0)
        mse = float(common.compute_error("MSE", a, r))
        out[f"runpy_psnr_{k}"] = np.float64(common.mse2psnr(mse))
        out[f"runpy_ssim_{k}"] = np.float64(common.compute_error("SSIM", a, r))
    x = np.linspace(-0.1, 1.5, 257).astype(np.float32)
    out["srgb_x"] = x
    out["srgb_to_linear"] = common.srgb_to_linear(x)
    out["linear_to_srgb"] = common.linear_to_srgb(np.maximum(x, 0))
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), **out)
    print("wrote", os.path.join(HERE, "metrics.npz"))


if __name__ == "__main__":
    main()
