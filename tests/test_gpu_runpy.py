"""scripts/run.py-style workflow on the GPU through instant-ngp-rendering_amd/run.py:
train on a synthetic nerf_synthetic-layout scene, evaluate PSNR/SSIM on held-out views,
save a snapshot and re-evaluate from it, write screenshots."""
import os

import numpy as np
import pytest

import synthetic as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scene(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("runpy_scene"))
    S.write_nerf_synthetic_scene(root, 40, 64, 64, seed=5, split="train")
    S.write_nerf_synthetic_scene(root, 4, 64, 64, seed=99, split="test")
    return root


def test_train_eval_snapshot_screenshot(scene, tmp_path):
    import run as R
    snap = str(tmp_path / "lego_like.ingp")
    shots = str(tmp_path / "shots")
    args = R.parse_args(["--scene", os.path.join(scene, "transforms_train.json"), "--network", "tiny_L4F2.json",
                         "--n_steps", "600", "--test_transforms", os.path.join(scene, "transforms_test.json"),
                         "--save_snapshot", snap, "--eval_spp", "2", "--quiet"])
    res = R.run(args, log=lambda *_: None)
    assert res["training_step"] == 600
    assert res["n_images"] == 4
    assert res["psnr"] > 18.0, res
    assert 0.5 < res["ssim"] <= 1.0
    # evaluation from the snapshot alone reproduces the numbers (same weights, same grid)
    args2 = R.parse_args(["--load_snapshot", snap, "--test_transforms", os.path.join(scene, "transforms_test.json"),
                          "--eval_spp", "2", "--screenshot_transforms", os.path.join(scene, "transforms_test.json"),
                          "--screenshot_frames", "0", "1", "--screenshot_dir", shots, "--screenshot_spp", "1", "--quiet"])
    res2 = R.run(args2, log=lambda *_: None)
    assert "training_step" not in res2
    np.testing.assert_allclose(res2["psnr"], res["psnr"], rtol=1e-4)
    assert sorted(os.listdir(shots)) == ["r_0.png", "r_1.png"]
