"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

    python tests/golden/make_golden.py

The reference cannot run here (CUDA sources, empty tiny-cuda-nn submodule),
so these vectors are produced by the oracle restatement: they pin the oracle against
regressions (tests/test_oracle.py) and the HIP path against the oracle on the GPU
(tests/test_gpu_golden.py) without re-running the oracle there.  Inputs are seeded;
large arrays (parameters, occupancy grids) are regenerated from their seeds by
tests/golden_util.py and only digests / samples of the big outputs are stored.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(os.path.dirname(HERE)), "instant-ngp-rendering_amd")]

import ngp_abi as A  # noqa: E402
import golden_util as G  # noqa: E402
from oracle_abi import Oracle, load, ptr  # noqa: E402


def encode_fixture(name, cfg_kw, n=512, seed=11):
    o = Oracle(A.default_config(**cfg_kw))
    o.set_params(G.seeded_params(o.n_params, o.n_mlp, seed))
    pos = G.seeded_positions(n, seed + 1)
    idx, w = o.encode_indices(pos)
    feat = o.encode(pos)
    np.savez_compressed(os.path.join(HERE, f"encode_{name}.npz"), cfg=json.dumps(cfg_kw), params_seed=seed, pos=pos,
                        idx=idx, w=w, feat=feat)


def mlp_fixture(name, cfg_kw, n=256, seed=21):
    o = Oracle(A.default_config(**cfg_kw))
    o.set_params(G.seeded_params(o.n_params, o.n_mlp, seed, mlp_scale=0.25, grid_scale=0.5))
    coords = G.seeded_coords(n, seed + 1)
    out = o.infer(coords)
    dens = o.density(coords[:, :3])
    enc = o.encode(coords[:, :3])
    rng = np.random.default_rng(seed + 2)
    dloss = rng.normal(0, 1, (n, 4)).astype(np.float16)
    denc = o.backward(enc, coords[:, 4:7], dloss)
    grads = o.get(A.GRADS_FP32)[: o.n_mlp].copy()
    np.savez_compressed(os.path.join(HERE, f"mlp_{name}.npz"), cfg=json.dumps(cfg_kw), params_seed=seed, coords=coords,
                        out=out, density=dens, dloss=dloss, denc=denc, mlp_grads=grads)


def sh_fixture(n=256, seed=31):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    out = np.zeros((n, 16), np.float32)
    lib = load()
    for i in range(n):
        o16 = np.zeros(16, np.float32)
        lib.oref_sh4(ptr(np.ascontiguousarray(d[i])), ptr(o16))
        out[i] = o16
    np.savez_compressed(os.path.join(HERE, "sh4.npz"), dirs=d, sh=out)


def bitfield_fixture(seed=41):
    o = Oracle(A.default_config(**G.CFG_A))
    grid = G.seeded_grid(seed)
    o.grid_set(grid)
    o.grid_bitfield(0)
    _, bits, mean = o.grid_get(G.CELLS)
    np.savez_compressed(os.path.join(HERE, "bitfield.npz"), grid_seed=seed, mean=np.float32(mean),
                        sha256=G.digest(bits), head=bits[:4096], mip1=bits[G.CELLS // 8: G.CELLS // 8 + 4096])


def train_fixture(seed=51):
    imgs, cams, focal = G.golden_views()
    o = Oracle(A.default_config(**G.CFG_A))
    o.set_params(G.seeded_params(o.n_params, o.n_mlp, seed))
    o.grid_set(G.sphere_grid())
    o.grid_bitfield(0)
    hd = G.host_dataset(imgs, cams, focal)
    R, B, MS = 64, 4096, 1 << 14
    o.train_step(G.golden_train_args(hd.ptr, hd.n, R, B, MS))
    st = o.stats()
    ns = o.scratch(A.SCRATCH_RAY_NUMSTEPS, np.uint32).reshape(-1, 2)
    coords = o.scratch(A.SCRATCH_COORDS, np.float32).reshape(-1, 8)[: st.measured_batch_size_before_compaction]
    cp = o.scratch(A.SCRATCH_RAY_COMPACTED, np.uint32).reshape(-1, 2)
    C_ = min(st.measured_batch_size, B)
    dl = o.scratch(A.SCRATCH_DLOSS, np.float16).reshape(-1, 4)[:C_]
    np.savez_compressed(os.path.join(HERE, "train_A.npz"), imgs=imgs, cams=cams, focal=np.float32(focal),
                        params_seed=seed, R=R, B=B, MS=MS, numsteps=ns, coords=coords, compacted=cp, dloss=dl,
                        loss=np.float32(st.loss), n_before=st.measured_batch_size_before_compaction,
                        n_after=st.measured_batch_size)


def render_fixture(seed=61):
    o = Oracle(A.default_config(**G.CFG_A))
    o.set_params(G.seeded_params(o.n_params, o.n_mlp, seed, grid_scale=1.0))
    o.grid_set(G.sphere_grid(0.3))
    o.grid_bitfield(0)
    ra = G.golden_render_args()
    frame, depth = o.render(ra)
    np.savez_compressed(os.path.join(HERE, "render_A.npz"), params_seed=seed, frame=frame, depth=depth)


def main():
    os.makedirs(HERE, exist_ok=True)
    encode_fixture("L16F2T19", dict(n_levels=16, F=2, log2_T=19))
    encode_fixture("L8F4T19", dict(n_levels=8, F=4, log2_T=19))
    encode_fixture("L4F2T14", dict(n_levels=4, F=2, log2_T=14, n_neurons=16))
    encode_fixture("L16F2T22A64", dict(n_levels=16, F=2, log2_T=22, aabb_scale=64))
    mlp_fixture("A", G.CFG_A)
    mlp_fixture("B", G.CFG_B)
    sh_fixture()
    bitfield_fixture()
    train_fixture()
    render_fixture()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
