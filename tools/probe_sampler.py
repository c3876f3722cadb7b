"""Probe: training-sampler time vs ray count and occupancy (diagnostic, GPU)."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), os.path.join(ROOT, "tests")]
import ngp_abi as A
from gpu_util import GpuModel, cuda_memcpy_h2d, random_params, stream
from scene_util import DeviceDataset, make_views, train_args, sphere_bitfield

cfg = A.default_config()
g = GpuModel(cfg)
rng = np.random.default_rng(0)
g.set_params(random_params(g.n_params, g.n_mlp, g.info, rng, 0.5))
imgs, cams, focal = make_views(16, 64, 64)
dd = DeviceDataset(imgs, cams, focal)
lib = g.lib
A.check(lib.ngp_timing_enable(g.h, -1))
CELLS = 128 ** 3
for name, grid in [("full", np.ones(CELLS, np.float32)), ("sphere0.3", sphere_bitfield(0.3)),
                   ("sphere0.1", sphere_bitfield(0.1)), ("empty", np.zeros(CELLS, np.float32))]:
    gp, bp, tp, mp = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
    A.check(lib.ngp_density_grid_bitfield(g.h, 0, stream()))
    A.check(lib.ngp_density_grid_buffers(g.h, C.byref(gp), C.byref(bp), C.byref(tp), C.byref(mp)))
    cuda_memcpy_h2d(gp.value, grid.astype(np.float32))
    A.check(lib.ngp_density_grid_bitfield(g.h, 0, stream()))
    torch.cuda.synchronize()
    for R in (1024, 8192, 32768, 131072):
        ta = train_args(dd.ptr, dd.n, R, 1 << 18, 1 << 22)
        for rep in range(3):
            g.zero_grads()
            A.check(lib.ngp_train_step(g.h, C.byref(ta), stream()))
            st = A.TrainStats()
            A.check(lib.ngp_train_read_stats(g.h, C.byref(st), stream()))
            res = {}
            for tname in ("train_sampler", "train_loss", "train_encode", "train_encode_bwd"):
                ms, u, n = C.c_double(), C.c_uint64(), C.c_uint32()
                A.check(lib.ngp_timing_read(g.h, A.TIMER[tname], C.byref(ms), C.byref(u), C.byref(n), 1))
                res[tname] = ms.value
        print(f"{name:10s} R={R:7d} samples={st.measured_batch_size_before_compaction:9d} " +
              " ".join(f"{k}={v*1000:8.1f}us" for k, v in res.items()), flush=True)
g.close()
