"""Helpers for the GPU parity tests: drive libngp_hip.so through its C-ABI with
torch tensors as plain device memory (plumbing only)."""
import ctypes as C

import numpy as np
import torch

import ngp_abi as A


def dev(x, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def vp(t):
    return C.c_void_p(t.data_ptr())


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class GpuModel:
    def __init__(self, cfg, seed=1337):
        self.lib = A.load()
        self.cfg = cfg
        self.h = C.c_void_p()
        A.check(self.lib.ngp_model_create(0, C.byref(cfg), seed, C.byref(self.h)))
        self.info = A.ModelInfo()
        A.check(self.lib.ngp_model_get_info(self.h, C.byref(self.info)))
        self.n_params = int(self.info.n_params)
        self.n_mlp = int(self.info.n_mlp_params)
        self.L = cfg.n_levels
        self.F = cfg.n_features_per_level

    def set_tuning(self, **kw):
        """ngp_model_set_tuning (launch shapes / march schedule; 0 = default)."""
        t = A.Tuning()
        A.check(self.lib.ngp_model_get_tuning(self.h, C.byref(t)))
        for k, v in kw.items():
            setattr(t, k, v)
        A.check(self.lib.ngp_model_set_tuning(self.h, C.byref(t)))

    def close(self):
        if self.h:
            torch.cuda.synchronize()
            A.check(self.lib.ngp_model_destroy(self.h))
            self.h = None

    def buffer(self, kind):
        p = C.c_void_p()
        n = C.c_size_t()
        A.check(self.lib.ngp_model_buffer(self.h, kind, C.byref(p), C.byref(n)))
        return p.value, n.value

    def set_params(self, params, reset=True):
        params = np.ascontiguousarray(params, np.float32)
        assert params.size == self.n_params
        ptr, nbytes = self.buffer(A.PARAMS_FP32)
        cuda_memcpy_h2d(ptr, params)
        A.check(self.lib.ngp_model_params_updated(self.h, int(reset), stream()))
        torch.cuda.synchronize()

    def get(self, kind, n=None):
        ptr, nbytes = self.buffer(kind)
        dt = np.uint16 if kind in (A.PARAMS_FP16, A.PARAMS_INFER_FP16, A.GRADS_GRID_FP16) else np.float32
        out = np.zeros(nbytes // np.dtype(dt).itemsize, dt)
        torch.cuda.synchronize()
        cuda_memcpy_d2h(out, ptr)
        return out

    def zero_grads(self):
        for kind in (A.GRADS_FP32, A.GRADS_GRID_FP16):
            ptr, nbytes = self.buffer(kind)
            cuda_memset(ptr, nbytes)

    def grads(self):
        """All gradients in parameter order as fp32: MLP (fp32 buffer) + hash grid (fp16 buffer)."""
        g = self.get(A.GRADS_FP32)
        g[self.n_mlp:] = self.get(A.GRADS_GRID_FP16).view(np.float16).astype(np.float32)
        return g

    def set_grads(self, grads):
        """Write fp32 MLP gradients and fp16 grid gradients; returns what the device holds (fp32)."""
        grads = np.ascontiguousarray(grads, np.float32)
        p, _ = self.buffer(A.GRADS_FP32)
        g32 = grads.copy()
        g32[self.n_mlp:] = 0.0  # the fp32 buffer's grid part is unused
        cuda_memcpy_h2d(p, g32)
        g16 = grads[self.n_mlp:].astype(np.float16)
        p16, _ = self.buffer(A.GRADS_GRID_FP16)
        cuda_memcpy_h2d(p16, g16.view(np.uint16))
        out = grads.copy()
        out[self.n_mlp:] = g16.astype(np.float32)
        return out

    def encode(self, pos, use_inf=False):
        pos = np.ascontiguousarray(pos, np.float32)
        n, stride = pos.shape
        p = dev(pos)
        enc = torch.zeros(self.L * n * self.F, dtype=torch.float16, device="cuda")
        A.check(self.lib.ngp_model_encode(self.h, vp(p), stride, n, vp(enc), int(use_inf), stream()))
        torch.cuda.synchronize()
        return enc.cpu().numpy().reshape(self.L, n, self.F)

    def encode_indices(self, pos):
        pos = np.ascontiguousarray(pos, np.float32)
        n, stride = pos.shape
        p = dev(pos)
        idx = torch.zeros(n * self.L * 8, dtype=torch.int32, device="cuda")
        w = torch.zeros(n * self.L * 8, dtype=torch.float32, device="cuda")
        A.check(self.lib.ngp_model_encode_indices(self.h, vp(p), stride, n, vp(idx), vp(w), stream()))
        torch.cuda.synchronize()
        return idx.cpu().numpy().view(np.uint32).reshape(n, self.L, 8), w.cpu().numpy().reshape(n, self.L, 8)

    def infer(self, coords, use_inf=False):
        coords = np.ascontiguousarray(coords, np.float32)
        n, fpc = coords.shape
        c = dev(coords)
        out = torch.zeros(n * 4, dtype=torch.float16, device="cuda")
        A.check(self.lib.ngp_model_infer(self.h, vp(c), fpc, n, vp(out), int(use_inf), stream()))
        torch.cuda.synchronize()
        return out.float().cpu().numpy().reshape(n, 4)

    def infer_padded(self, coords, layout_rm, use_inf=False, pad=0):
        """ngp_model_infer_padded: [n][16] (column-major, stride 16 + pad) or [16][n + pad] (row-major),
        returned as [n][16]."""
        coords = np.ascontiguousarray(coords, np.float32)
        n, fpc = coords.shape
        c = dev(coords)
        stride = n + pad if layout_rm else 16 + pad
        out = torch.full(((16 if layout_rm else n) * stride,), float("nan"), dtype=torch.float16, device="cuda")
        A.check(self.lib.ngp_model_infer_padded(self.h, vp(c), fpc, n, vp(out), stride, int(layout_rm), int(use_inf),
                                                stream()))
        torch.cuda.synchronize()
        o = out.float().cpu().numpy()
        return o.reshape(16, stride)[:, :n].T.copy() if layout_rm else o.reshape(n, stride)[:, :16].copy()

    def density(self, pos, use_inf=False):
        pos = np.ascontiguousarray(pos, np.float32)
        n, stride = pos.shape
        p = dev(pos)
        out = torch.zeros(n, dtype=torch.float16, device="cuda")
        A.check(self.lib.ngp_model_density(self.h, vp(p), stride, n, vp(out), int(use_inf), stream()))
        torch.cuda.synchronize()
        return out.float().cpu().numpy()

    def backward(self, enc16, dirs, dloss16, weight=None):
        n = dirs.shape[0]
        e = dev(enc16.astype(np.float16))
        d = dev(np.ascontiguousarray(dirs, np.float32))
        dl = dev(dloss16.astype(np.float16))
        w = None if weight is None else dev(np.ascontiguousarray(weight, np.float32))
        denc = torch.zeros(self.L * n * self.F, dtype=torch.float16, device="cuda")
        A.check(self.lib.ngp_model_backward(self.h, vp(e), vp(d), n, vp(dl), None if w is None else vp(w), vp(denc),
                                            stream()))
        torch.cuda.synchronize()
        return denc.float().cpu().numpy().reshape(self.L, n, self.F)

    def backward_extra(self, enc16, dirs, extra, dloss16, weight=None):
        """ngp_model_backward_extra: extra [n][<= EXTRA_ROW] (padded to rows of A.EXTRA_ROW);
        returns (dL/denc, dL/dextra [n][A.EXTRA_ROW])."""
        n = dirs.shape[0]
        e = dev(enc16.astype(np.float16))
        d = dev(np.ascontiguousarray(dirs, np.float32))
        xr = np.zeros((n, A.EXTRA_ROW), np.float32)
        xr[:, :extra.shape[1]] = extra
        x = dev(xr)
        dl = dev(dloss16.astype(np.float16))
        w = None if weight is None else dev(np.ascontiguousarray(weight, np.float32))
        denc = torch.zeros(self.L * n * self.F, dtype=torch.float16, device="cuda")
        dx = torch.zeros(n * A.EXTRA_ROW, dtype=torch.float32, device="cuda")
        A.check(self.lib.ngp_model_backward_extra(self.h, vp(e), vp(d), vp(x), n, vp(dl), None if w is None else vp(w),
                                                  vp(denc), vp(dx), stream()))
        torch.cuda.synchronize()
        return denc.float().cpu().numpy().reshape(self.L, n, self.F), dx.cpu().numpy().reshape(n, A.EXTRA_ROW)

    def encode_backward(self, pos, denc16):
        pos = np.ascontiguousarray(pos, np.float32)
        p = dev(pos)
        d = dev(denc16.astype(np.float16))
        A.check(self.lib.ngp_model_encode_backward(self.h, vp(p), pos.shape[1], pos.shape[0], vp(d), stream()))
        torch.cuda.synchronize()


_hip = None


def _hiplib():
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    return _hip


def cuda_copy(dst, src, nbytes):
    torch.cuda.synchronize()
    assert _hiplib().hipMemcpy(C.c_void_p(dst), C.c_void_p(src), nbytes, 3) == 0  # D2D


def cuda_memcpy_d2h(out, src):
    torch.cuda.synchronize()
    assert _hiplib().hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(src), out.nbytes, 2) == 0


def cuda_memcpy_h2d(dst, arr):
    torch.cuda.synchronize()
    arr = np.ascontiguousarray(arr)
    assert _hiplib().hipMemcpy(C.c_void_p(dst), arr.ctypes.data_as(C.c_void_p), arr.nbytes, 1) == 0


def cuda_memset(dst, nbytes):
    torch.cuda.synchronize()
    assert _hiplib().hipMemset(C.c_void_p(dst), 0, nbytes) == 0


def random_params(n_params, n_mlp, info, rng, grid_scale=0.5):
    p = np.zeros(n_params, np.float32)
    for l in range(info.n_layers):
        fan_in, fan_out = info.layer_in[l], info.layer_out[l]
        s = np.sqrt(6.0 / (fan_in + fan_out))
        off = info.layer_param_offset[l]
        p[off:off + fan_in * fan_out] = rng.uniform(-s, s, fan_in * fan_out)
    p[n_mlp:] = rng.uniform(-grid_scale, grid_scale, n_params - n_mlp)
    return p
