"""Data-parallel retry probe (diagnostic, GPU box): four host-staged ranks on one GPU train the DP test
scene in deterministic mode with ngp_tuning.debug bits 0 (no retries), 4 (forced early-stop violations:
full forward from the first step), 8 (forced sample-capacity overflows) and 12 (both); per step every
rank records a checksum of its parameters, density grid and batch statistics, and the first step where a
variant departs from the retry-free run is printed.
Usage: python tools/dp_retry_probe.py [--steps 24] [--world 4]"""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "instant-ngp-rendering_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import synthetic as S  # noqa: E402
import test_gpu_distributed as T  # noqa: E402


def worker(rank, world, port, scene, q, debug, steps, config):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tb = T._testbed(scene, config)
        if debug:
            tb.set_tuning({"debug": debug})
        tb.init_distributed_host(rank, world, T._host_allreduce(dist))
        tb.deterministic = True
        tb.shall_train = True
        rec = []
        full = {}
        while tb.training_step < steps:
            tb.frame()
            p = T._params(tb)
            st = tb.last_train_stats()
            rec.append((tb.training_step, float(np.sum(p, dtype=np.float64)), float(np.abs(p).sum(dtype=np.float64)),
                        float(np.sum(tb.density_grid(), dtype=np.float64)), int(st["measured_batch_size"]),
                        int(st["measured_batch_size_before_compaction"]), float(st["loss"]),
                        int(st["forward_early_stop_violations_total"]), int(st.get("sample_capacity_overflow", 0))))
            if rank == 0 and tb.training_step in (2, 3, 4):
                full[tb.training_step] = p
        q.put(dict(rank=rank, rec=rec, full=full, n_mlp=T._n_mlp(tb)))
    finally:
        dist.destroy_process_group()


def run(scene, world, debug, steps, config):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = T._free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, scene, q, debug, steps, config)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        d = q.get(timeout=300)
        res[d["rank"]] = d
    for p in procs:
        p.join(timeout=60)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--config", default="lego_L16F2.json")
    a = ap.parse_args()
    root = tempfile.mkdtemp(prefix="dp_probe_")
    S.write_nerf_synthetic_scene(root, 10, 48, 48, seed=5, split="train")
    base = run(root, a.world, 0, a.steps, a.config)
    for debug in (8,):
        v = run(root, a.world, debug, a.steps, a.config)
        n_mlp = base[0]["n_mlp"]
        for step in (2, 3, 4):
            pa, pb = base[0]["full"][step], v[0]["full"][step]
            d = pa != pb
            idx = np.nonzero(d)[0]
            print(f"step {step}: {d[:n_mlp].sum()} of {n_mlp} MLP params differ, {d[n_mlp:].sum()} of {d.size - n_mlp} grid params;"
                  f" first differing indices {idx[:8].tolist()} max |diff| {np.abs(pa - pb).max() if d.any() else 0}")
            if d[n_mlp:].any():
                gi = idx[idx >= n_mlp] - n_mlp
                print("   grid diff index histogram (by 2^17 bins):", np.bincount(gi >> 17).tolist()[:100])
        first = None
        for i, (x, y) in enumerate(zip(base[0]["rec"], v[0]["rec"])):
            if x[1:7] != y[1:7]:
                first = i
                break
        print(f"debug {debug}: first step differing from the retry-free run: {None if first is None else base[0]['rec'][first][0]}")
        lo = max(0, (first or 0) - 2)
        for x, y in list(zip(base[0]["rec"], v[0]["rec"]))[lo:lo + 5]:
            print("   plain", x)
            print("   probe", y)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
