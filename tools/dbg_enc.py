import json, os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "instant-ngp-rendering_amd")
import numpy as np
import test_gpu_golden as T
f = T.fixture("encode_L16F2T19.npz")
g = T.gpu_model(json.loads(str(f["cfg"])), int(f["params_seed"]))
e = g.encode(f["pos"]).astype(np.float32)
d = np.argwhere(e != f["feat"])
print("env", os.environ.get("NGP_ENC_LPT"), os.environ.get("NGP_ENC_GATHER"), "shape", e.shape, "mismatch", d.tolist())
for ix in d.tolist():
    print(ix, e[tuple(ix)], f["feat"][tuple(ix)], "pos", f["pos"][ix[1]] if e.shape[1] == f["pos"].shape[0] else None)
g.close()
