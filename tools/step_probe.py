#!/usr/bin/env python3
"""Host-side split of the headline bench step (100M x 100M --intersect, text in HBM): wall
time of each engine call (load, op, format, rows, free) over N steps, with the GPU's own
time (the kernels) in between; bg_load's phase marks with BEDGPU_HOSTPROF=1 (stderr)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

import torch  # noqa: E402
from bedops_amd.engine import Group  # noqa: E402

W = bench.WORKLOADS["intersect"]
L = bench.bedgen_lib()
mask = (1 << 64) - 1
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
grp = Group(device=0, uid=bytes(128), nranks=1, rank=0)
eng = grp.engines[0]
bufs, texts = [], []
for (seed, mode), n in zip(W["gen"], W["rows"]):
    p, nb, r = bench.gen(L, n, seed, mask, mode)
    bufs.append(bench.to_device(torch, p, nb, dev))
    L.bedgen_free(p)
    texts.append(nb)
torch.cuda.synchronize(dev)
inputs = [((t.data_ptr(), nb), k) for t, nb, k in zip(bufs, texts, W["kinds"])]
acc = {}


def tick(name, t0):
    t = time.perf_counter()
    acc[name] = acc.get(name, 0.0) + (t - t0)
    return t


N = int(os.environ.get("STEPS", "20"))
for i in range(N + 2):
    if i == 2:
        acc.clear()
        eng.sync()
        T0 = time.perf_counter()
    t = time.perf_counter()
    s = eng.load(inputs)
    t = tick("load", t)
    r = bench.run_op(eng, "intersect", s)
    t = tick("op", t)
    nbytes = r.format()
    t = tick("format", t)
    r.rows()
    t = tick("rows", t)
    r.free()
    s.free()
    t = tick("free", t)
eng.sync()
T = time.perf_counter() - T0
print(f"steps {N}: {1e3 * T / N:.3f} ms/step; per call (ms): " +
      ", ".join(f"{k} {1e3 * v / N:.3f}" for k, v in acc.items()))
grp.close()
