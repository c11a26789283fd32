"""Expected fired-row count of a bench workload: distinct (window, key) pairs of the
accepted records (tumbling windows, no late records when the watermark delay covers the
jitter). Used to cross-check bench.py's rows_fired at full size."""
import sys

import torch

sys.path.insert(0, ".")
import bench as B  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "zipf"
wl = B.WORKLOADS[w]
assert wl["window"][0] == "tumbling"
size = wl["window"][1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
dev = torch.device("cuda", 0)
key, ts, val = B.gen_columns(n, wl["keys"], wl["rate"], 0, dev, jitter=wl["jitter"], zipf=wl["zipf"])
del val
comp = torch.div(ts - B.T0, size, rounding_mode="floor") * (1 << 26) + key
del key, ts
u = torch.unique(comp)
print(w, n, "distinct (window, key):", u.numel(), flush=True)
