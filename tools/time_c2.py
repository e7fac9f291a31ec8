"""Quick timing of the WST forward at a config (dev tool)."""
import argparse, sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import wst_amd
from wst_amd import _lib
if os.environ.get("AB_LIB"):          # A/B variant build in the package dir (tools/variant.sh)
    _lib.use_library(os.environ["AB_LIB"])
from wst_amd.frontend import scatter_device
ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1024); ap.add_argument("--C", type=int, default=3)
ap.add_argument("--M", type=int, default=64); ap.add_argument("--J", type=int, default=4)
ap.add_argument("--L", type=int, default=8); ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--pooled", type=int, default=0)
a = ap.parse_args()
x = torch.from_numpy(np.random.default_rng(1).integers(0,256,(a.B*a.C,a.M,a.M),dtype=np.uint8).astype(np.float32)/255).cuda()
for _ in range(2): scatter_device(x, a.M, a.M, a.J, a.L, 2, False, pooled=bool(a.pooled))
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters): scatter_device(x, a.M, a.M, a.J, a.L, 2, False, pooled=bool(a.pooled))
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1)/a.iters
print(f"B={a.B} C={a.C} M={a.M} J={a.J} L={a.L}: {ms:.3f} ms/step  {a.B/ms*1e3:.0f} patches/s")
