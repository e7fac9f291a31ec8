"""Per-kernel ms of one pooled (mean/std) forward at a geometry (dev tool).
usage: WST_KM_GEOM=planes,M,J python tools/pooled_ms.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, wst_amd  # noqa: F401
from wst_amd import _lib
B, M, J = (int(v) for v in os.environ.get("WST_KM_GEOM", "3072,64,4").split(","))
x = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (B, M, M), dtype=np.uint8).astype(np.float32) / 255).cuda()
plan = _lib.Plan(M, M, J, 8)
out = torch.empty((B, 2 * plan.K), device="cuda")
st = torch.cuda.current_stream().cuda_stream
chunk = min(B, plan.preferred_batch())
wsb = plan.workspace_bytes(chunk); ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
for _ in range(2): plan.forward(x.data_ptr(), B, out.data_ptr(), True, ws.data_ptr(), wsb, st)
torch.cuda.synchronize()
nslot = 1 + 2 * J
acc = [0.0] * nslot
for _ in range(5):
    ms = plan.forward_profiled(x.data_ptr(), B, out.data_ptr(), True, ws.data_ptr(), wsb, st, nslot)
    acc = [a + b for a, b in zip(acc, ms)]
acc = [round(a / 5, 3) for a in acc]
print(os.environ.get("WST_LIB", "default"), f"pooled {B}x{M}^2 J={J}", "prep", acc[0], "o1", acc[1:1 + J],
      "o2", acc[1 + J:], "sum", round(sum(acc), 3), flush=True)
