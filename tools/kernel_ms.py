"""Per-kernel HIP-event milliseconds of one c2 forward (dev tool)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, wst_amd
from wst_amd import _lib
B = 3072
x = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (B, 64, 64), dtype=np.uint8).astype(np.float32) / 255).cuda()
plan = _lib.Plan(64, 64, 4, 8)
out = torch.empty((B, plan.K, 4, 4), device="cuda")
wsb = plan.workspace_bytes(2048); ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for _ in range(2): plan.forward(x.data_ptr(), B, out.data_ptr(), False, ws.data_ptr(), wsb, st)
acc = [0.0] * 9
for _ in range(5):
    ms = plan.forward_profiled(x.data_ptr(), B, out.data_ptr(), False, ws.data_ptr(), wsb, st, 9)
    acc = [a + b for a, b in zip(acc, ms)]
acc = [a / 5 for a in acc]
print(os.environ.get("WST_LIB", "default"), "kernel ms prep,o1[0..3],o2[0..3]", [round(a, 3) for a in acc], "total", round(sum(acc), 3))
