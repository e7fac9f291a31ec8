"""Per-kernel HIP-event milliseconds of one c2 forward at several chunk sizes (dev tool).
usage: python tools/kernel_ms.py [chunk_planes ...]   (default 2048)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, wst_amd  # noqa: F401
from wst_amd import _lib
if os.environ.get("AB_LIB"):          # A/B variant build in the package dir (tools/variant.sh)
    _lib.use_library(os.environ["AB_LIB"])
# geometry: env WST_KM_GEOM="planes,M,J[,L]" (default the c2 step: 3072 planes of 64^2, J=4, L=8)
_g = [int(v) for v in os.environ.get("WST_KM_GEOM", "3072,64,4").split(",")]
B, M, J = _g[:3]
LL = _g[3] if len(_g) > 3 else 8
x = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (B, M, M), dtype=np.uint8).astype(np.float32) / 255).cuda()
plan = _lib.Plan(M, M, J, LL)
POOLED = os.environ.get("KM_POOLED") == "1"   # pooled mean / std output (the reference's features)
out = torch.empty((B, 2 * plan.K) if POOLED else (B, plan.K, plan.Mo, plan.No), device="cuda")
st = torch.cuda.current_stream().cuda_stream
nslot = 1 + 2 * J
for chunk in [int(a) for a in sys.argv[1:]] or [2048]:
    wsb = plan.workspace_bytes(chunk); ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    for _ in range(2): plan.forward(x.data_ptr(), B, out.data_ptr(), POOLED, ws.data_ptr(), wsb, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): plan.forward(x.data_ptr(), B, out.data_ptr(), POOLED, ws.data_ptr(), wsb, st)
    e1.record(); torch.cuda.synchronize()
    wall = e0.elapsed_time(e1) / 10
    acc = [0.0] * nslot
    for _ in range(5):
        ms = plan.forward_profiled(x.data_ptr(), B, out.data_ptr(), POOLED, ws.data_ptr(), wsb, st, nslot)
        acc = [a + b for a, b in zip(acc, ms)]
    acc = [round(a / 5, 3) for a in acc]
    print(os.environ.get("AB_LIB", "default"), f"chunk={chunk} wall={wall:.3f} ms",
          "prep", acc[0], "o1", acc[1:1 + J], "o2", acc[1 + J:], "sum", round(sum(acc), 3), flush=True)
    if os.environ.get("KM_DUMP"):   # the outputs of the first 64 planes, for a cross-library check
        np.save(os.environ["KM_DUMP"], out[:64].cpu().numpy())
    del ws
