"""Per-phase s_memtime stamps of wave 0 of the first 512 k_o2w workgroups (c2, j1 = 0), with the
timer calibrated against the launch's wall time (dev tool).  usage: WST_LIB=var_st.so python tools/stamps2.py"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, wst_amd  # noqa: F401
from wst_amd import _lib
B, J = 3072, 4
x = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (B, 64, 64), dtype=np.uint8).astype(np.float32) / 255).cuda()
plan = _lib.Plan(64, 64, J, 8)
out = torch.empty((B, plan.K, 4, 4), device="cuda")
st = torch.cuda.current_stream().cuda_stream
wsb = plan.workspace_bytes(2048); ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
lib = ctypes.CDLL(os.path.join(os.path.dirname(_lib.__file__), os.environ.get("WST_LIB", "libwst_hip.so")))
for _ in range(3): plan.forward(x.data_ptr(), 2048, out.data_ptr(), False, ws.data_ptr(), wsb, st)
torch.cuda.synchronize()
lib.wst_dbg_clear_3_3()
ms = plan.forward_profiled(x.data_ptr(), 2048, out.data_ptr(), False, ws.data_ptr(), wsb, st, 1 + 2 * J)
torch.cuda.synchronize()
n = 512 * 64
buf = (ctypes.c_ulonglong * n)()
assert lib.wst_dbg_stamps_3_3(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(512, 64).astype(np.int64)
nslot = int((a[0] > 0).sum())
print("kernel ms", [round(v, 3) for v in ms])
print(f"slots {nslot}; span of first-512 blocks {a[:, nslot-1].max() - a[:, 0].min()} ticks; "
      f"per-block life median {np.median(a[:, nslot-1]-a[:, 0]):.0f}; start spread {a[:, 0].max()-a[:, 0].min()}")
d = np.diff(a[:, :nslot], axis=1)
for i in range(nslot - 1):
    print(f"  {i:2d}->{i+1:2d}: median {np.median(d[:, i]):8.0f}  mean {d[:, i].mean():8.0f}")
