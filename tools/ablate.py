"""Timing ablation of k_o1 / k_o2 phases (dev tool): per WST_DEBUG_SKIP mask, per-kernel ms.

Needs the diagnostic build (the production library ignores WST_DEBUG_SKIP):
    make -C <pkg>/csrc OUT=../libwst_hip_diag.so OBJ=../build_diag EXTRA=-DWST_DIAG -j16
and loads it through _lib.use_library (ABL_LIB names the file)."""
import os, subprocess, sys, json
masks = {"full": 0, "no_o1_fold": 128, "no_o1_ifft": 1, "no_S1": 2, "no_U1_fft": 4, "no_o2_fold": 8,
         "no_o2_ifft": 16, "no_o2_lowpass": 64, "no_order2_paths": 8 | 16 | 64,
         "o2_only_load": 4 | 8 | 16 | 64, "no_o2_fold_s2": 256, "no_o2_fold_box": 512,
         "no_o2_spectrum_load": 1024, "no_o2_emit": 2048}
LIB = os.environ.get("ABL_LIB", "libwst_hip_diag.so")
if len(sys.argv) > 1:
    masks = {k: v for k, v in masks.items() if k in sys.argv[1:]}
child = r'''
import os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np, torch, wst_amd
from wst_amd import _lib
_lib.use_library(os.environ["ABL_LIB"])
geo = [int(v) for v in os.environ.get("WST_KM_GEOM", "3072,64,4").split(",")]
B, M, J = geo[:3]
L = geo[3] if len(geo) > 3 else 8
x = torch.from_numpy(np.random.default_rng(1).integers(0,256,(B,M,M),dtype=np.uint8).astype(np.float32)/255).cuda()
plan = _lib.Plan(M,M,J,L)
out = torch.empty((B, plan.K, plan.Mo, plan.No), device="cuda")
wsb = plan.workspace_bytes(min(B, plan.preferred_batch())); ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for _ in range(2): plan.forward(x.data_ptr(), B, out.data_ptr(), False, ws.data_ptr(), wsb, st)
acc = [0.0]*(1+2*J)
for _ in range(3):
    ms = plan.forward_profiled(x.data_ptr(), B, out.data_ptr(), False, ws.data_ptr(), wsb, st, 1+2*J)
    acc = [a+b for a,b in zip(acc, ms)]
print(json.dumps([a/3 for a in acc]))
'''
res = {}
for name, m in masks.items():
    env = dict(os.environ, WST_DEBUG_SKIP=str(m), ABL_LIB=LIB)
    r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("[")]
    res[name] = json.loads(line[-1]) if line else r.stderr[-300:]
    print(name, res[name], flush=True)
