"""Probe kernels at several launch shapes (dev tool): copy GB/s, FMA TFLOP/s."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, wst_amd  # noqa: F401
from wst_amd import _lib
lib = _lib.load()
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream().cuda_stream
for nbytes in (1 << 28, 1 << 30, 1 << 31):
    src = torch.ones(nbytes // 4, device=dev); dst = torch.empty_like(src)
    for _ in range(3): _lib.check_aux(lib.wst_probe_copy(src.data_ptr(), dst.data_ptr(), nbytes, st))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): _lib.check_aux(lib.wst_probe_copy(src.data_ptr(), dst.data_ptr(), nbytes, st))
    e1.record(); e1.synchronize()
    print(f"copy {nbytes>>20} MiB: {2 * nbytes * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9:.0f} GB/s", flush=True)
    del src, dst
    src = torch.ones(nbytes // 4, device=dev); dst = torch.empty_like(src)
    e0.record()
    for _ in range(10): dst.copy_(src)
    e1.record(); e1.synchronize()
    print(f"  torch copy_ {nbytes>>20} MiB: {2 * nbytes * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9:.0f} GB/s", flush=True)
    del src, dst
for nthreads, iters in ((256 * 2048, 8192), (256 * 4096, 8192), (256 * 4096, 16384), (256 * 8192, 8192)):
    scratch = torch.empty(nthreads, device=dev)
    _lib.check_aux(lib.wst_probe_fma(scratch.data_ptr(), nthreads, iters, st))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5): _lib.check_aux(lib.wst_probe_fma(scratch.data_ptr(), nthreads, iters, st))
    e1.record(); e1.synchronize()
    tf = 2.0 * 32 * iters * nthreads * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e12
    print(f"fma {nthreads} threads x {iters}: {tf:.1f} TF", flush=True)
