#!/usr/bin/env python3
"""Headline benchmark: BASELINE.json metric "patches/sec (whole node) + HBM-roofline %,
64x64 RGB WST J=4 L=8 order-2" on BASELINE config 2 (batch of 1024 64x64 RGB patches per GPU).

A "step" = one Scattering2D(J=4, L=8, order 2) pass over one resident batch of 1024 RGB patches
(3072 planes) -> full coefficient tensor (1024, 3, 417, 4, 4) fp32, via the C ABI (libwst_hip.so).
Inputs are synthetic uint8/255 patches (mimicking load_rgb_image, train_and_save_model.py:51-56)
generated once and resident in HBM before timing.

Multi-GPU (one process per GPU): `bench.py --gpus N` started without WORLD_SIZE launches
itself as N ranks through torch.distributed.run (the parent never touches the GPU); under an
external torchrun the world size must equal --gpus.  The patches shard across ranks with no
data-path collective (weak scaling: every rank processes its own 1024-patch batch); value = all
patches of all ranks / max-over-ranks wall time.  `--gather` additionally times an RCCL
all-gather of the pooled features (reported separately, never in `value`).  c3 is the one
strong-scaling job: 1M patches generated on the devices by global patch index, sharded, pooled,
and all-gathered inside the timed step.

Extra JSON fields:
  roofline     : dominant kernel (largest HIP-event time of the step; k_o2 at j1=0 on c2)
                 algorithmic FLOP per launch / HIP-event launch time
                 vs the fp32 VALU peak (SURVEY §8(d) flop convention 5 n^2 log2 n^2 per n x n FFT);
                 traffic from committed rocprofv3 PMC passes when they match this library build.
  measured     : BW_meas (streaming-copy probe) and FP32_meas (FMA probe), this run, this GPU
                 (informational: the roofline is priced against the spec peaks only).
  lib_built_from_src : the loaded libwst_hip.so is the one __graft_entry__.build() produced from
                 these sources (libwst_hip.build.json; build_record says whether make recompiled).
  cpu_baseline : the float64 oracle (oracle/kymatio_ref.py, a port of kymatio 0.3.0) on the
                 host cores, rank 0 at every N, before the GPU is touched, bounded sample:
                 (i) run the way the reference runs it (plan rebuilt per patch, 3 serial channel
                 calls + mean/std, train_and_save_model.py:346-378), one core = `value`;
                 (ii) `multi_core`: the same float64 code in a fork pool of `workers` processes
                 (cached plan, batched calls).  `workers` = the host CPUs this process may use:
                 its affinity set capped by OMP_NUM_THREADS -- on the GPU box that is one GPU's
                 share of the host (16 of 256 CPUs), the pool size the box allows.
"""
import argparse
import hashlib
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "patches/sec (whole node) + HBM-roofline %, 64x64 RGB WST J=4 L=8 order-2"
FP32_PEAK_TFLOPS = 157.3      # MI355X FP32 vector == f32 MFMA dense peak (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
LDS_RESIDENT_MAX = 136        # levels larger than this run HBM-staged (csrc/wst_staged.h)

CONFIGS = {
    "c2": dict(workload="c2: 1024 x 64x64 RGB patches, Scattering2D J=4 L=8 order-2 (per GPU)",
               C=3, M=64, N=64, J=4, L=8, batch=1024),
    "c1": dict(workload="c1: 64x64 RGB patch, J=2 L=8 order-2 (batch as given)",
               C=3, M=64, N=64, J=2, L=8, batch=1024),
    "c3": dict(workload="c3: 1M synthetic 64x64 RGB patches (generated on device by global patch "
                        "index) sharded over the ranks, J=4 L=8 order-2 pooled features + RCCL "
                        "all-gather (one job per step)",
               C=3, M=64, N=64, J=4, L=8, batch=1024, total=1_000_000),
    "c4": dict(workload="c4: noise-robustness sweep -- 13 (type, intensity) cases of the reference's "
                        "experiments/ (add_noise.py formulas, device draws) on 1024 64x64 RGB patches, "
                        "each -> J=4 L=8 order-2 pooled features (per GPU)",
               C=3, M=64, N=64, J=4, L=8, batch=1024),
    "c5": dict(workload="c5: 64 x 256x256 4-band patches, Scattering2D J=6 L=12 order-2 (per GPU; "
                        "384^2 and 192^2 levels HBM-staged)",
               C=4, M=256, N=256, J=6, L=12, batch=64),
    # the geometry the reference's experiments were run at (128x128 RGB
    # images, J=2, L=8: train_and_save_model.py:352-359 on experiment_report image_shape)
    "f3": dict(workload="f3: 256 x 128x128 RGB patches, Scattering2D J=2 L=8 order-2 (the reference's "
                        "experiment geometry; P = 136)",
               C=3, M=128, N=128, J=2, L=8, batch=256),
}


# the reference's noise sweep: experiments/<type>/*/datasets_<type>_<I>
NOISE_SWEEP = [("gaussian", 30), ("gaussian", 50), ("poisson", 40), ("poisson", 60),
               ("salt_and_pepper", 5), ("salt_and_pepper", 15), ("salt_and_pepper", 25),
               ("speckle", 15), ("speckle", 35), ("speckle", 55),
               ("uniform", 10), ("uniform", 25), ("uniform", 40)]

C3_SEED = 1            # c3 patches: wst_patch_generate(seed=1, global index)


def fft_flops(n1, n2):
    n = n1 * n2
    return 5.0 * n * math.log2(n) if n > 1 else 0.0


def alg_flops_per_plane(PM, PN, J, L, max_order=2):
    """kymatio cascade FFT FLOPs per plane (SURVEY §8(d) convention), split by the kernel that
    performs each part: {"k_prep": X^ + S0, "k_o1_j1=j": U1 ifft + S1 (+ the row half of the U1
    fft when order 2 follows), "k_o2_j1=j": column half of the U1 fft + every U2 ifft/fft + S2}."""
    mM, mN = PM >> J, PN >> J
    out = {"k_prep": fft_flops(PM, PN) + fft_flops(mM, mN)}
    for j1 in range(J):
        n1 = (PM >> j1, PN >> j1)
        do2 = max_order >= 2 and j1 < J - 1
        u1 = L * fft_flops(*n1)
        out[f"k_o1_j1={j1}"] = u1 + L * fft_flops(mM, mN) + (u1 / 2 if do2 else u1)
        if do2:
            f = u1 / 2
            for j2 in range(j1 + 1, J):
                n2 = (PM >> j2, PN >> j2)
                f += L * L * (2 * fft_flops(*n2) + fft_flops(mM, mN))
            out[f"k_o2_j1={j1}"] = f
    return out


def kernel_slots(J, max_order=2):
    """Slot order of wst_forward_profiled: [k_prep, k_o1 j1=0..J-1, k_o2 j1=0..J-1]."""
    return ["k_prep"] + [f"k_o1_j1={j}" for j in range(J)] + [f"k_o2_j1={j}" for j in range(J)]


def staged_levels(PM, PN, J):
    """Leading levels r with max(PM, PN) >> r > 136 run HBM-staged (wst_plan_create's rb)."""
    rb = 0
    while rb < J and max(PM, PN) >> rb > LDS_RESIDENT_MAX:
        rb += 1
    return rb


def family(P):
    """FFT size family of a padded size: its odd part when compiled, else 0 (generic DFT)."""
    o = P
    while o % 2 == 0:
        o //= 2
    return o if o in (1, 3, 5, 7, 9, 11, 13, 15, 17, 27) else 0


def rocprof_name(slot, PM, PN, J):
    """Kernel name (template prefix) rocprofv3 reports for a timing slot.  Slots of HBM-staged
    levels (j1 < rb, c5's 384^2 / 192^2) run several kernels; they are named by the composite."""
    fm, fn = family(PM), family(PN)
    rb = staged_levels(PM, PN, J)
    if slot == "k_prep":
        if rb:
            return f"k_big_mean + k_big_rows<{PM}, 0> + k_big_cols<{PM}, 0> + k_big_final"
        return f"k_prep<{fm}, {fn}"
    kind, j1 = slot.split("_j1=")
    j1 = int(j1)
    if j1 < rb:
        n = PM >> j1
        if kind == "k_o1":
            return f"k_big_rows<{n}, 1> + k_big_cols<{n}, 1> + k_big_final + U1hat k_big_rows<{n}, 0>"
        return f"staged order-2 k_big_rows/cols + k_big_final + k_o2<{fm}, {fn}, 136, 1, 1"
    n = max(PM, PN) >> j1
    cap = 12 if n <= 12 else 24 if n <= 24 else 48 if n <= 48 else 136
    return f"{kind}<{fm}, {fn}, {cap}"


def lib_sha():
    from wst_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def src_sha():
    """Hash of the kernel sources + build recipe (stable across rebuilds of the same code, unlike
    the .so bytes): ties committed PMC profiles to the code they measured."""
    from wst_amd import _lib
    csrc = os.path.join(os.path.dirname(_lib.LIB_PATH), "csrc")
    h = hashlib.sha256()
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                   if f.endswith((".hip", ".h", ".cpp")) or f == "Makefile")
    files.append(os.path.join(ROOT, "include", "wst_hip.h"))
    for p in files:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_provenance():
    """The record __graft_entry__.build() left beside the library: was the loaded .so built from
    these sources (same src_sha) and is it the file that build produced (same lib_sha)?"""
    from wst_amd import _lib
    path = os.path.join(os.path.dirname(_lib.LIB_PATH), "libwst_hip.build.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return {"lib_built_from_src": None, "build_record": None}
    return {"lib_built_from_src": rec.get("src_sha") == src_sha() and rec.get("lib_sha") == lib_sha(),
            "build_record": {k: rec.get(k) for k in ("src_sha", "lib_sha", "rebuilt", "make_q_before")}}


def pmc_file_config(name):
    """Config a PMC summary file belongs to: profiles/pmc_<tag>_<config>.json (tools/profile_cfg.sh);
    the suffix-less pmc_<tag>.json of tools/profile_round.sh is the default config c2."""
    stem = name[len("pmc_"):-len(".json")]
    last = stem.rsplit("_", 1)[-1]
    return last if last in CONFIGS else "c2"


def pmc_summary(sha, config="c2"):
    """The newest committed rocprofv3 PMC summary (tools/pmc_hbm.py) of this exact build and
    geometry.  Kernel names repeat across geometries (c5's LDS-resident levels instantiate the same
    k_o2<3, 3, 136, ...> as c2), so only files of this config count; c3 / c4 run c2's kernels."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    want = "c2" if config in ("c3", "c4") else config
    for name in sorted(os.listdir(pdir), reverse=True):
        if name.startswith("pmc_") and name.endswith(".json") and pmc_file_config(name) == want:
            try:
                d = json.load(open(os.path.join(pdir, name)))
            except Exception:
                continue
            if sha in (d.get("lib_sha"), d.get("src_sha")):
                return d
    return None


def pmc_traffic(sha, kernel, config="c2"):
    """HBM bytes per launch of `kernel` (template prefix "k_o2<3, 3, 136"; variants append
    ", SQ, HG>") from the matching PMC summary."""
    d = pmc_summary(sha, config)
    if d is None:
        return None
    for kname, v in d.get("hbm_bytes_per_launch", {}).items():
        if kname == kernel + ">" or kname.startswith(kernel + ","):
            return v
    return None


BIG_SIZES = (96, 144, 160, 192, 256, 272, 288, 320, 384, 512)   # csrc/wst_launch.h WST_BIG_SIZES


def staged_sequence(PM, PN, J, L, nst, max_order=2):
    """[(timing slot, kernel)] of one chunk's HBM-staged levels, in launch order (a mirror of
    staged_levels in csrc/wst_hip.hip; nst = rb for square compiled-family planes)."""
    def big(kind, n, inv):
        return f"k_big_{kind}<{n if n in BIG_SIZES else 0}, {'true' if inv else 'false'}>"
    fm, fn = family(PM), family(PN)
    rb = staged_levels(PM, PN, J)
    seq = [("k_prep", "k_big_mean"), ("k_prep", big("rows", PN, False)),
           ("k_prep", big("cols", PM, False)), ("k_prep", "k_big_final")]
    for j1 in range(rb):
        m1, n1 = PM >> j1, PN >> j1
        do2 = max_order >= 2 and j1 < J - 1
        o1, o2 = f"k_o1_j1={j1}", f"k_o2_j1={j1}"
        seq += [(o1, big("rows", n1, True)), (o1, big("cols", m1, True)), (o1, "k_big_final")]
        if not do2:
            continue
        seq += [(o1, big("rows", n1, False))]      # kRowHalf: U1hat from the column spectra
        for j2 in range(j1 + 1, nst):
            seq += [(o2, big("rows", PN >> j2, True)), (o2, big("cols", PM >> j2, True))] * L
            seq.append((o2, "k_big_final"))
        if max(j1 + 1, nst) < J:
            seq.append((o2, f"k_o2<{fm}, {fn}, 136, 1, 1>"))
    return seq


def slot_traffic(summary, seq, slot):
    """HBM bytes per chunk of a composite timing slot: the PMC dispatch sequence is matched
    against the staged launch order `seq` chunk by chunk and the slot's kernels summed (mean over
    the matched chunks); None when the recorded sequence does not follow `seq`."""
    disp = (summary or {}).get("dispatch_seq")
    if not disp:
        return None
    names = [n for n, _ in disp]
    exp = [k for _, k in seq]
    tot, nmatch, i = 0, 0, 0
    while i + len(exp) <= len(names):
        if names[i:i + len(exp)] == exp:
            tot += sum(disp[i + k][1] for k, (sl, _) in enumerate(seq) if sl == slot)
            nmatch += 1
            i += len(exp)
        else:
            i += 1
    return round(tot / nmatch) if nmatch else None


# ------------------------------------------------------------------------------------------
# CPU baseline (runs on rank 0 before the GPU is touched: the all-cores leg forks)
# ------------------------------------------------------------------------------------------
def cpu_workers():
    """Host cores this process may use: the affinity set, capped by OMP_NUM_THREADS when the
    environment sets one (the GPU box sets 16 = one GPU's share of the host).  Ranks started by
    launch_ranks inherit the parent's count in WST_CPU_WORKERS: torch.distributed.run sets
    OMP_NUM_THREADS=1 in every rank when nproc > 1, which is not the host's core budget."""
    inherited = os.environ.get("WST_CPU_WORKERS")
    if inherited and inherited.isdigit() and int(inherited) > 0:
        return int(inherited)
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_workers_basis():
    """How cpu_workers() chose its count (stated in the bench line)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"affinity": aff, "os_cpu_count": os.cpu_count(),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
            "WST_CPU_WORKERS": os.environ.get("WST_CPU_WORKERS"),
            "rule": "affinity set capped by OMP_NUM_THREADS (the GPU box sets 16: one GPU's share "
                    "of the host, the worker-pool size the box allows)"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _single_thread():
    try:
        from threadpoolctl import threadpool_limits
        return threadpool_limits(1)
    except Exception:
        return None


def _all_cores_worker(cfg, budget_s, seed, conn):
    """Forked child: cached-plan oracle, batches of 4 patches, until the budget runs out."""
    import numpy as np
    _single_thread()
    from oracle import kymatio_ref as kr
    sc = kr.Scattering2D(J=cfg["J"], shape=(cfg["M"], cfg["N"]), L=cfg["L"])
    rng = np.random.default_rng(seed)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        xb = rng.integers(0, 256, (4, cfg["C"], cfg["M"], cfg["N"]), dtype=np.uint8).astype(np.float32) / 255
        S = sc(xb)
        np.mean(S, axis=(-2, -1)), np.std(S, axis=(-2, -1))
        n += 4
    conn.send((n, time.perf_counter() - t0))
    conn.close()


def cpu_baseline(cfg, budget_s):
    """(i) Reference-faithful CPU path on the float64 oracle: per patch, Scattering2D rebuilt
    (train_and_save_model.py:359) and 3 serial channel calls + mean/std (:364-376), one thread.
    (ii) The same float64 code on every host core this process may use: a fork pool, each worker
    with a cached plan and batched calls."""
    import multiprocessing as mp

    import numpy as np
    lim = _single_thread()
    from oracle import kymatio_ref as kr
    rng = np.random.default_rng(1)
    n, t0 = 0, time.perf_counter()
    while True:
        img = rng.integers(0, 256, (cfg["C"], cfg["M"], cfg["N"]), dtype=np.uint8).astype(np.float32) / 255
        kr.extract_wst_features(img, J=cfg["J"], L=cfg["L"])      # builds its own Scattering2D
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 256:
            break
    faithful = n / el
    if lim is not None and hasattr(lim, "unregister"):
        lim.unregister()
    workers = cpu_workers()
    allc = None
    if el / n * 4 <= budget_s:         # a worker can finish a few batches inside the budget
        ctx = mp.get_context("fork")
        pipes, procs = [], []
        for w in range(workers):
            a, b = ctx.Pipe(duplex=False)
            p = ctx.Process(target=_all_cores_worker, args=(cfg, budget_s, 100 + w, b))
            p.start()
            pipes.append(a)
            procs.append(p)
        res = [a.recv() for a in pipes]
        for p in procs:
            p.join()
        tot = sum(r[0] for r in res)
        wall = max(r[1] for r in res)
        allc = {"value": round(tot / wall, 3), "unit": "patches/s", "cores": workers,
                "workers": workers, "workers_basis": cpu_workers_basis(),
                "sample": f"{tot} patches over {workers} forked workers in {wall:.1f} s (cached plan, "
                          f"batches of 4, float64 oracle, one thread each)"}
    return {
        "value": round(faithful, 3), "unit": "patches/s", "cores": 1, "kind": "port",
        "sample": (f"{n} patches of ({cfg['C']},{cfg['M']},{cfg['N']}) in {el:.1f} s: oracle/kymatio_ref.py "
                   f"float64 port of kymatio 0.3.0, plan rebuilt per patch + 3 channel calls + mean/std "
                   f"(train_and_save_model.py:346-378), single thread"),
        "multi_core": allc,
        "host_cpu_count": os.cpu_count(),
        "host_affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
        "cpu_model": _cpu_model(),
    }


# ------------------------------------------------------------------------------------------
# launcher (parent, no GPU) and in-run probes
# ------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """Re-run this script as n ranks under torch.distributed.run, as a child process (the parent
    has not touched the GPU and does not exec); returns the launcher's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("WST_CPU_WORKERS", str(cpu_workers()))   # the parent's budget, not torchrun's 1
    return subprocess.call(cmd, env=env)


def measure_probes(torch, lib, dev, stream):
    """BW_meas (16-B streaming copy, 1 GiB -> 1 GiB, contiguous 8 KiB tiles per workgroup: 6.13 TB/s
    measured, 97 % of the guide's 6.29; 2 GiB 5.93) and
    FP32_meas (32 independent FMA chains per lane, 16 waves per SIMD, long enough that launch and
    clock ramp do not count: 151 TF at 4096 x 256 threads x 16384 steps against 122-145 for shorter
    runs)."""
    from wst_amd import _lib
    nbytes = 1 << 30
    src = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        _lib.check_aux(lib.wst_probe_copy(src.data_ptr(), dst.data_ptr(), nbytes, stream))
    e0.record()
    reps = 10
    for _ in range(reps):
        _lib.check_aux(lib.wst_probe_copy(src.data_ptr(), dst.data_ptr(), nbytes, stream))
    e1.record()
    e1.synchronize()
    bw = 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    nthreads, iters = 256 * 4096, 16384
    scratch = torch.empty(nthreads, dtype=torch.float32, device=dev)
    _lib.check_aux(lib.wst_probe_fma(scratch.data_ptr(), nthreads, iters, stream))
    e0.record()
    reps = 5
    for _ in range(reps):
        _lib.check_aux(lib.wst_probe_fma(scratch.data_ptr(), nthreads, iters, stream))
    e1.record()
    e1.synchronize()
    tf = 2.0 * 32 * iters * nthreads * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12
    return {"bw_gbs": round(bw, 1), "fp32_tflops": round(tf, 2),
            "bw_probe": "16-B/lane non-temporal copy in 8 KiB tiles, 1 GiB -> 1 GiB, bytes read + written",
            "fp32_probe": f"{nthreads} lanes x 32 independent v_fma_f32 chains x {iters} steps"}


def launch_check(args, rank, world):
    """--launch-check: the rank plumbing alone (gloo, no GPU): every rank reports in."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([rank + 1.0])
    dist.all_reduce(t)
    ok = world == dist.get_world_size() and t.item() == world * (world + 1) / 2
    if rank == 0:
        print(json.dumps({"launch_check": {"world": dist.get_world_size(), "gpus": args.gpus,
                                           "rank_sum": t.item(), "ok": ok}}), flush=True)
    dist.destroy_process_group()
    if not ok:
        sys.exit(1)


def c3_check(cfg, rows, lo, hi, full_output=False, nsample=64, seed=C3_SEED):
    """Recreate `nsample` sampled patches of the global range [lo, hi) on the host
    (oracle/patchgen.py) and compare their rows of `rows` (row i - lo = patch i: pooled features, or
    the full (C, K, Mo, No) maps) with the float64 oracle, per feature / coefficient max-normalised.
    After an all-gather [lo, hi) is the whole job, so other ranks' shards are checked too."""
    import numpy as np
    from oracle import kymatio_ref as kr
    from oracle import patchgen
    idx = np.random.default_rng(77).choice(cfg["total"], min(cfg["total"], 64 * 64), replace=False)
    mine = [int(i) for i in idx if lo <= i < hi][:nsample]
    if not mine:
        return 0.0, 0
    sc = kr.Scattering2D(J=cfg["J"], shape=(cfg["M"], cfg["N"]), L=cfg["L"])
    xs = np.stack([patchgen.generate_patches_u8(seed, i, 1, cfg["C"], cfg["M"], cfg["N"])[0]
                   for i in mine]).astype(np.float32) / 255
    ref = []
    for b0 in range(0, len(mine), 8):      # one batched oracle call per 8 patches
        S = sc(xs[b0:b0 + 8])                                       # (b, C, K, Mo, No)
        if full_output:                                             # per (channel, coefficient)
            ref.append(S.reshape(S.shape[0], S.shape[1] * S.shape[2], -1))
        else:   # extract_wst_features layout: per channel [mean(K) | std(K)]
            ref.append(np.concatenate([S.mean(axis=(-2, -1)), S.std(axis=(-2, -1))],
                                      axis=-1).reshape(S.shape[0], -1))
    ref = np.concatenate(ref)
    got = np.stack([rows[i - lo].cpu().numpy().reshape(ref.shape[1:]) for i in mine]).astype(np.float64)
    if full_output:   # per coefficient: max |d| / max |S| over the sampled patches and positions
        scale = np.abs(ref).max(axis=(0, 2))
        err = np.abs(got - ref).max(axis=(0, 2))
    else:
        scale = np.abs(ref).max(axis=0)
        err = np.abs(got - ref).max(axis=0)
    scale = np.where(scale > 0, scale, 1.0)
    return float((err / scale).max()), len(mine)


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (ranks); default 1 or WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="patches per GPU (default: config)")
    ap.add_argument("--pooled", action="store_true", help="fused mean/std epilogue output")
    ap.add_argument("--gather", action="store_true", help="also time an RCCL all-gather of features")
    ap.add_argument("--c3-output", choices=("pooled", "full"), default="pooled",
                    help="c3: gather pooled features (10 GB at 1M) or the full coefficient tensor "
                         "(N, 3, 417, 4, 4) (80 GB at 1M)")
    ap.add_argument("--c3-gather", choices=("all", "root"), default="all",
                    help="c3: all-gather to every rank, or gather to rank 0")
    ap.add_argument("--c3-total", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds per CPU-baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probes", action="store_true", help="skip the BW / FP32 probe kernels")
    ap.add_argument("--profile-iters", type=int, default=5)
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus))          # parent: no GPU call, no exec
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is None:
        args.gpus = world
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} ranks")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.launch_check:
        return launch_check(args, rank, world)

    cfg = dict(CONFIGS[args.config])
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, args.cpu_budget)      # before any GPU call (the pool forks)

    import numpy as np
    import torch
    import torch.distributed as dist

    import wst_amd  # noqa: F401
    from wst_amd import _lib

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == args.gpus

    B = args.batch or cfg["batch"]
    C, M, N, J, L = cfg["C"], cfg["M"], cfg["N"], cfg["J"], cfg["L"]
    planes = B * C
    lib = _lib.load()

    rng = np.random.default_rng(1 + rank)
    x = torch.from_numpy(rng.integers(0, 256, (B, C, M, N), dtype=np.uint8).astype(np.float32) / 255).to(dev)
    plan = _lib.Plan(M, N, J, L, 2, False)
    K, Mo, No = plan.K, plan.Mo, plan.No
    out = torch.empty((planes, 2 * K) if args.pooled else (planes, K, Mo, No), dtype=torch.float32, device=dev)
    ws_bytes = plan.workspace_bytes(min(planes, plan.preferred_batch()))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        plan.forward(x.data_ptr(), planes, out.data_ptr(), args.pooled, ws.data_ptr(), ws_bytes, stream)

    units_per_step = B                    # patches one rank processes per step
    scaling = "weak"
    extra = {}
    c3_state = None
    if args.config == "c4":
        from wst_amd import noise as wnoise
        x_u8 = torch.from_numpy(rng.integers(0, 256, (B, M, N, C), dtype=np.uint8)).to(dev)
        xin = torch.empty((B, C, M, N), dtype=torch.float32, device=dev)
        feats = torch.empty((len(NOISE_SWEEP), planes, 2 * K), dtype=torch.float32, device=dev)
        counter = [0]

        def step():  # noqa: F811
            counter[0] += 1
            for i, (nt, inten) in enumerate(NOISE_SWEEP):
                _lib.check_aux(lib.wst_noise_generate(wnoise.NOISE_TYPES[nt], float(inten), x_u8.data_ptr(),
                                                      B, M, N, C, 1000 * counter[0] + i, 1, xin.data_ptr(),
                                                      stream))
                plan.forward(xin.data_ptr(), planes, feats[i].data_ptr(), True, ws.data_ptr(), ws_bytes,
                             stream)
        units_per_step = B * len(NOISE_SWEEP)
        extra["sweep"] = [f"{t}_{i}" for t, i in NOISE_SWEEP]
    elif args.config == "c3":
        from wst_amd import distributed as wdist
        if args.c3_total:
            cfg["total"] = args.c3_total
        total = cfg["total"]
        full_out = args.c3_output == "full"
        row = C * K * Mo * No if full_out else C * 2 * K
        # receive / shard buffers allocated once, outside the timed step; the plan writes each
        # batch's outputs straight into this rank's rows of the gather's send buffer
        sg = wdist.ShardGather(total, (row,), torch.float32, dev, root_only=args.c3_gather == "root")
        lo, hi, mine = sg.lo, sg.hi, sg.mine
        xb = torch.empty((B, C, M, N), dtype=torch.float32, device=dev)

        def gen(first, nb):
            # patches first .. first + nb - 1 of the job, keyed by global index
            _lib.check_aux(lib.wst_patch_generate(C3_SEED, first, nb, C, M, N, 1, xb.data_ptr(), stream))
            return xb

        def comp(xin, nb, rows):
            plan.forward(xin.data_ptr(), nb * C, rows.data_ptr(), not full_out, ws.data_ptr(), ws_bytes, stream)

        result = [None]

        def step():  # noqa: F811
            result[0] = wdist.run_sharded_job(sg, B, gen, comp)
        units_per_step = mine
        scaling = "strong"
        c3_state = (sg, result, full_out)
        extra["c3"] = {"total_patches": total, "patches_this_rank": mine, "output": args.c3_output,
                       "bytes_per_patch": row * 4,
                       "collective": ("none (one rank)" if world == 1 else
                                      "RCCL all_gather_into_tensor (equal shards: no compaction)"
                                      if args.c3_gather == "all" else "RCCL gather to rank 0"),
                       "gathered_bytes": sg.bytes_moved()}

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    ms_per_step = dt / args.steps * 1e3
    if args.config == "c3":
        value = total * args.steps / dt
    else:
        value = units_per_step * world * args.steps / dt

    if c3_state is not None:        # sampled patches vs the float64 oracle
        sg, result, full_out = c3_state
        gathered = result[0] is not None and (world == 1 or sg.full is not None)
        if gathered:
            err, nchk = c3_check(cfg, result[0], 0, total, full_out)    # the gathered job
        else:
            err, nchk = c3_check(cfg, sg.local, lo, hi, full_out,       # this rank's shard
                                 nsample=max(8, -(-64 // world)))
        if world > 1 and not (gathered and args.c3_gather == "all"):
            t = torch.tensor([err, float(nchk)], dtype=torch.float64, device=dev)
            e2 = t.clone()
            dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(e2[1:], op=dist.ReduceOp.SUM)
            err, nchk = t[0].item(), int(e2[1].item())
        extra["c3"]["oracle_check"] = {"patches": nchk, "max_rel_err": err, "tol": 1e-5,
                                       "ok": err <= 1e-5}

    # per-kernel HIP-event durations on the launch stream (separate, untimed passes; the library
    # records the events while it enqueues and reads them after the pass, so the kernels run back
    # to back as in step(): the same steady state rocprofv3's kernel trace sees)
    slots = kernel_slots(J)
    acc = [0.0] * len(slots)
    plan.forward_profiled(x.data_ptr(), planes, out.data_ptr(), args.pooled, ws.data_ptr(), ws_bytes,
                          stream, len(slots))             # discarded: event pool warm-up
    for _ in range(args.profile_iters):
        ms = plan.forward_profiled(x.data_ptr(), planes, out.data_ptr(), args.pooled, ws.data_ptr(),
                                   ws_bytes, stream, len(slots))
        acc = [a + b for a, b in zip(acc, ms)]
    kms = dict(zip(slots, (a / args.profile_iters for a in acc)))
    nchunks = math.ceil(planes / min(planes, plan.preferred_batch()))
    flops = alg_flops_per_plane(plan.PM, plan.PN, J, L)
    kms = {k: v for k, v in kms.items() if k in flops}
    dom = max(kms, key=kms.get)                     # dominant kernel of the step
    dom_flop = planes * flops[dom]
    achieved = dom_flop / (kms[dom] * 1e-3) / 1e12
    probes = None if args.no_probes else measure_probes(torch, lib, dev, stream)
    sha = src_sha()
    dname = rocprof_name(dom, plan.PM, plan.PN, J)
    summary = pmc_summary(sha, args.config) or pmc_summary(lib_sha(), args.config)
    rb, nst, _ = plan.staging()            # the plan's own level schedule (wst_plan_staging)
    if dom != "k_prep" and int(dom.split("=")[1]) >= rb:
        traffic = pmc_traffic(sha, dname, args.config) or pmc_traffic(lib_sha(), dname, args.config)
    else:   # composite slot of the staged levels: its kernels summed per chunk
        traffic = slot_traffic(summary, staged_sequence(plan.PM, plan.PN, J, L, nst), dom)
        if traffic is None and summary is not None:
            print(f"bench: warning: the PMC dispatch sequence of {summary.get('src_sha')} matches no "
                  f"chunk of the staged launch order (rb={rb}, nst={nst}); roofline.traffic is null",
                  file=sys.stderr, flush=True)
    avg_ms = kms[dom] / nchunks
    roofline = {
        "bound": "valu", "pipe": "fp32 VALU (LDS FFT butterflies; f32 MFMA only in the wide low-pass)",
        "kernel": f"{dom} ({dname}, ...>)", "achieved": round(achieved, 4), "peak": FP32_PEAK_TFLOPS,
        "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 5),
        "traffic": traffic,
        # the same launch against the HBM roof: PMC bytes (FETCH_SIZE counts Infinity-Cache hits
        # too) over the HIP-event duration, / the 8 TB/s spec peak
        "hbm_frac": (round(traffic / (avg_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 5) if traffic else None),
        "timing": (f"HIP events around each launch on its stream, kernels back to back (no host wait "
                   f"between them), mean of {args.profile_iters} untimed forwards after the timed steps"),
        "launches_per_step": nchunks,
        "avg_launch_ms": round(avg_ms, 4),
        "alg_flop_per_launch": round(dom_flop / nchunks),
        "kernel_ms_per_step": {k: round(v, 4) for k, v in kms.items()},
        "all_kernels_tflops": round(planes * sum(flops.values()) / (sum(kms.values()) * 1e-3) / 1e12, 4),
        "src_sha": sha, "lib_sha": lib_sha(),
    }
    patch_flop = C * sum(flops.values())
    patch_bytes = C * M * N * 4 + (C * 2 * K * 4 if args.pooled else C * K * Mo * No * 4)
    rate_per_gpu = value / world
    bw = probes["bw_gbs"] if probes else HBM_PEAK_GBS
    step_roof = {
        "alg_flop_per_patch": round(patch_flop), "alg_bytes_per_patch": patch_bytes,
        "valu_frac": round(patch_flop * rate_per_gpu / (FP32_PEAK_TFLOPS * 1e12), 5),
        "hbm_roofline_pct": round(100 * patch_bytes * rate_per_gpu / (HBM_PEAK_GBS * 1e9), 5),
        "hbm_roofline_pct_of_measured": round(100 * patch_bytes * rate_per_gpu / (bw * 1e9), 5),
    }

    gather = None
    if args.gather and world > 1:
        feats = torch.empty((planes, 2 * K), dtype=torch.float32, device=dev)
        plan.forward(x.data_ptr(), planes, feats.data_ptr(), True, ws.data_ptr(), ws_bytes, stream)
        allf = torch.empty((world * planes, 2 * K), dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(allf, feats)
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(5):
            dist.all_gather_into_tensor(allf, feats)
        torch.cuda.synchronize(dev)
        gather = {"what": "pooled features all_gather", "bytes_per_rank": feats.numel() * 4,
                  "ms": round((time.perf_counter() - g0) / 5 * 1e3, 4)}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "patches/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic uint8/255 RGB patches (load_rgb_image distribution), resident in HBM",
            "config": {"workload": cfg["workload"], "patches_per_gpu": units_per_step, "channels": C,
                       "shape": [M, N], "J": J, "L": L, "max_order": 2, "K": K,
                       "output": ("pooled [mean|std]" if (args.pooled or args.config == "c4" or
                                                       (args.config == "c3" and args.c3_output == "pooled"))
                                  else f"full ({K},{Mo},{No}) fp32"),
                       "parallelism": f"patch-sharded x{world} (no collective in step)"
                                      if args.config != "c3" else
                                      f"patch-sharded x{world} + RCCL {'all-gather' if args.c3_gather == 'all' else 'gather'}"
                                      f" of {'the coefficient tensor' if args.c3_output == 'full' else 'pooled features'}"},
            "roofline": roofline, "step_roofline": step_roof, "measured": probes, "cpu_baseline": cpu,
        }
        line.update(build_provenance())
        if gather:
            line["gather"] = gather
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
