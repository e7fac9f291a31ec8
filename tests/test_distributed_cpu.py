"""N>1 path on CPU: world-size-2 gloo ranks shard patches with ``shard_range`` and reassemble
them with ``gather_shards``; the per-shard compute is the float64 oracle (test-only) so the result
must equal the single-process transform exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from wst_amd import distributed as wd


def test_shard_range_partitions():
    for n in (0, 1, 5, 8, 1000003):
        for world in (1, 2, 3, 8):
            spans = [wd.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
                assert b0 == a1
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
            assert sizes == sorted(sizes, reverse=True)
    with pytest.raises(ValueError):
        wd.shard_range(4, 2, 2)


def _oracle_compute(xs):
    from oracle import kymatio_ref as kr
    feats = [kr.extract_wst_features(np.asarray(x, dtype=np.float32), J=1, L=4) for x in xs]
    return torch.from_numpy(np.stack(feats) if feats else np.zeros((0, 3 * 2 * 5)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        imgs = np.random.default_rng(3).integers(0, 256, (n, 3, 16, 16)).astype(np.float32) / 255
        full = wd.extract_sharded(imgs, J=1, L=4, compute=_oracle_compute)
        q.put((rank, full.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [5, 4, 1])
def test_gloo_world2_shard_and_gather_equals_single_process(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    imgs = np.random.default_rng(3).integers(0, 256, (n, 3, 16, 16)).astype(np.float32) / 255
    ref = _oracle_compute(imgs).numpy()
    for r in (0, 1):
        assert res[r].shape == ref.shape
        np.testing.assert_array_equal(res[r], ref)


# ---- BASELINE c3's step logic end to end on gloo ranks (bench.py --config c3 runs the same
# ShardGather / run_sharded_job / c3_check; here the per-patch compute is the float64 oracle) ----
C3_CFG = dict(C=3, M=16, N=16, J=2, L=4)
C3_SEED = 5


def _c3_functions(full):
    from oracle import kymatio_ref as kr
    from oracle import patchgen
    c = C3_CFG
    sc = kr.Scattering2D(J=c["J"], shape=(c["M"], c["N"]), L=c["L"])

    def gen(first, nb):
        # patches first .. first + nb - 1 keyed by global index (the device generator's restatement)
        return patchgen.generate_patches_u8(C3_SEED, first, nb, c["C"], c["M"], c["N"]).astype(np.float32) / 255

    def comp(x, nb, rows):
        for p in range(nb):
            if full:
                rows[p] = torch.from_numpy(sc(x[p]).reshape(-1))
            else:
                rows[p] = torch.from_numpy(kr.extract_wst_features(x[p], J=c["J"], L=c["L"], scattering=sc))
    K = 1 + c["J"] * c["L"] + c["L"] ** 2 * c["J"] * (c["J"] - 1) // 2
    row = c["C"] * K * (c["M"] >> c["J"]) * (c["N"] >> c["J"]) if full else c["C"] * 2 * K
    return gen, comp, row


def _c3_job(total, full, root_only):
    import bench
    gen, comp, row = _c3_functions(full)
    sg = wd.ShardGather(total, (row,), torch.float64, "cpu", root_only=root_only)
    res = wd.run_sharded_job(sg, 2, gen, comp)
    check = None
    if res is not None:
        cfg = dict(C3_CFG, total=total)
        check = bench.c3_check(cfg, res, 0, total, full, nsample=4, seed=C3_SEED)
    return sg, res, check


def _c3_worker(rank, world, port, total, full, root_only, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sg, res, check = _c3_job(total, full, root_only)
        # the bench's rank reduction of the check (max error, summed count) over the ranks
        t = torch.tensor([check[0] if check else 0.0, float(check[1]) if check else 0.0], dtype=torch.float64)
        e = t.clone()
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(e[1:], op=dist.ReduceOp.SUM)
        q.put((rank, None if res is None else res.numpy(), (sg.lo, sg.hi), sg.bytes_moved(),
               t[0].item(), int(e[1].item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,full,root_only", [(7, False, False), (6, True, False), (5, False, True)])
def test_c3_step_gloo_world2_equals_world1(total, full, root_only):
    """global-index patch generation -> shard -> compute into the gather's send buffer -> all-gather
    (or gather to rank 0) -> sampled oracle check: the assembled job equals the world-1 job."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c3_worker, args=(r, 2, port, total, full, root_only, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, ref, check1 = _c3_job(total, full, False)          # world 1: no process group
    ref = ref.numpy()
    assert check1[0] <= 1e-12 and check1[1] >= 1
    spans = [res[r][1] for r in (0, 1)]
    assert spans[0][0] == 0 and spans[0][1] == spans[1][0] and spans[1][1] == total
    for r in (0, 1):
        got, _, moved, err, n = res[r]
        if root_only and r == 1:
            assert got is None
        else:
            assert got.shape == ref.shape
            np.testing.assert_array_equal(got, ref)
        assert moved == 2 * ((total + 1) // 2) * ref.shape[1] * 8   # padded shards
        assert err <= 1e-12 and n >= 1
