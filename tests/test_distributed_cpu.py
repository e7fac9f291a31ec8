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
