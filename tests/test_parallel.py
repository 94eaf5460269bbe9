"""CPU tests of the multi-GPU host logic (tcam_wsol_video_amd/parallel.py):

* DistributedSampler frame order (wsol_loader.py:1008-1012) vs torch's own sampler;
* the CAM-TMP neighbour windows vs the oracle's restatement of wsol_loader.py:447-458,
  544-569;
* sync_tensor_across_gpus (dlib/parallel/__init__.py:14-23) over gloo, world 2;
* bench.py refusing a world size that differs from --gpus.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import model_ref as R
from tcam_wsol_video_amd import parallel as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 5, 7, 8, 13, 64])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("shuffle", [False, True])
@pytest.mark.parametrize("drop_last", [False, True])
def test_sampler_indices_match_torch(n, world, shuffle, drop_last):
    from torch.utils.data import DistributedSampler
    if drop_last and n < world:
        pytest.skip("torch yields nothing")
    data = list(range(n))
    for rank in range(world):
        s = DistributedSampler(data, num_replicas=world, rank=rank, shuffle=shuffle, seed=7,
                               drop_last=drop_last)
        s.set_epoch(3)
        assert P.distributed_sampler_indices(n, rank, world, shuffle=shuffle, seed=7, epoch=3,
                                             drop_last=drop_last) == list(iter(s))


def test_sampler_pads_with_duplicates_counted():
    # 5 frames over 2 ranks -> 6 evaluated, frame 0 twice
    got = [P.distributed_sampler_indices(5, r, 2) for r in range(2)]
    assert got == [[0, 2, 4], [1, 3, 0]]


@pytest.mark.parametrize("mode", ["before", "after", "before-after", "instant"])
@pytest.mark.parametrize("k", [0, 1, 2, 5])
@pytest.mark.parametrize("n", [1, 2, 3, 9])
def test_knn_window_matches_reference_restatement(mode, k, n):
    if mode == "instant" and k:
        with pytest.raises(ValueError):
            P.knn_window(n, k, mode)
        return
    frames = [f"f{i:03d}" for i in range(n)]
    w = P.knn_window(n, k, mode)
    for i, f in enumerate(frames):
        ref = [frames.index(x) for x in R.knn_frames(frames, f, k, mode)]
        got = [int(j) for j in w[i] if j >= 0]
        assert got == ref, (i, got, ref)


def test_temporal_windows_of_shards_tile_the_clip():
    tc = P.TemporalCAM(k=2, mode="before-after")
    full = P.knn_window(16, 2, "before-after")
    rows = [tc.window(16, r, 4).numpy() for r in range(4)]
    np.testing.assert_array_equal(np.concatenate(rows), full)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.full((2, 3), float(rank)) + torch.arange(6.).view(2, 3)
    q.put((rank, P.sync_tensor_across_gpus(t).numpy()))
    dist.destroy_process_group()


def test_sync_tensor_across_gpus_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    base = np.arange(6.).reshape(2, 3)
    want = np.concatenate([base, base + 1])
    for r in range(2):
        np.testing.assert_array_equal(res[r], want)


def test_sync_tensor_without_process_group_is_identity():
    t = torch.arange(4.)
    assert P.sync_tensor_across_gpus(t) is t
    assert P.sync_tensor_across_gpus(None) is None


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=1" in r.stderr
