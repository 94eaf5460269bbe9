"""CPU, world_size 2 over gloo: the multi-GPU exchange step of the hot path
(one all-reduce of the BoxEvaluator counters, replacing the reference's
all_gather + sum in BoxEvaluator._synch_across_gpus, wsol_metrics.py:372-388)
and the frame sharding used by bench.py."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tcam_wsol_video_amd.metrics import BoxEvaluator
    ev = BoxEvaluator(list(np.arange(0, 1, 0.25)), device="cpu")
    ev.counters += torch.arange(ev.counters.numel(), dtype=torch.int32).view_as(ev.counters) * (rank + 1)
    ev.cnt = 3 + rank
    ev._synch_across_gpus()
    q.put((rank, ev.counters.numpy().copy(), ev.cnt, ev.compute()))
    dist.destroy_process_group()


def test_counter_allreduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    base = np.arange(3 * 3 * 4, dtype=np.int32).reshape(3, 3, 4)
    for rank, counters, cnt, acc in res:
        np.testing.assert_array_equal(counters, base * 3)  # rank0 x1 + rank1 x2
        assert cnt == 7
    assert res[0][3] == res[1][3]


def test_bench_frame_sharding_is_disjoint():
    import bench
    a = bench.make_clip(4, seed=1000 + 0)[0]
    b = bench.make_clip(4, seed=1000 + 1)[0]
    assert a.shape == (4, 3, 224, 224) and not torch.equal(a, b)


def _overflow_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tcam_wsol_video_amd import ops
    dev = torch.device("cpu")
    out = []
    # round 1: only rank 1's f16x3 flag is set -> both ranks raise the same error
    if rank == 1:
        ops.f16_overflow_flag(dev).fill_(1)
    for _ in range(2):
        try:
            ops.check_f16_overflow(dev, all_ranks=True)
            out.append(None)
        except FloatingPointError as e:
            out.append(str(e))
    # the collective still lines up afterwards (no rank left behind)
    t = torch.tensor([rank + 1.0])
    dist.all_reduce(t)
    q.put((rank, out, float(t)))
    dist.destroy_process_group()


def test_f16_overflow_check_is_rank_consistent_gloo_world2():
    """runner.py / training.py: an f16x3 overflow on ONE rank must stop every rank at the
    same check (the flag is MAX-reduced before the decision); the next check, with the
    flag reset, raises on none — and the group is still usable."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, out0, s0), (r1, out1, s1) = res
    assert out0[0] is not None and out0[0] == out1[0]
    assert out0[1] is None and out1[1] is None
    assert s0 == s1 == 3.0


def test_f16_overflow_redirect_keeps_side_work_apart():
    """training.prefetch_encoder: launches inside f16_overflow_into(flag) set that flag, not
    the device's; merge_f16_overflow ORs it in when the result is consumed."""
    from tcam_wsol_video_amd import ops
    dev = torch.device("cpu")
    ops.check_f16_overflow(dev, all_ranks=False)   # reset
    side = torch.zeros(1, dtype=torch.int32)
    with ops.f16_overflow_into(side):
        ops.f16_overflow_flag(dev).fill_(1)         # what a side-stream launch would set
    assert int(ops.f16_overflow_flag(dev)) == 0 and int(side) == 1
    ops.check_f16_overflow(dev, all_ranks=False)    # nothing yet
    ops.merge_f16_overflow(side)
    try:
        ops.check_f16_overflow(dev, all_ranks=False)
        raised = False
    except FloatingPointError:
        raised = True
    assert raised
