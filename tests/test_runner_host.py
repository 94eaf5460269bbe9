"""Host logic of main.py's knn_tc training batches and validation sweep (runner.py),
against restatements of the reference's loader (datasets/wsol_loader.py:447-503, 881-900;
process/parseit.py:642-643) and Trainer.evaluate (learning/train_wsol.py:1473-1480).
No GPU: only the host-side batch assembly is exercised."""
import argparse

import numpy as np
import pytest

from tcam_wsol_video_amd import runner


def _ref_left(lframes, frame, k):       # wsol_loader.py:447-451
    idx = lframes.index(frame)
    return lframes[max(0, idx - k): idx]


def _ref_right(lframes, frame, k):      # wsol_loader.py:453-458
    idx = lframes.index(frame)
    n = len(lframes)
    return lframes[min(idx + 1, n - 1): min(idx + k + 1, n)]


@pytest.mark.parametrize("n,k", [(1, 1), (2, 1), (5, 1), (5, 2), (7, 3), (3, 4)])
def test_knn_frames_matches_reference_slices(n, k):
    frames = [f"s/{i:03d}.jpg" for i in range(n)]
    for f in range(n):
        exp = _ref_left(frames, frames[f], k) + [frames[f]] + _ref_right(frames, frames[f], k)
        assert runner.knn_frames(frames, f, k) == exp
    # the reference's right slice starts at min(f + 1, n - 1): the last frame of a shot is
    # its own right neighbour
    if n > 1:
        assert runner.knn_frames(frames, n - 1, k)[-2:] == [frames[-1], frames[-1]]


def _split(n_shots=5, per_shot=(4, 1, 6, 3, 2)):
    shots = [f"vid{s}/shot{s}" for s in range(n_shots)]
    ids = [f"{sh}/{i:05d}.jpg" for sh, n in zip(shots, per_shot) for i in range(n)]
    labels = {i: 0 for i in ids}
    return runner.Split(ids, labels, {i: [] for i in ids}, lambda i: None, shot_ids=shots)


@pytest.mark.parametrize("knn,batch", [(0, 3), (1, 6), (1, 7), (2, 10)])
def test_train_batches_shot_mode(knn, batch):
    """One random frame (or its knn group) per shot, batch_size // (2 knn + 1) shots per
    batch (parseit.py:642-643); seq_iter = shot index, frm_iter = position in the group
    (wsol_loader.py:616-624) collated flat (_temporal_default_collate)."""
    sp = _split()
    args = argparse.Namespace(knn_tc=knn, batch_size=batch, seed=3)
    rng = np.random.default_rng(0)
    batches = list(runner.train_batches(sp, args, 0, 1, 2, rng))
    per = batch // (2 * knn + 1) if knn else batch
    order = runner.distributed_sampler_indices(5, 0, 1, shuffle=True, seed=3, epoch=2)
    assert len(batches) == -(-len(order) // per)
    rng2 = np.random.default_rng(0)
    seen = []
    for (ids, seq, frm), start in zip(batches, range(0, len(order), per)):
        assert len(ids) <= batch
        exp_ids, exp_seq, exp_frm = [], [], []
        for idx in order[start:start + per]:
            frames = sp.shots[sp.shot_ids[idx]]
            f = int(rng2.integers(0, len(frames)))
            g = (_ref_left(frames, frames[f], knn) + [frames[f]] +
                 _ref_right(frames, frames[f], knn)) if knn else [frames[f]]
            exp_ids += g
            exp_seq += [float(idx)] * len(g)
            exp_frm += [float(i) for i in range(len(g))]
            seen.append(idx)
        assert (ids, seq, frm) == (exp_ids, exp_seq, exp_frm)
    assert sorted(seen) == list(range(5))


def test_train_batches_frame_mode_and_knn_refusal():
    ids = [f"v/s/{i:03d}.jpg" for i in range(10)]
    sp = runner.Split(ids, {i: 0 for i in ids}, {i: [] for i in ids}, lambda i: None)
    args = argparse.Namespace(knn_tc=0, batch_size=4, seed=0)
    b = list(runner.train_batches(sp, args, 0, 1, 1, np.random.default_rng(0)))
    assert [len(x[0]) for x in b] == [4, 4, 2] and all(x[1] is None for x in b)
    assert sorted(i for x in b for i in x[0]) == ids
    args.knn_tc = 1
    with pytest.raises(SystemExit):
        list(runner.train_batches(sp, args, 0, 1, 1, np.random.default_rng(0)))


def test_synthetic_train_split_is_shot_indexed_with_knn():
    args = runner.parser(train=True).parse_args(["--synthetic", "2", "--knn_tc", "1"])
    sp = runner._splits(args, ["train", "val"])
    assert sp["train"].shot_ids is not None and len(sp["train"].shot_ids) == 2
    assert all(len(sp["train"].shots[s]) == 32 for s in sp["train"].shot_ids)
    assert sp["val"].shot_ids is None


def test_validation_interval_follows_the_dataset():
    """train_wsol.py:1473-1480: the validation split of CUB / ILSVRC / YTOv1 / YTOv2.2
    runs at VALID_FAST_CAM_CURVE_INTERVAL = .004 (constants.py:294)."""
    assert runner.VALID_FAST_CAM_CURVE_INTERVAL == .004
    assert len(np.arange(0, 1, .004)) == 250
    a = runner.parser(train=True).parse_args([])
    assert a.dataset == runner.YTOV22 and a.dataset in runner.FAST_VALID_DATASETS
    assert a.keep_last_n_checkpoints == 2          # config.py:171
    for t in ("sl_tc", "crf_tc", "max_sizepos_tc", "rgb_jcrf_tc"):
        assert getattr(a, f"{t}_start_ep") == 0 and getattr(a, f"{t}_end_ep") == -1


def test_loss_is_on_matches_elementary_loss():
    from tcam_wsol_video_amd.losses import ElementaryLoss, loss_is_on
    for s, e in [(None, None), (0, -1), (2, 5), (None, 3), (4, None), (3, 1)]:
        el = ElementaryLoss(start_epoch=s, end_epoch=e)
        for ep in range(8):
            assert loss_is_on(s, e, ep) == el.is_on(ep)
    assert loss_is_on(0, -1, 100) and not loss_is_on(2, 5, 6) and loss_is_on(2, 5, 5)
