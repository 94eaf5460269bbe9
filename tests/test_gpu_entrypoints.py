"""eval.py / main.py (tcam_wsol_video_amd/runner.py) end to end on the GPU:

* eval on an on-disk dataset in the reference's WSOL metadata layout (JPEG frames,
  image_ids / class_labels / image_sizes / localization.txt) with a best-model checkpoint,
  against the oracle's CPU pipeline on the same files (PIL decode -> Pillow resize ->
  batch-1 forward -> findContours sweep -> BoxEvaluator, inference_wsol.py:248-457);
* main.py on synthetic clips: one epoch of TCAM training with CAM-TMP seeds, checkpoints
  and best model in the reference formats, then eval.py from that best model.
"""
import contextlib
import io
import json
import os

import numpy as np
import pytest
import torch

from oracle import bbox_ref as BR
from oracle import frames_ref as FRR
from oracle import model_ref as R
from tcam_wsol_video_amd import checkpoints as CK
from tcam_wsol_video_amd.metrics import resize_bbox
from tcam_wsol_video_amd.models import build_r50_tcam
from tcam_wsol_video_amd.runner import eval_main, load_metadata, train_main
from tcam_wsol_video_amd.utils.seeding import synthetic_boxes, synthetic_clip

pytestmark = pytest.mark.gpu


def _write_dataset(root, n_shots=2, n_frames=6):
    from PIL import Image
    meta = os.path.join(root, "meta", "test")
    os.makedirs(meta)
    lines = {"image_ids": [], "class_labels": [], "image_sizes": [], "localization": []}
    for s in range(n_shots):
        clip = synthetic_clip(n_frames, seed=70 + s)
        boxes = synthetic_boxes(clip, 480)     # x scale exact; y rescaled below
        for t in range(n_frames):
            i = f"car/data/{s:04d}/shots/001/frame{t:04d}.jpg"
            path = os.path.join(root, "frames", i)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            Image.fromarray(clip[t]).save(path, quality=95)
            x0, y0, x1, y1 = boxes[t]
            lines["image_ids"].append(i)
            lines["class_labels"].append(f"{i},{3 + s}")
            lines["image_sizes"].append(f"{i},480,360")
            lines["localization"].append(f"{i},{x0 + 0.25},{y0 * 360 / 480 + 0.5},"
                                         f"{x1 - 0.25},{y1 * 360 / 480}")
    for k, v in lines.items():
        with open(os.path.join(meta, k + ".txt"), "w") as f:
            f.write("\n".join(v) + "\n")
    return os.path.join(root, "meta"), os.path.join(root, "frames")


def _run(fn, argv):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert fn(argv) == 0
    return [json.loads(ln) for ln in buf.getvalue().splitlines() if ln.startswith("{")]


def test_eval_on_metadata_dataset_matches_oracle(cuda, tmp_path):
    from PIL import Image
    meta, frames = _write_dataset(str(tmp_path))
    model = build_r50_tcam(seed=9)
    CK.save_best_model(model, "TCAM", str(tmp_path / "best"), 12)
    out = _run(eval_main, ["--metadata_root", meta, "--data_root", frames, "--splits", "test",
                           "--checkpoint", str(tmp_path / "best"), "--batch_size", "5",
                           "--cam_curve_interval", "0.01"])[0]
    res = out["results"]["test"]
    assert out["checkpoint_step"] == 12 and res["frames"] == 12
    # the oracle CPU pipeline over the same files
    ids, labels, boxes, sizes = load_metadata(os.path.join(meta, "test"))
    sd = {k: v.detach() for k, v in model.state_dict().items()}
    taus = list(np.arange(0, 1, 0.01))
    ev = BR.BoxEvaluatorRef(taus)
    for i in ids:
        with Image.open(os.path.join(frames, i)) as im:
            img = np.asarray(im.convert("RGB"))
        x, _ = FRR.transform(img, 224, 224)
        lo, fc, _ = R.tcam_forward(sd, torch.from_numpy(x)[None])
        sm = R.cam_to_scoremap(R.segmentation_cam(fc), (224, 224))[0]
        _, order = torch.sort(lo[0], descending=True, stable=True)
        gt = np.asarray([resize_bbox(b, sizes[i], (224, 224)) for b in boxes[i]])
        ev.accumulate(sm, gt, labels[i], order.numpy())
    ref = ev.compute()
    # CAMs agree to 1e-4; a frame whose uint8 CAM straddles a level may move one count
    for a, b in zip(res["BoxAcc"], ref):
        assert abs(a - b) <= 100.0 / 12 + 1e-9, (res["BoxAcc"], ref)


def test_eval_device_and_host_jpeg_decode_agree(cuda, tmp_path):
    """eval.py on an on-disk JPEG dataset: device decode (default) and PIL host decode
    (--jpeg_decode host, the reference's Image.open(...).convert('RGB')) give identical
    results -- the decode is bit-identical, so every counter is."""
    meta, frames = _write_dataset(str(tmp_path))
    model = build_r50_tcam(seed=11)
    CK.save_best_model(model, "TCAM", str(tmp_path / "best"), 3)
    args = ["--metadata_root", meta, "--data_root", frames, "--splits", "test",
            "--checkpoint", str(tmp_path / "best"), "--batch_size", "4",
            "--cam_curve_interval", "0.01"]
    dev = _run(eval_main, args)[0]["results"]["test"]
    host = _run(eval_main, args + ["--jpeg_decode", "host"])[0]["results"]["test"]
    def metrics(r):   # drop the timing fields
        return {k: v for k, v in r.items() if not k.startswith("frames_per_s")}
    assert metrics(dev) == metrics(host) and len(metrics(dev)) >= 5


def test_main_trains_and_eval_reads_its_best_model(cuda, tmp_path):
    exp = str(tmp_path / "exp")
    logs = _run(train_main, ["--synthetic", "1", "--max_epochs", "2", "--batch_size", "16",
                             "--exp_path", exp, "--checkpoint_save", "2", "--sl_tc_knn", "1",
                             "--sl_tc_knn_mode", "before", "--cam_curve_interval", "0.01"])
    assert [lg["epoch"] for lg in logs] == [1, 2]
    assert all(np.isfinite(lg["losses"]).all() for lg in logs)
    it, cpt = CK.find_last_checkpoint(os.path.join(exp, "checkpoints"), CK.CHP_CP)
    assert it == 4 and len(cpt[CK.CHP_O]["param_groups"]) == 2
    assert CK._t_from(cpt[CK.CHP_T]) == pytest.approx(1.01 ** 2, rel=1e-6)
    out = _run(eval_main, ["--synthetic", "1", "--checkpoint", os.path.join(exp, "best_loc"),
                           "--cam_curve_interval", "0.01", "--splits", "test",
                           "--sl_tc_knn", "1", "--sl_tc_knn_mode", "before"])[0]
    assert out["results"]["test"]["frames"] == 32
    # resuming picks the last checkpoint up and trains nothing more for max_epochs=2
    logs2 = _run(train_main, ["--synthetic", "1", "--max_epochs", "2", "--batch_size", "16",
                              "--exp_path", exp, "--checkpoint_save", "100"])
    assert logs2 == []
