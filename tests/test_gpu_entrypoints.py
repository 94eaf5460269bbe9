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


def _train(argv, final=None):
    """main.py's per-epoch JSON lines (the final test evaluation's line, main.py:117-160,
    goes to ``final`` when a list is given)."""
    lines = _run(train_main, argv)
    if final is not None:
        final.extend(lg["final_test"] for lg in lines if "final_test" in lg)
    return [lg for lg in lines if "epoch" in lg]


def _run_collect(fn, argv):
    buf, got = io.StringIO(), {}
    with contextlib.redirect_stdout(buf):
        assert fn(argv, collect=got) == 0
    out = [json.loads(ln) for ln in buf.getvalue().splitlines() if ln.startswith("{")]
    return out, got


def _oracle_vs_device(meta, frames, got, res, cam_fn):
    """The oracle CPU pipeline over the same files (PIL decode -> Pillow resize ->
    batch-1 forward -> CAM, inference_wsol.py:248-346): every fp32 CAM within 1e-4 of the
    device's; then the oracle evaluator (findContours sweep + BoxEvaluator,
    wsol_metrics.py:127-433) fed the DEVICE's uint8 CAMs and logits must reproduce the
    device counters exactly."""
    from PIL import Image
    ids, labels, boxes, sizes = load_metadata(os.path.join(meta, "test"))
    assert sorted(got) == sorted(ids)
    ev = BR.BoxEvaluatorRef(list(np.arange(0, 1, 0.01)))
    for i in ids:
        with Image.open(os.path.join(frames, i)) as im:
            img = np.asarray(im.convert("RGB"))
        x, _ = FRR.transform(img, 224, 224)
        cam_ref = cam_fn(torch.from_numpy(x)[None], labels[i])
        cam, u8, lo = got[i]
        assert np.abs(cam.double().numpy() - cam_ref).max() < 1e-4, i
        sm = np.minimum((u8.numpy().astype(np.float64) + 0.5) / 255.0, 1.0)
        _, order = torch.sort(lo, descending=True, stable=True)
        gt = np.asarray([resize_bbox(b, sizes[i], (224, 224)) for b in boxes[i]])
        ev.accumulate(sm, gt, labels[i], order.numpy())
    assert res["BoxAcc"] == [float(a) for a in ev.compute()]
    assert res["best_tau"] == ev.best_tau_list
    assert res["top1_loc"] == [float(v) for v in ev.top1]
    assert res["top5_loc"] == [float(v) for v in ev.top5]


def test_eval_on_metadata_dataset_matches_oracle(cuda, tmp_path):
    meta, frames = _write_dataset(str(tmp_path))
    model = build_r50_tcam(seed=9)
    CK.save_best_model(model, "TCAM", str(tmp_path / "best"), 12)
    outs, got = _run_collect(eval_main, ["--metadata_root", meta, "--data_root", frames,
                                         "--splits", "test", "--checkpoint",
                                         str(tmp_path / "best"), "--batch_size", "5",
                                         "--cam_curve_interval", "0.01"])
    out = outs[0]
    res = out["results"]["test"]
    assert out["checkpoint_step"] == 12 and res["frames"] == 12
    sd = {k: v.detach() for k, v in model.state_dict().items()}

    def cam_fn(x, label):
        _, fc, _ = R.tcam_forward(sd, x)
        return R.cam_to_scoremap(R.segmentation_cam(fc), (224, 224))[0]
    _oracle_vs_device(meta, frames, got, res, cam_fn)


def test_eval_std_cl_matches_oracle(cuda, tmp_path):
    """eval.py --task STD_CL: config 1's path (the stage-1 CAM, cams/cam.py:31-99 with the
    label as class index, inference_wsol.py:248-346) through CAMComputer's STD_CL branch."""
    from tcam_wsol_video_amd.models import build_r50_stdcl
    meta, frames = _write_dataset(str(tmp_path))
    model = build_r50_stdcl(seed=13)
    CK.save_best_model(model, "STD_CL", str(tmp_path / "best"), 4)
    outs, got = _run_collect(eval_main, ["--task", "STD_CL", "--metadata_root", meta,
                                         "--data_root", frames, "--splits", "test",
                                         "--checkpoint", str(tmp_path / "best"),
                                         "--batch_size", "5", "--cam_curve_interval", "0.01"])
    res = outs[0]["results"]["test"]
    assert outs[0]["task"] == "STD_CL" and res["frames"] == 12
    sd = {k: v.detach() for k, v in model.state_dict().items()}

    def cam_fn(x, label):
        _, A = R.stdcl_forward(sd, x)
        return R.std_cam(sd, A, label, (224, 224))[1]
    _oracle_vs_device(meta, frames, got, res, cam_fn)


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
    logs = _train(["--synthetic", "1", "--max_epochs", "2", "--batch_size", "16",
                             "--exp_path", exp, "--checkpoint_save", "2", "--sl_tc_knn", "1",
                             "--sl_tc_knn_mode", "before", "--cam_curve_interval", "0.01",
                             "--opt__step_size", "1", "--opt__gamma", "0.5"])
    # main.py:83-88 evaluates before the first epoch, then one line per epoch
    assert [lg["epoch"] for lg in logs] == [0, 1, 2]
    assert all(np.isfinite(lg["losses"]).all() for lg in logs[1:])
    assert [lg["lr"] for lg in logs[1:]] == [0.005, 0.0025]      # MyStepLR after each epoch
    it, cpt = CK.find_last_checkpoint(os.path.join(exp, "checkpoints"), CK.CHP_CP)
    # the reference's TCAM optimizer: ONE group over every parameter (instantiators.py:751)
    assert it == 4 and len(cpt[CK.CHP_O]["param_groups"]) == 1
    assert cpt[CK.CHP_LR]["last_epoch"] == 2
    assert CK._t_from(cpt[CK.CHP_T]) == pytest.approx(1.01 ** 2, rel=1e-6)
    out = _run(eval_main, ["--synthetic", "1", "--checkpoint", os.path.join(exp, "best_loc"),
                           "--cam_curve_interval", "0.01", "--splits", "test",
                           "--sl_tc_knn", "1", "--sl_tc_knn_mode", "before"])[0]
    assert out["results"]["test"]["frames"] == 32
    # resuming picks the last checkpoint up (epoch floor(4 / 2) = 2, main.py:78-81),
    # evaluates it and trains nothing more for max_epochs=2
    logs2 = _train(["--synthetic", "1", "--max_epochs", "2", "--batch_size", "16",
                              "--exp_path", exp, "--checkpoint_save", "100"])
    assert len(logs2) == 1 and logs2[0]["epoch"] == 2 and "losses" not in logs2[0]


def test_main_decays_t_and_switches_seeder(cuda, tmp_path):
    """DecayTemp (decay_temp.py:20-79) driven per epoch by main: t decays linearly from
    sl_tc_knn_t to sl_tc_min_t over sl_tc_knn_epoch_switch_uniform epochs and the seeder
    switches to seed_uniform from that epoch on (Trainer.train(epoch=e+1),
    train_wsol.py:944-965)."""
    exp = str(tmp_path / "exp")
    logs = _train(["--synthetic", "1", "--max_epochs", "3", "--batch_size", "32",
                             "--exp_path", exp, "--checkpoint_save", "100", "--sl_tc_knn", "1",
                             "--sl_tc_knn_mode", "before", "--sl_tc_knn_t", "2.0",
                             "--sl_tc_min_t", "0.5", "--sl_tc_knn_epoch_switch_uniform", "2",
                             "--cam_curve_interval", "0.05", "--opt__lr_scheduler", "False"])
    st = [lg["tmp_manager"] for lg in logs[1:]]
    assert st[0].startswith("epoch=1,sl_tc_knn_t=1.25,") and st[0].endswith("seed_weighted.")
    assert st[1].startswith("epoch=2,sl_tc_knn_t=0.5,") and st[1].endswith("seed_uniform.")
    assert st[2].startswith("epoch=3,sl_tc_knn_t=0.5,") and st[2].endswith("seed_uniform.")
    assert all(np.isfinite(lg["losses"]).all() for lg in logs[1:])
    assert all(lg["lr"] == 0.01 for lg in logs[1:])


def _val_oracle(args_list, interval):
    """The uint8 CAMs main.py's validation sees (same seeded model and synthetic split),
    through the oracle evaluator (findContours sweep + BoxEvaluator) at ``interval``."""
    from tcam_wsol_video_amd import runner
    from tcam_wsol_video_amd.models import create_model
    from tcam_wsol_video_amd.utils.seeding import seed_module_
    args = runner.parser(train=True).parse_args(args_list)
    model = create_model(**runner._model_kwargs(args))
    seed_module_(model, args.seed)
    model = model.to(torch.device("cuda", 0)).eval()
    val = runner._splits(args, ["train", "val"])["val"]
    got = {}
    runner.evaluate(model, val, args, torch.device("cuda", 0), collect=got,
                    cam_curve_interval=interval)
    ev = BR.BoxEvaluatorRef(list(np.arange(0, 1, interval)))
    for i in val.ids:
        _, u8, lo = got[i]
        sm = np.minimum((u8.numpy().astype(np.float64) + 0.5) / 255.0, 1.0)
        _, order = torch.sort(lo, descending=True, stable=True)
        ev.accumulate(sm, np.asarray(val.gt[i]), val.labels[i], order.numpy())
    return ev


@pytest.mark.parametrize("dataset,interval", [("YouTube-Objects-v2.2", 0.004),
                                              ("OpenImages", 0.01)])
def test_main_validation_sweeps_the_reference_tau_grid(cuda, tmp_path, dataset, interval):
    """Trainer.evaluate (train_wsol.py:1473-1480): main.py's validation of a YTO / CUB /
    ILSVRC run sweeps VALID_FAST_CAM_CURVE_INTERVAL = .004 (250 taus, constants.py:294)
    whatever --cam_curve_interval says; other datasets keep it.  BoxAcc and best tau equal
    the oracle evaluator's at that grid on the device's uint8 CAMs (model selection,
    train_wsol.py:1681-1726, runs on these numbers)."""
    argv = ["--synthetic", "1", "--max_epochs", "0", "--batch_size", "16", "--exp_path",
            str(tmp_path / "exp"), "--cam_curve_interval", "0.01", "--dataset", dataset]
    logs = _train(argv)
    assert len(logs) == 1 and logs[0]["epoch"] == 0
    res = logs[0]["val"]
    assert res["cam_curve_interval"] == interval
    ev = _val_oracle(argv, interval)
    assert res["BoxAcc"] == [float(a) for a in ev.compute()]
    assert res["best_tau"] == ev.best_tau_list
    assert len(ev.cam_threshold_list) == (250 if interval == 0.004 else 100)


def test_main_knn_tc_rgb_joint_crf(cuda, tmp_path):
    """main.py --knn_tc 1 --rgb_jcrf_tc True (losses/tcam.py:158-232 over the knn_tc
    loader's shot groups, wsol_loader.py:479-503): the RgbJoint slot is on and finite, its
    epoch window gates it (rgb_jcrf_tc_start_ep 2: zero in epoch 1), and the batch holds
    batch_size // 3 shots of 3 frames, filled to batch_size."""
    exp = str(tmp_path / "exp")
    logs = _train(["--synthetic", "4", "--max_epochs", "2", "--batch_size", "8",
                             "--exp_path", exp, "--checkpoint_save", "100", "--knn_tc", "1",
                             "--rgb_jcrf_tc", "True", "--rgb_jcrf_tc_start_ep", "2",
                             "--cam_curve_interval", "0.05", "--sl_tc_knn", "1",
                             "--sl_tc_knn_mode", "before"])
    l1, l2 = logs[1]["losses"], logs[2]["losses"]
    assert len(l1) == 5 and len(l2) == 5
    assert l1[4] == 0.0 and np.isfinite(l2[4]) and l2[4] != 0.0
    assert all(np.isfinite(l1)) and all(np.isfinite(l2))
    # 4 shots at 8 // 3 = 2 shots per batch: 2 steps per epoch
    assert logs[2]["step"] == 4
    it, cpt = CK.find_last_checkpoint(os.path.join(exp, "checkpoints"), CK.CHP_CP)
    assert [n for n, _ in cpt[CK.CHP_T]] == ["con_ran_field_tcams",
                                             "rgb_joint_con_ran_field_tcams",
                                             "max_size_positive_tcams", "self_learning_tcams"]


def test_main_box_v2_metric_best_loc_and_best_cl(cuda, tmp_path):
    """main.py --box_v2_metric True (parseit.py:684-689: multi_contour_eval and
    multi_iou_eval): validation BoxAcc from every contour's box, bit-equal to the oracle
    evaluator with multi_contour_eval on the device's uint8 CAMs; model selection on the
    mean BoxAcc over the IoU thresholds (train_wsol.py:1515-1519); the classification
    accuracy (_compute_accuracy, train_wsol.py:1400-1435) and its BEST_CL model
    (train_wsol.py:1735-1756) beside BEST_LOC; the final test evaluation of both
    (main.py:117-160)."""
    exp = str(tmp_path / "exp")
    argv = ["--synthetic", "1", "--max_epochs", "1", "--batch_size", "16", "--exp_path", exp,
            "--checkpoint_save", "100", "--cam_curve_interval", "0.01", "--box_v2_metric",
            "True", "--dataset", "OpenImages"]
    final = []
    logs = _train(argv, final)
    assert [lg["epoch"] for lg in logs] == [0, 1]
    res0 = logs[0]["val"]
    assert res0["box_v2_metric"] is True
    assert res0["localization"] == pytest.approx(float(np.average(res0["BoxAcc"])), abs=0)
    # the epoch-0 validation against the oracle (multi-contour evaluator, argmax accuracy)
    from tcam_wsol_video_amd import runner
    from tcam_wsol_video_amd.models import create_model
    from tcam_wsol_video_amd.utils.seeding import seed_module_
    args = runner.parser(train=True).parse_args(argv)
    model = create_model(**runner._model_kwargs(args))
    seed_module_(model, args.seed)
    model = model.to(cuda).eval()
    val = runner._splits(args, ["train", "val"])["val"]
    got = {}
    runner.evaluate(model, val, args, cuda, collect=got, cam_curve_interval=0.01)
    ev = BR.BoxEvaluatorRef(list(np.arange(0, 1, 0.01)), multi_contour_eval=True)
    for i in val.ids:
        _, u8, lo = got[i]
        sm = np.minimum((u8.numpy().astype(np.float64) + 0.5) / 255.0, 1.0)
        _, order = torch.sort(lo, descending=True, stable=True)
        ev.accumulate(sm, np.asarray(val.gt[i]), val.labels[i], order.numpy())
    assert res0["BoxAcc"] == [float(a) for a in ev.compute()]
    assert res0["best_tau"] == ev.best_tau_list
    assert res0["classification_acc"] == ev.cls_correct / float(ev.cnt) * 100
    # both best models exist; the frozen classifier's accuracy never improves after the
    # first evaluation, so BEST_CL is the step-0 model (PerformanceMeter: first maximum)
    it_cl, _ = CK.find_last_checkpoint(os.path.join(exp, "best_cl"), CK.CHP_BEST_M)
    it_loc, _ = CK.find_last_checkpoint(os.path.join(exp, "best_loc"), CK.CHP_BEST_M)
    assert it_cl == 0 and it_loc in (0, logs[1]["step"])
    assert len(final) == 1 and sorted(final[0]) == ["best_cl", "best_loc"]
    assert final[0]["best_cl"]["checkpoint_step"] == 0
    assert final[0]["best_cl"]["frames"] == 32


@pytest.mark.parametrize("amp", [False, True])
def test_main_stage1_std_cl_trains_and_feeds_tcam(cuda, tmp_path, amp):
    """main.py --task STD_CL --arch STDClassifier --freeze_encoder False (README.md:239-266,
    stage 1): the classifier trains end to end (encoder backward on the device), validation
    selects best_loc / best_cl, the checkpoint holds the reference's two SGD groups, resume
    works, and the best model loads as TCAM's --pretrained_classifier (README.md:267-276)."""
    exp = str(tmp_path / "exp")
    argv = ["--task", "STD_CL", "--arch", "STDClassifier", "--freeze_cl", "False",
            "--freeze_encoder", "False", "--support_background", "True", "--synthetic", "1",
            "--max_epochs", "2", "--batch_size", "8", "--exp_path", exp, "--checkpoint_save",
            "3", "--cam_curve_interval", "0.01", "--opt__lr", "0.001", "--opt__step_size", "1",
            "--opt__gamma", "0.9", "--amp", str(amp)]
    final = []
    logs = _train(argv, final)
    assert [lg["epoch"] for lg in logs] == [0, 1, 2]
    assert all(np.isfinite(lg["loss"]) for lg in logs[1:])
    assert logs[1]["lr"] == pytest.approx([0.0009, 0.009], rel=1e-6)
    assert logs[2]["lr"] == pytest.approx([0.00081, 0.0081], rel=1e-6)
    if not amp:   # (AMP: GradScaler may back off on its first steps, as torch's does)
        assert all(lg["skipped_steps"] == 0 for lg in logs[1:])
    it, cpt = CK.find_last_checkpoint(os.path.join(exp, "checkpoints"), CK.CHP_CP)
    assert it == 8 and len(cpt[CK.CHP_O]["param_groups"]) == 2
    assert [len(g["params"]) for g in cpt[CK.CHP_O]["param_groups"]] == [129, 32]
    assert cpt[CK.CHP_T] == [["cl_loss", 0.0]]
    assert final and set(final[0]) == {"best_loc", "best_cl"}
    for key in ("best_loc", "best_cl"):
        assert os.path.isdir(os.path.join(exp, key))
    # TCAM stage 2 reads the stage-1 classifier
    tcam = build_r50_tcam(seed=1)
    CK.load_pretrained_classifier(tcam, os.path.join(exp, "best_loc"))
    _, best = CK.find_last_checkpoint(os.path.join(exp, "best_loc"), CK.CHP_BEST_M)
    for k, v in best["encoder"].items():
        assert torch.equal(tcam.encoder.state_dict()[k].cpu(), v.cpu()), k
    # resume: the last checkpoint (epoch floor(8 / 4) = 2) is evaluated, nothing more trained
    logs2 = _train(argv[:-2] + ["--checkpoint_save", "100", "--amp", str(amp)])
    assert len(logs2) == 1 and logs2[0]["epoch"] == 2
