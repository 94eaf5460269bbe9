"""tcam_wsol_video_amd — MI355X-native (gfx950) TCAM hot path.

CAM + bbox extraction for ResNet50-TCAM (sbelharbi/tcam-wsol-video) on
hand-written HIP kernels behind a C ABI (include/tcam_hip.h), with the
reference's model / CAM-extractor / BoxEvaluator API on top.
"""
from .models import (UnetTCAM, STDClassifier, ResNetEncoder, WGAP, create_model,  # noqa: F401
                     build_r50_tcam, build_r50_stdcl, TCAM, STD_CL)
from .metrics import BoxEvaluator, compute_bboxes_from_scoremaps, calculate_multiple_iou  # noqa
from .inference import CAMComputer, SegmentationCam, CAM, build_tcam_extractor  # noqa: F401

__all__ = ["UnetTCAM", "STDClassifier", "create_model", "BoxEvaluator", "CAMComputer",
           "SegmentationCam", "CAM", "compute_bboxes_from_scoremaps"]
