"""tcam_wsol_video_amd — MI355X-native (gfx950) TCAM hot path.

CAM + bbox extraction for the TCAM family (ResNet50 / VGG16 / InceptionV3,
sbelharbi/tcam-wsol-video), the dense-CRF bilateral filter and the decoder training
step, on hand-written HIP kernels behind a C ABI (include/tcam_hip.h), with the
reference's model / CAM-extractor / BoxEvaluator / DenseCRFLoss API on top.
"""
from .models import (UnetTCAM, STDClassifier, ResNetEncoder, WGAP, create_model,  # noqa: F401
                     build_r50_tcam, build_r50_stdcl, build_vgg16_tcam,
                     build_inceptionv3_tcam, build_stdcl, TCAM, STD_CL)
from .backbones import VGGEncoder, InceptionV3Encoder  # noqa: F401
from .metrics import BoxEvaluator, compute_bboxes_from_scoremaps, calculate_multiple_iou  # noqa
from .inference import CAMComputer, SegmentationCam, CAM, build_tcam_extractor  # noqa: F401
from .crf import DenseCRFLoss, ColorDenseCRFLoss  # noqa: F401
from .seeding import TCAMSeeder, GetRoiSingleCam, prepare_std_cams  # noqa: F401
from . import camstore, checkpoints  # noqa: F401

__all__ = ["UnetTCAM", "STDClassifier", "create_model", "BoxEvaluator", "CAMComputer",
           "SegmentationCam", "CAM", "compute_bboxes_from_scoremaps", "DenseCRFLoss",
           "ColorDenseCRFLoss", "VGGEncoder", "InceptionV3Encoder", "TCAMSeeder",
           "GetRoiSingleCam", "prepare_std_cams"]
