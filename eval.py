#!/usr/bin/env python3
"""Evaluation entry point (the behaviour the reference's eval.py intends):
load the best model, run CAM + bbox extraction over the requested splits on the MI355X
path, print BoxAcc / top-1 / top-5 localisation as one JSON line.

    python eval.py --task TCAM --encoder_name resnet50 --checkpoint <dir> \\
        --metadata_root <folds>/YouTube-Objects-v1.0 --data_root <frames> --splits test
    python eval.py --synthetic 4            # seeded YTOv2.2-shaped clips, no dataset
    torchrun --nproc-per-node 8 eval.py ...  # frames sharded as DistributedSampler
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from tcam_wsol_video_amd.runner import eval_main  # noqa: E402

if __name__ == "__main__":
    sys.exit(eval_main())
