#!/usr/bin/env python3
"""TCAM training entry point (/root/reference main.py:33-167 for --task TCAM): frozen
stage-1 classifier, decoder trained from CAM-TMP seeds + dense-CRF + ELB size losses,
validation BoxAcc every epoch, best model and training checkpoints in the reference's
file formats — every tensor operation on the MI355X path.

    torchrun --nproc-per-node 8 main.py --task TCAM --encoder_name resnet50 \\
        --metadata_root <folds> --data_root <frames> --std_cams_folder <cams> \\
        --pretrained_classifier <stage-1 best model dir> --batch_size 32 --max_epochs 100 \\
        --sl_tc_knn 1 --sl_tc_knn_mode before
    python main.py --synthetic 2 --max_epochs 1     # seeded synthetic clips
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from tcam_wsol_video_amd.runner import train_main  # noqa: E402

if __name__ == "__main__":
    sys.exit(train_main())
