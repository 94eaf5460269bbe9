"""Build libtcam_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch
extension): the .so travels with the repo snapshot to the GPU box."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libtcam_hip.so")
SOURCES = ["conv.hip", "conv_x6.hip", "s3.hip", "pool.hip", "cam.hip", "bbox.hip", "bbox_multi.hip", "bilateral.hip", "train.hip", "enc_train.hip", "seed.hip", "frames.hip", "jpeg.hip", "stem.hip", "info.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
         "-Wno-unused-function", "-Wno-unused-variable"]


def _needs(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src, os.path.join(CSRC, "common.h"), os.path.join(CSRC, "s3_util.h"),
            os.path.join(os.path.dirname(HERE), "include", "tcam_hip.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    objdir = os.path.join(CSRC, "build")
    os.makedirs(objdir, exist_ok=True)
    jobs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(objdir, s + ".o")
        if force or _needs(obj, src):
            jobs.append([HIPCC, *FLAGS, "-c", src, "-o", obj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    objs = [os.path.join(objdir, s + ".o") for s in SOURCES]
    if force or jobs or not os.path.exists(OUT):
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT, *objs])
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
