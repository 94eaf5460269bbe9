"""Per-launch conv timing of one forward (one stream, HIP events around every conv launch):
which layers of a model's x6 forward take the time, at the bench's frame count.

    python scripts/layer_times.py [r50|vgg16|inceptionv3] [frames]

Prints one line per conv launch (shape descriptor M/K/N/taps/sources, ms, TF) sorted by
time, and the total."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tcam_wsol_video_amd import ops  # noqa: E402
from tcam_wsol_video_amd.models import (build_inceptionv3_tcam, build_r50_tcam,  # noqa: E402
                                        build_vgg16_tcam)


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "r50"
    size = 299 if arch == "inceptionv3" else 224
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else (8 if arch == "inceptionv3" else 32)
    build = {"r50": build_r50_tcam, "vgg16": build_vgg16_tcam,
             "inceptionv3": build_inceptionv3_tcam}[arch]
    dev = torch.device("cuda")
    model = build(seed=0).to(dev)
    x, _, _ = bench.make_clip(frames, seed=1000, size=size)
    x = x.to(dev)
    with torch.no_grad():
        for _ in range(3):
            model(x, want_fcams=False)
        torch.cuda.synchronize()
        rows = {}
        for _ in range(5):
            timer = []
            ops.set_launch_timer(timer)
            model(x, want_fcams=False)
            torch.cuda.synchronize()
            ops.set_launch_timer(None)
            for i, t in enumerate(timer):
                ms = t[2].elapsed_time(t[3])
                key = (i, t[4] if len(t) > 4 else t[0])
                rows[key] = (min(rows.get(key, (1e9,))[0], ms), t[1])
    tot = sum(v[0] for v in rows.values())
    fl = sum(v[1] for v in rows.values())
    print(f"{arch} {frames} frames: {len(rows)} conv launches, {tot:.3f} ms, "
          f"{fl / tot / 1e9:.1f} TF")
    for (i, desc), (ms, f) in sorted(rows.items(), key=lambda kv: -kv[1][0]):
        print(f"{i:3d} {desc:40s} {ms:7.3f} ms {f / ms / 1e9:6.1f} TF {100 * ms / tot:5.1f} %")


if __name__ == "__main__":
    main()
