"""Conv-family timing of the TIMED region from a rocprofv3 kernel trace of bench.py, for
comparison with the bench line's live HIP-event roofline (roofline.avg_launch_ms,
roofline.conv_busy_ms_per_step):

    python scripts/trace_conv.py <..._kernel_trace.csv> --warmup W --steps K [--per-step 59]

The conv launches are taken in dispatch order; the first W*per_step belong to the warmup,
the next K*per_step to the timed region.  Prints the timed launches' average duration and
the union of their [start, end] intervals per step (the two forward streams overlap)."""
import argparse
import csv
import json

CONV = ("conv_x6_kernel", "conv3x3_thin_kernel", "stem_f16x3_kernel", "bottleneck_f16x3_kernel")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--per-step", type=int, default=59)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if any(k in r["Kernel_Name"] for k in CONV)]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    t = rows[a.warmup * a.per_step:(a.warmup + a.steps) * a.per_step]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in t)
    busy, c0, c1 = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > c1:
            busy += c1 - c0
            c0, c1 = s, e
        else:
            c1 = max(c1, e)
    busy += c1 - c0
    print(json.dumps({"timed_conv_launches": len(t),
                      "avg_launch_ms": round(sum(e - s for s, e in iv) / len(iv) / 1e6, 4),
                      "conv_busy_ms_per_step": round(busy / a.steps / 1e6, 3),
                      "span_ms_per_step": round((iv[-1][1] - iv[0][0]) / a.steps / 1e6, 3)}))


if __name__ == "__main__":
    main()
