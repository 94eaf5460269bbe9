"""What the GPU does during the TIMED region of bench.py, from a rocprofv3 kernel trace:

    python scripts/trace_timeline.py <..._kernel_trace.csv> --warmup W --steps K [--per-step 59]

The timed region is the span of the conv launches W*per_step .. (W+K)*per_step in dispatch
order (as scripts/trace_conv.py).  Reports, per step: the span, the union of all kernels'
busy intervals (span - union = time with NO kernel on the device), and per kernel family
the summed duration, the launch count and the time during which that family ran ALONE
(nothing else on the device: the part of it no other stream hides)."""
import argparse
import csv
import json
import re
from collections import defaultdict

CONV = ("conv_x6_kernel", "conv3x3_thin_kernel")


def family(name: str) -> str:
    n = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    if n.startswith("at::") or "at::native" in name:
        return "torch:" + n.split("<")[0].split("::")[-1]
    return n.split("<")[0] + ("<" + n.split("<", 1)[1][:40] if "<" in n else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--per-step", type=int, default=59)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    conv = sorted((r for r in rows if any(k in r["Kernel_Name"] for k in CONV)),
                  key=lambda r: int(r["Dispatch_Id"]))
    t = conv[a.warmup * a.per_step:(a.warmup + a.steps) * a.per_step]
    t0 = min(int(r["Start_Timestamp"]) for r in t)
    t1 = max(int(r["End_Timestamp"]) for r in t)
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        s, e = max(s, t0), min(e, t1)
        if e > s:
            ev.append((s, e, family(r["Kernel_Name"])))
    # sweep: union busy and per-family "alone" time
    pts = []
    for s, e, f in ev:
        pts.append((s, 1, f))
        pts.append((e, -1, f))
    pts.sort(key=lambda x: (x[0], x[1]))
    active = defaultdict(int)
    busy = 0
    alone = defaultdict(int)
    last = t0
    for x, d, f in pts:
        n = sum(active.values())
        if n > 0:
            busy += x - last
            if n == 1:
                (only,) = [k for k, v in active.items() if v]
                alone[only] += x - last
        last = x
        active[f] += d
        if active[f] == 0:
            del active[f]
    fams = defaultdict(lambda: [0, 0])
    for s, e, f in ev:
        fams[f][0] += e - s
        fams[f][1] += 1
    K = a.steps
    out = {"span_ms_per_step": round((t1 - t0) / K / 1e6, 3),
           "busy_union_ms_per_step": round(busy / K / 1e6, 3),
           "idle_ms_per_step": round((t1 - t0 - busy) / K / 1e6, 3),
           "families": {f: {"sum_ms": round(v[0] / K / 1e6, 3), "launches": round(v[1] / K, 2),
                            "alone_ms": round(alone[f] / K / 1e6, 3)}
                        for f, v in sorted(fams.items(), key=lambda kv: -kv[1][0])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
