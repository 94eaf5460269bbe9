"""Render a rocprofv3 --stats kernel_stats.csv as a markdown table (profiles/*_summary.md).

    python scripts/prof_summary.py profiles/round1_bench_kernel_stats.csv "command" > out.md
"""
import csv
import sys


def main():
    path, cmd = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# rocprofv3 kernel summary: `{path}`\n")
    if cmd:
        print(f"Command: `{cmd}`\n")
    conv = [r for r in rows if "conv_x6_kernel" in r["Name"] or "conv3x3_thin_kernel" in r["Name"]]
    if conv:
        n = sum(int(r["Calls"]) for r in conv)
        t = sum(float(r["TotalDurationNs"]) for r in conv)
        print(f"conv family (conv_x6_kernel + conv3x3_thin_kernel): {n} launches, {t / 1e6:.2f} ms total, "
              f"average {t / n / 1e6:.4f} ms per launch ({100 * t / total:.1f} % of kernel time)\n")
    print("| kernel | calls | avg us | total ms | % |")
    print("|---|---|---|---|---|")
    for r in rows[:25]:
        name = r["Name"].replace("(anonymous namespace)::", "").replace("|", "/")
        name = name.split("((")[0][:90]
        print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main()
