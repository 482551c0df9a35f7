#!/usr/bin/env python3
"""Markdown summary of a rocprofv3 --kernel-trace --stats CSV (run_kernel_stats.csv): per kernel calls, total / mean /
min / max duration, share.   kernel_stats_csv.py <run_kernel_stats.csv> [title] > out.md"""
import csv
import sys


def main(path, title="kernel stats"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print("# %s\n" % title)
    print("Source: `rocprofv3 --kernel-trace --stats` (%s).\n" % path.split("/")[-1])
    print("| kernel | calls | total us | mean us | min us | max us | % |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        print("| `%s` | %s | %.1f | %.1f | %.1f | %.1f | %.2f |" % (
            r["Name"].replace("|", "/")[:140], r["Calls"], float(r["TotalDurationNs"]) / 1e3,
            float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3, float(r["Percentage"])))


if __name__ == "__main__":
    main(*sys.argv[1:])
