#!/usr/bin/env python3
"""Kernel-trace summary (calls, average / total duration per kernel) from a rocprofv3 --kernel-trace SQLite
output (.db), as the markdown tables under profiles/.

  kernel_stats_db.py <dir-with-.db> [title]"""
import glob
import sqlite3
import sys


def stats(path):
    acc = {}
    for f in glob.glob(path + "/**/*.db", recursive=True) + glob.glob(path + "/*.db"):
        c = sqlite3.connect(f)
        q = ("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        for name, dur in c.execute(q):
            n, t = acc.get(name, (0, 0))
            acc[name] = (n + 1, t + dur)
    return acc


if __name__ == "__main__":
    acc = stats(sys.argv[1])
    total = sum(t for _, t in acc.values()) or 1
    print("# %s\n" % (sys.argv[2] if len(sys.argv) > 2 else "kernel stats"))
    print("| kernel | calls | avg us | total us | total % |\n|---|---|---|---|---|")
    for name, (n, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        print("| %s | %d | %.1f | %.1f | %.2f |" % (name[:110], n, t / n / 1e3, t / 1e3, 100.0 * t / total))
