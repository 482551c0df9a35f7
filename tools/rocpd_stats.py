#!/usr/bin/env python3
"""Kernel statistics (calls, average / total duration) from a rocprofv3 SQLite database (rocpd schema), as the
markdown table committed under profiles/: python tools/rocpd_stats.py results.db [title]."""
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute("select %s, count(*), avg(end - start), sum(end - start) from kernels group by %s "
                     "order by sum(end - start) desc" % (name, name)).fetchall()
    total = sum(r[3] for r in rows) or 1
    return [(r[0], r[1], r[2] / 1e3, r[3] / 1e3, 100.0 * r[3] / total) for r in rows]


def main():
    db = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else db
    print("# %s\n\n| kernel | calls | avg us | total us | total %% |\n|---|---|---|---|---|" % title)
    for k, n, avg, tot, pct in stats(db):
        print("| %s | %d | %.1f | %.1f | %.2f |" % (k[:110], n, avg, tot, pct))


if __name__ == "__main__":
    main()
