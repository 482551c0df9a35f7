#!/usr/bin/env python3
"""Per-dispatch PMC counters from a rocprofv3 --pmc run (SQLite .db output), filtered by kernel name.

  pmc_db.py <dir-with-.db> <kernel-substring> [counter ...]   -> prints one row per dispatch
Used for the PMC passes under profiles/ (tools/ldpc_hr_probe.py and bench.py runs)."""
import glob
import sqlite3
import sys


def dispatches(path, kernel):
    rows = {}
    for f in glob.glob(path + "/**/*.db", recursive=True) + glob.glob(path + "/*.db"):
        c = sqlite3.connect(f)
        for did, name, cn, v, dur in c.execute(
                "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
            if kernel in name:
                d = rows.setdefault((f, did), {"kernel": name, "duration_ns": dur})
                d[cn] = d.get(cn, 0.0) + v
    return [rows[k] for k in sorted(rows)]


if __name__ == "__main__":
    ds = dispatches(sys.argv[1], sys.argv[2])
    names = sys.argv[3:] or sorted({k for d in ds for k in d if k not in ("kernel",)})
    print("n", len(ds))
    for i, d in enumerate(ds):
        print(i, " ".join("%s=%.4g" % (n, d.get(n, float("nan"))) for n in names))
