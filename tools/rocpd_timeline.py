#!/usr/bin/env python3
"""Kernel timeline of the last steps of a rocprofv3 --kernel-trace run (rocpd SQLite): per kernel its start / end
(us from the step's first kernel), queue and name; per step the GPU-busy union and the idle gaps.  A step starts at
each dispatch of the anchor kernel (name substring).
  rocpd_timeline.py results.db <anchor> [steps=2] [min_gap_us=5]"""
import sqlite3
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("srs_amd::", "")
    return n.split("(")[0][:80]


def main():
    db, anchor = sys.argv[1], sys.argv[2]
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    min_gap = float(sys.argv[4]) if len(sys.argv) > 4 else 5.0
    c = sqlite3.connect(db)
    rows = c.execute("select start, end, queue_id, name from kernels order by start").fetchall()
    print("kernels per queue:", c.execute("select queue_id, count(*) from kernels group by queue_id").fetchall())
    starts = [r[0] for r in rows if anchor in r[3]]
    if len(starts) < 2:
        print("anchor %r seen %d times" % (anchor, len(starts)))
        return
    print("all step intervals (us):", " ".join("%.0f" % ((b - a) / 1e3) for a, b in zip(starts[:-1], starts[1:])))
    bounds = list(zip(starts[:-1], starts[1:]))
    if nsteps < 0:  # the slowest step after the first five (warm-up, setup)
        bounds = [max(bounds[5:], key=lambda ab: ab[1] - ab[0])]
    else:
        bounds = bounds[-nsteps:]
    for s0, s1 in bounds:
        ks = [r for r in rows if s0 <= r[0] < s1]
        print("## step: %.1f us between anchors, %d kernels" % ((s1 - s0) / 1e3, len(ks)))
        busy, cur_s, cur_e, gaps = 0, None, None, []
        for st, en, q, name in ks:
            if cur_e is None or st > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    if (st - cur_e) / 1e3 >= min_gap:
                        gaps.append(((cur_e - s0) / 1e3, (st - cur_e) / 1e3, short(name)))
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
        if cur_e is not None:
            busy += cur_e - cur_s
        print("busy %.1f us; gaps >= %.0f us (at, length, next kernel):" % (busy / 1e3, min_gap))
        for g in gaps:
            print("  %8.1f %7.1f  %s" % g)
        for st, en, q, name in ks:
            print("  %8.1f %8.1f %6.1f q%-3d %s" % ((st - s0) / 1e3, (en - s0) / 1e3, (en - st) / 1e3, q,
                                                  short(name)))


if __name__ == "__main__":
    main()
