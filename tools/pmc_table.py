#!/usr/bin/env python3
"""Per-kernel PMC table of a bench run from separate rocprofv3 --pmc passes (CSV output).

  pmc_table.py <out.json> <dir_sq_a> <dir_sq_b> <dir_fetch> <dir_write>

Pass A: SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
        SQ_BUSY_CYCLES; pass B: SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU
        GRBM_GUI_ACTIVE; FETCH_SIZE and WRITE_SIZE in passes of their own (MI355X_MICROARCH.md PMC slots).
Derived per kernel (per launch averages):
  valu_busy   = SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (1024 SIMDs x kernel cycles), kernel cycles =
                GRBM_GUI_ACTIVE / 8 (the sum over the 8 XCDs, MI355X_MICROARCH.md DVFS note) -- the fraction of
                SIMD cycles issuing VALU, the VALU roofline of an issue-bound kernel;
  valu_per_wave, lds_per_wave, wait / issue-stall / active shares of wave cycles;
  hbm_mb      = (2 x FETCH_SIZE + WRITE_SIZE) KiB (gfx950: FETCH_SIZE counts half of a wide stream).
"""
import collections
import csv
import glob
import json
import re
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    names = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            k = re.sub(r"srs_amd::|\(anonymous namespace\)::|void |at::native::", "", r["Kernel_Name"])
            k = re.sub(r"\(.*", "", k)[:60]
            key = (k, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[k] = r["Kernel_Name"]
        for (k, _), c in per.items():
            for n, v in c.items():
                agg[k][n].append(v)
    return agg


def mean(x):
    return sum(x) / len(x) if x else 0.0


def main(out, da, db, dfetch, dwrite):
    a, b, f, w = load(da), load(db), load(dfetch), load(dwrite)
    rows = {}
    for k in a:
        ca, cb = a[k], b.get(k, {})
        waves = mean(ca["SQ_WAVES"])
        cyc = mean(cb.get("GRBM_GUI_ACTIVE", [])) / 8.0
        wc = mean(ca["SQ_WAVE_CYCLES"]) or 1.0
        rows[k] = {
            "launches": len(ca["SQ_WAVES"]),
            "waves": waves,
            "kernel_cycles": cyc,
            "valu_per_wave": mean(ca["SQ_INSTS_VALU"]) / max(waves, 1),
            "valu_busy": mean(ca["SQ_ACTIVE_INST_VALU"]) * 4 / (1024 * cyc) if cyc else None,
            "lds_per_wave": mean(cb.get("SQ_INSTS_LDS", [])) / max(waves, 1),
            "lds_bank_conflict_cycles": mean(cb.get("SQ_LDS_BANK_CONFLICT", [])),
            "lds_array_busy": mean(cb.get("SQ_LDS_IDX_ACTIVE", [])) / (256 * cyc) if cyc else None,
            "wait_share": mean(ca["SQ_WAIT_ANY"]) / wc,
            "issue_stall_share": mean(ca["SQ_WAIT_INST_ANY"]) / wc,
            "active_share": mean(ca["SQ_ACTIVE_INST_ANY"]) / wc,
            "hbm_mb": (2 * mean(f.get(k, {}).get("FETCH_SIZE", [])) + mean(w.get(k, {}).get("WRITE_SIZE", []))) * 1024 / 1e6,
            "fetch_mb": 2 * mean(f.get(k, {}).get("FETCH_SIZE", [])) * 1024 / 1e6,
            "write_mb": mean(w.get(k, {}).get("WRITE_SIZE", [])) * 1024 / 1e6,
        }
    json.dump(rows, open(out, "w"), indent=1)
    print("%-60s %7s %9s %6s %6s %6s %6s %8s %8s" % ("kernel", "waves", "valu/w", "vbusy", "wait", "stall", "ldsbsy",
                                                    "rd MB", "wr MB"))
    for k, r in sorted(rows.items(), key=lambda kv: -kv[1]["kernel_cycles"]):
        print("%-60s %7.0f %9.0f %6.2f %6.2f %6.2f %6.2f %8.1f %8.1f" % (
            k, r["waves"], r["valu_per_wave"], r["valu_busy"] or 0, r["wait_share"], r["issue_stall_share"],
            r["lds_array_busy"] or 0, r["fetch_mb"], r["write_mb"]))


if __name__ == "__main__":
    main(*sys.argv[1:])
