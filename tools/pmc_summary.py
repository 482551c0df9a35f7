#!/usr/bin/env python3
"""Summarises rocprofv3 outputs for the LDPC decoder kernel.

  pmc_summary.py traffic <fetch_dir> <write_dir> <out.json> [kernel substring ...]
      HBM traffic per launch from separate FETCH_SIZE / WRITE_SIZE passes
      (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of a wide coalesced
      stream on gfx950 -> doubled; both are in KiB).
  pmc_summary.py stats <kernel_stats.csv> <out.md>
"""
import csv
import glob
import json
import sys

KERNEL = "ldpc_decode_kernel"


def counter(dirname, name, kernel=KERNEL):
    files = glob.glob(dirname + "/**/*counter_collection.csv", recursive=True)
    vals = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return vals


def traffic(fetch_dir, write_dir, out, *kernels):
    kernels = kernels or (KERNEL,)
    per = {}
    for k in kernels:
        fetch = counter(fetch_dir, "FETCH_SIZE", k)
        write = counter(write_dir, "WRITE_SIZE", k)
        f = sum(fetch) / len(fetch)
        w = sum(write) / len(write)
        per[k] = {
            "launches": [len(fetch), len(write)],
            "fetch_size_kib_raw": f,
            "write_size_kib": w,
            "hbm_read_bytes_corrected": 2 * f * 1024,
            "hbm_write_bytes": w * 1024,
            "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
        }
    res = dict(per[kernels[0]]) if len(kernels) == 1 else {"kernels": per}
    res["kernel"] = " + ".join(kernels)
    res["hbm_bytes_per_launch"] = sum(v["hbm_bytes_per_launch"] for v in per.values())
    res["note"] = ("FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half of a wide coalesced read); "
                   "separate --pmc passes for FETCH_SIZE and WRITE_SIZE; per launch of each kernel, summed")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


def stats(path, out):
    rows = list(csv.DictReader(open(path)))
    with open(out, "w") as fo:
        fo.write("| kernel | calls | total ns | avg ns | min ns | max ns | % |\n|---|---|---|---|---|---|---|\n")
        for r in rows:
            fo.write("| %s | %s | %s | %s | %s | %s | %s |\n" % (
                r["Name"][:90], r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["MinNs"], r["MaxNs"],
                r["Percentage"]))
    print(open(out).read())


if __name__ == "__main__":
    if sys.argv[1] == "traffic":
        traffic(*sys.argv[2:])
    else:
        stats(*sys.argv[2:4])
