#!/usr/bin/env python3
"""VALU-issue model of the high-rate LDPC decoder from a rocprofv3 --pmc pass over tools/ldpc_hr_probe.py.

  pmc_valu_model.py <pmc_dir> <out.json>

The probe launches ldpc_decode_hr_kernel on 4,544 BG1 Z=384 codeblocks at fixed iteration counts (random LLRs never
pass the CRC): for it in (1, 2, 3, 4, 6), for crc in (off, CRC24B), 1 warm-up + 10 launches.  SQ_INSTS_VALU and
SQ_WAVES per launch give the VALU wave-instructions per codeblock; a linear fit over the iteration counts (CRC on,
the PUSCH decoder's configuration) splits them into a per-codeblock fixed part and a per-iteration part.  SQ_ACTIVE_INST_VALU (quad-cycles in which a SIMD issued VALU work) gives the VALU issue
cycles the same way -- per wave-instruction it is ~2.7 cycles for plain 32-bit ops and ~4.3 for packed / 3-source
ones at this occupancy, so instruction counts alone understate the bound -- and bench.py scales the cycle fit to the
pipeline's measured iterations: valu issue bound = cycles / (1,024 SIMDs x 2.4 GHz), frac = bound / kernel time.
Counters (one pass): SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE."""
import csv
import glob
import json
import sys

import numpy as np

KERNEL = "ldpc_decode_hr_kernel"
NCB = 4544
ITS = (1, 2, 3, 4, 6)


def per_dispatch(pmc_dir):
    d = {}
    for f in glob.glob(pmc_dir + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            d.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def main(pmc_dir, out):
    rows = per_dispatch(pmc_dir)
    assert len(rows) == len(ITS) * 2 * 11, len(rows)
    res = {"kernel": KERNEL, "codeblocks_per_launch": NCB, "source": "rocprofv3 --pmc over tools/ldpc_hr_probe.py"}
    for ci, crc in enumerate(("nocrc", "crc24b")):
        valu, waves, lds, cyc, busy = [], [], [], [], []
        for ii, it in enumerate(ITS):
            blk = rows[(ii * 2 + ci) * 11 + 1:(ii * 2 + ci) * 11 + 11]  # skip the warm-up launch
            valu.append(np.mean([r["SQ_INSTS_VALU"] for r in blk]) / NCB)
            waves.append(np.mean([r["SQ_WAVES"] for r in blk]) / NCB)
            lds.append(np.mean([r.get("SQ_INSTS_LDS", 0.0) for r in blk]) / NCB)
            cyc.append(np.mean([r.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 for r in blk]) / NCB)
            busy.append(np.mean([r.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / (1024 * r["GRBM_GUI_ACTIVE"] / 8)
                                 for r in blk if r.get("GRBM_GUI_ACTIVE")] or [0.0]))
        sl, ic = np.polyfit(ITS, valu, 1)
        csl, cic = np.polyfit(ITS, cyc, 1)
        res[crc] = {"valu_per_cb": dict(zip(map(str, ITS), valu)), "waves_per_cb": waves[0],
                    "lds_per_cb": dict(zip(map(str, ITS), lds)),
                    "valu_per_cb_fixed": ic, "valu_per_cb_iteration": sl,
                    "valu_cycles_per_cb": dict(zip(map(str, ITS), cyc)),
                    "valu_cycles_per_cb_fixed": cic, "valu_cycles_per_cb_iteration": csl,
                    "cycles_per_valu_instruction": dict(zip(map(str, ITS), [c / v for c, v in zip(cyc, valu)])),
                    "valu_busy": dict(zip(map(str, ITS), busy))}
    res["valu_per_cb_fixed"] = res["crc24b"]["valu_per_cb_fixed"]
    res["valu_per_cb_iteration"] = res["crc24b"]["valu_per_cb_iteration"]
    res["valu_cycles_per_cb_fixed"] = res["crc24b"]["valu_cycles_per_cb_fixed"]
    res["valu_cycles_per_cb_iteration"] = res["crc24b"]["valu_cycles_per_cb_iteration"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
