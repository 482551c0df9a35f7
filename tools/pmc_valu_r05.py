#!/usr/bin/env python3
"""r05 VALU model of the in-step ldpc_decode_hr_kernel from tools/pmc_table.py's output over the bench command
(rocprofv3 --pmc passes of tools/gpu_r05_evidence.sh): SQ_INSTS_VALU per codeblock at the step's mean iterations, the
measured SQ_ACTIVE_INST_VALU busy fraction, and the cycles per VALU instruction they imply.

  pmc_valu_r05.py <pmc_table.json> <bench.json> <out.json>
"""
import json
import sys


def main(pmc, bench, out):
    rows = json.load(open(pmc))
    b = json.load(open(bench))
    k = next(n for n in rows if n.startswith("ldpc_decode_hr_kernel<0, 4, 1>"))
    r = rows[k]
    cbs = b["config"]["pusch"]["codeblocks"] * b["config"]["cells_per_step_per_gpu"]
    its = b["pusch_ldpc_iterations_mean"]
    insts_per_cb = r["valu_per_wave"] * r["waves"] / cbs
    nominal = r["valu_per_wave"] * r["waves"] * 2 / (1024 * r["kernel_cycles"])
    m = {
        "kernel": k, "launches": r["launches"], "codeblocks_per_launch": cbs, "iterations_mean": its,
        "waves_per_launch": r["waves"], "valu_insts_per_wave": r["valu_per_wave"], "valu_insts_per_cb": insts_per_cb,
        "valu_insts_per_cb_iteration_upper": insts_per_cb / its, "kernel_cycles": r["kernel_cycles"],
        "cycles_per_valu_insn": 2.0, "valu_issue_frac_nominal": nominal, "valu_busy": r["valu_busy"],
        "implied_cycles_per_valu_insn": 2.0 * r["valu_busy"] / nominal if nominal else None,
        "wait_share": r["wait_share"], "issue_stall_share": r["issue_stall_share"],
        "lds_array_busy": r["lds_array_busy"], "scale_by_iterations": False,
        "note": "valu_issue_frac_nominal = SQ_INSTS_VALU x 2 cycles (MI355X_MICROARCH.md: a wave64 VALU instruction "
                "issues over 2 cycles) / (1,024 SIMDs x kernel cycles, GRBM_GUI_ACTIVE / 8); valu_busy = "
                "SQ_ACTIVE_INST_VALU x 4 / the same.  Their ratio is the mean issue cost per instruction: the kernel's "
                "VOP3P packed-int16 instructions take ~4 cycles (dependent v_pk pairs, r03 microbenchmark 4.3).",
    }
    json.dump(m, open(out, "w"), indent=1)
    print(json.dumps(m, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
