#!/bin/bash
# The four rocprofv3 --pmc passes read by tools/pmc_table.py, one counter set per run (counters only, no
# tracing domains), each under its own time limit; CSV output under <outdir>/{a,b,fetch,write}.
#   tools/pmc_passes.sh <outdir> <program> [args...]     (run from the repository root)
set -euo pipefail
out=$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
pass() {
  local name=$1
  shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- "${CMD[@]}" \
    > "$out/$name.log" 2>&1
}
CMD=("$@")
pass a SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES
pass b SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
