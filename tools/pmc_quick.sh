#!/bin/bash
# Kernel trace and one SQ counter pass of the headline bench (short), each step under its own limit:
#   tools/pmc_quick.sh <outdir>
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
BENCH=(python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- "${BENCH[@]}" \
  > "$out/trace.log" 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d "$out/a" -o run -- "${BENCH[@]}" \
  > "$out/a.log" 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$out/b" -o run -- "${BENCH[@]}" > "$out/b.log" 2>&1 || exit 3
python3 tools/pmc_table.py "$out/table.json" "$out/a" "$out/b" "$out/a" "$out/a" > "$out/table.txt" 2>&1
