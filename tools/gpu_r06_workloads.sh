#!/bin/bash
# Round-6 secondary bench lines in one GPU session (each step under its own time limit; a failure ends the script):
# configs[1] LDPC, configs[2] OFDM, the one-cell graph, PUCCH slot forms, the slot pipeline all-data and mixed.
#   tools/gpu_r06_workloads.sh <outdir>
set -uo pipefail
out=$1
mkdir -p "$out"
run() {
  local name=$1
  shift
  timeout -k 10 300 python3 bench.py "$@" > "$out/$name.json" 2> "$out/$name.err" || { echo "$name failed"; exit 3; }
  echo "$name $(grep -o '"value": [0-9.e+]*' "$out/$name.json" | head -1)"
}
run ldpc --workload ldpc
run ofdm --workload ofdm
run one_cell_graph --graph --slots-pipeline 1 --no-cpu-baseline
run pucch --workload pucch
run slot_pipeline --workload slot_pipeline --no-cpu-baseline
run slot_pipeline_mixed --workload slot_pipeline --mixed --no-cpu-baseline
echo "workloads ok"
