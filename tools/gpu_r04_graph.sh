#!/bin/bash
# round-4: HIP-graph replay of the pipeline step (64 cells and one cell) after the two-stream step change.
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step graph 200 python -X faulthandler bench.py --graph --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step one_cell_graph 200 python -X faulthandler bench.py --graph --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step sp 200 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
step slot 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
exit 0
