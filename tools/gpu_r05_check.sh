#!/bin/bash
# One gpurun session of the r05 kernel work: the given GPU tests, the headline bench line, its rocprofv3 kernel
# trace, and the one-cell HIP-graph latency line.  Every GPU step has its own time limit; a step that faults,
# aborts or times out ends the script.
#   tools/gpu_r05_check.sh <outdir> [pytest selection...]
out=${1:-gpurun_out/r05c}
shift
mkdir -p "$out"
export TMPDIR=/tmp
ok() { # continue after success or ordinary test failures only
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "step ended with $rc: stopping" | tee -a "$out/steps.log"
    exit "$rc"
  fi
}
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > "$out/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc" >> "$out/steps.log"; ok $rc
  tail -3 "$out/pytest.log"
fi
BENCH=(python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1)
timeout -k 10 300 "${BENCH[@]}" > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc" >> "$out/steps.log"; ok $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- "${BENCH[@]}" \
  > "$out/trace.log" 2>&1
rc=$?; echo "trace rc=$rc" >> "$out/steps.log"; ok $rc
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --graph --slots-pipeline 1 \
  > "$out/one_cell_graph.json" 2> "$out/one_cell_graph.err"
rc=$?; echo "one-cell rc=$rc" >> "$out/steps.log"; ok $rc

# the graph-capture probe: the PDSCH chain forked onto its own stream inside the capture (SRSRAN_AMD_GRAPH_FORK=1)
if [ -n "$GRAPH_FORK_PROBE" ]; then
  SRSRAN_AMD_GRAPH_FORK=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph \
    --slots-pipeline 1 > "$out/graph_fork.json" 2> "$out/graph_fork.err"
  echo "graph fork probe rc=$?" >> "$out/steps.log"
fi
echo done >> "$out/steps.log"
