#!/bin/bash
# r05 end-of-round records in one gpurun session: the whole GPU suite, smoke(), the default bench line (with the CPU
# baseline leg), its rocprofv3 kernel trace, the one-cell graph line, configs[1] / configs[2] and the slot benches.
# Every GPU step has its own time limit; a step that faults, aborts or times out ends the script.
#   tools/gpu_r05_final.sh <outdir>
out=${1:-gpurun_out/r05f}
mkdir -p "$out"
export TMPDIR=/tmp
ok() { # continue after success or ordinary test failures only
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "step ended with $rc: stopping" | tee -a "$out/steps.log"
    exit "$rc"
  fi
}
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > "$out/gpu_suite.log" 2>&1
rc=$?; echo "suite rc=$rc" >> "$out/steps.log"; ok $rc
tail -2 "$out/gpu_suite.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc" >> "$out/steps.log"; ok $rc
timeout -k 10 600 python3 bench.py > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc" >> "$out/steps.log"; ok $rc
BENCH=(python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- "${BENCH[@]}" \
  > "$out/trace.log" 2>&1
rc=$?; echo "trace rc=$rc" >> "$out/steps.log"; ok $rc
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --graph --slots-pipeline 1 \
  > "$out/one_cell_graph.json" 2> "$out/one_cell_graph.err"
rc=$?; echo "one-cell rc=$rc" >> "$out/steps.log"; ok $rc
for w in ldpc ofdm sch_slot slot_pipeline; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > "$out/$w.json" 2> "$out/$w.err"
  rc=$?; echo "$w rc=$rc" >> "$out/steps.log"; ok $rc
done
timeout -k 10 300 python3 bench.py --workload slot_pipeline --mixed --no-cpu-baseline > "$out/slot_pipeline_mixed.json" \
  2> "$out/slot_pipeline_mixed.err"
rc=$?; echo "mixed rc=$rc" >> "$out/steps.log"; ok $rc
echo done >> "$out/steps.log"
