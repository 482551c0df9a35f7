#!/bin/bash
# Round-6 headline evidence in one GPU session: the default bench line (CPU-baseline leg included), its rocprofv3
# kernel-trace summary, the four PMC passes of the same command (tools/pmc_passes.sh) and smoke().  Every GPU step
# runs under its own time limit and a failing step ends the script.
#   tools/gpu_r06_final.sh <outdir>
set -uo pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 420 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; exit 3; }
QUICK=(python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- "${QUICK[@]}" \
  > "$out/trace.log" 2>&1 || { echo "trace failed"; exit 3; }
cp "$out/trace/run_kernel_stats.csv" "$out/kernel_stats.csv" 2>/dev/null || true
timeout -k 10 700 tools/pmc_passes.sh "$out/pmc" "${QUICK[@]}" || { echo "pmc failed"; exit 3; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.log" 2>&1 \
  || { echo "smoke failed"; exit 3; }
echo "final ok"
