#!/bin/bash
# round-4 end: the default bench line (with the CPU-baseline leg), its kernel-trace summary, the configs[1] / [2]
# workloads, the graph and one-cell forms; logs and summaries under gpurun_out/r04z.
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step bench 400 python bench.py
step prof 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_b -o b -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1
python tools/rocpd_stats.py "$(find /tmp/prof_b -name "*.db" -print -quit)" "r04 headline bench (rocprofv3 --kernel-trace --stats -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1)" > $O/bench_kernel_stats.md
find /tmp/prof_b -name "*stats*.csv" -exec cp {} $O/ \;
step ldpc 300 python bench.py --workload ldpc --no-cpu-baseline
step ofdm 300 python bench.py --workload ofdm --no-cpu-baseline
step sp 200 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
step slot 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
step graph 200 python bench.py --graph --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step one_cell_graph 200 python bench.py --graph --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
exit 0
