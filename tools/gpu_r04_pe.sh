#!/bin/bash
# round-4: single-launch fused PDSCH encoder -- encoder parity tests, then the benches touching it and a trace.
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -2 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -q -rf --timeout 240 --timeout-method thread"
step tests 500 $PYT tests/test_sch_gpu.py tests/test_sch_slot_gpu.py tests/test_integration_gpu.py tests/test_phy_plugins_gpu.py tests/test_pipeline_gpu.py -k "encode or pdsch or pipeline or small_z or slot"
step bench 200 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step bench_graph 200 python bench.py --graph --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step slot 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
step sp 300 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
step one_cell_graph 200 python bench.py --graph --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
export TMPDIR=/tmp
step prof_pipe 300 rocprofv3 --kernel-trace --stats -d $O/prof_pipe -o pipe -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1
step prof_sp 300 rocprofv3 --kernel-trace --stats -d $O/prof_sp -o sp -- python bench.py --workload slot_pipeline --steps 5 --no-latency --no-cpu-baseline
exit 0
