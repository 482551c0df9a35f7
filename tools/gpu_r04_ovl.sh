#!/bin/bash
# round-4: the benches with the two chains on two consecutive pool streams (bench_pipeline.chain_streams).
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
for r in 1 2; do
  step bench$r 200 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
  step sp$r 200 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
  step slot$r 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
done
step graph 200 python bench.py --graph --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step one_cell_graph 200 python bench.py --graph --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
exit 0
