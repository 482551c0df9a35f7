#!/bin/bash
# round-4: packed decoder with repeating lanes masked out of the layers -- decoder / slot parity, then slot benches.
set -o pipefail
O=gpurun_out/r04pk2
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -2 "$O/$name.log" | cut -c1-220
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -q -rf --timeout 300 --timeout-method thread"
step tests 700 $PYT tests/test_ldpc_decoder_gpu.py tests/test_golden.py tests/test_sch_slot_gpu.py tests/test_sch_gpu.py
step slot 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
step sp 200 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
exit 0
