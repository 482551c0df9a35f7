#!/bin/bash
# Mixed-Z slot decoding: decoder + slot parity tests, sch_slot bench, headline bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run t_slot 700 python -u -m pytest tests/test_sch_slot_gpu.py tests/test_ldpc_decoder_gpu.py tests/test_golden.py tests/test_sch_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu
run b_slot 300 python bench.py --workload sch_slot --steps 20 --warmup 3
run b_head 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
