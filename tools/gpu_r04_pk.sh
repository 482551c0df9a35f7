#!/bin/bash
# round-4 GPU checks and benches: the previously failing tests, then bench.py (headline + pinned sibling), sch_slot /
# slot_pipeline with the packed decoder on and off, the PDSCH chain fused and unfused, and kernel traces.
# Stops at the first GPU step that faults, hangs or aborts (exit status other than 0 / 1).
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -2 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -q -rf --timeout 240 --timeout-method thread"
step tests 400 $PYT tests/test_sch_slot_gpu.py tests/test_integration_gpu.py tests/test_phy_plugins_gpu.py -k "small_z or hw_pdsch_enc or pusch_plugin or ofdm_factory"
step bench 300 python bench.py --no-cpu-baseline
step bench_unfused 200 env SRSRAN_AMD_PDSCH_FUSED=0 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step slot_pk 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
step slot_nopk 200 env SRSRAN_AMD_LDPC_PK=0 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
step sp_pk 300 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
step sp_nopk 300 env SRSRAN_AMD_LDPC_PK=0 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
step one_cell 200 python bench.py --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step one_cell_graph 200 python bench.py --graph --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step bench_graph 200 python bench.py --graph --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step ldpc_cfg1 200 python bench.py --workload ldpc --no-cpu-baseline
export TMPDIR=/tmp
step prof_slot 300 rocprofv3 --kernel-trace --stats -d $O/prof_slot -o slot -- python bench.py --workload sch_slot --steps 10 --no-latency --no-cpu-baseline
step prof_pipe 300 rocprofv3 --kernel-trace --stats -d $O/prof_pipe -o pipe -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1
exit 0
