#!/bin/bash
# round-4: A/B of two library builds on the sch_slot bench (SRSRAN_AMD_LIB), with kernel statistics of each.
set -o pipefail
O=gpurun_out/r04ab
mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-libsrsran_amd var_nomask}; do
  for r in 1 2; do
    SRSRAN_AMD_LIB=$PWD/srsran_project_amd/lib/$v.so timeout -k 10 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > $O/slot_${v}_$r.log 2>&1 || exit $?
    tail -1 $O/slot_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v run $r', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
  done
  SRSRAN_AMD_LIB=$PWD/srsran_project_amd/lib/$v.so timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p_$v -o p -- python bench.py --workload sch_slot --steps 10 --no-latency --no-cpu-baseline > $O/prof_$v.log 2>&1 &&
    python tools/rocpd_stats.py "$(find /tmp/p_$v -name "*.db" -print -quit)" "sch_slot $v" > $O/stats_$v.md || exit $?
done
