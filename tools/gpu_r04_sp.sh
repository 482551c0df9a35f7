#!/bin/bash
# round-4: slot-form regressions -- slot_pipeline and sch_slot with the packed runtime-Z decoder and the fused PDSCH
# encoder each switched off (SRSRAN_AMD_LDPC_PK=0, SRSRAN_AMD_PDSCH_FUSED=0), then a kernel trace of the default.
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -1 "$O/$name.log" | cut -c1-260
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
export TMPDIR=/tmp
for cfg in "def" "pk0:SRSRAN_AMD_LDPC_PK=0" "fu0:SRSRAN_AMD_PDSCH_FUSED=0" "both0:SRSRAN_AMD_LDPC_PK=0 SRSRAN_AMD_PDSCH_FUSED=0"; do
  n=${cfg%%:*}; e=""; [ "$n" != "$cfg" ] && e=${cfg#*:}
  step sp_$n 200 env $e python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
  step slot_$n 200 env $e python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
done
step prof_sp 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_sp -o sp -- python bench.py --workload slot_pipeline --steps 5 --no-latency --no-cpu-baseline &&
  python tools/rocpd_stats.py "$(find /tmp/prof_sp -name "*.db" -print -quit)" "r04 slot_pipeline" > $O/prof_sp_stats.md
exit 0
