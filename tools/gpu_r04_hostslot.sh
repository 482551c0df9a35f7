#!/bin/bash
# round-4: host time of the sch_slot calls in three processes (tools/sch_slot_host_probe.py).
set -o pipefail
for r in 1 2 3; do
  PYTHONPATH=. timeout -k 10 120 python tools/sch_slot_host_probe.py 2>&1 | grep -v amdgpu.ids || exit $?
done
