#!/bin/bash
# probe.sh <variant>...: tools/ldpc_hr_probe.py with each abx/<variant>/libsrsran_amd.so ("-" = in-tree build)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for v in "$@"; do
  lib=$PWD/abx/$v/libsrsran_amd.so; [ "$v" = "-" ] && lib=$PWD/srsran_project_amd/lib/libsrsran_amd.so
  echo "== $v"
  SRSRAN_AMD_LIB=$lib timeout -k 10 120 python tools/ldpc_hr_probe.py > gpurun_out/probe_$v.log 2>&1 || { tail -5 gpurun_out/probe_$v.log; exit 1; }
  tail -2 gpurun_out/probe_$v.log
done
