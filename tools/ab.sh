#!/bin/bash
# ab.sh <variant>... : bench each exp/<variant>/libsrsran_amd.so (short runs, no CPU baseline).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for r in 1 2; do
for v in "$@"; do
  SRSRAN_AMD_LIB=$PWD/abx/$v/libsrsran_amd.so timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -3 gpurun_out/ab_$v.err; exit $rc; fi
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']; print('$v', round(d['value']), d['unit'], round(r.get('kernel_ms', r.get('step_event_ms', 0)),4), 'ms', round(r['achieved']), 'GB/s', {k: round(r[k]['GB/s']) for k in ('modulate','demodulate') if k in r})"
done
done
