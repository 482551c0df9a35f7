#!/usr/bin/env python3
"""bench.py -- MI355X LDPC decoder throughput (BASELINE.json configs[1]).

Workload (one "step"): decode one batch of BG1, Z=384 full-length codeblocks
(66*384 = 25344 LLRs each, rate 1/3, 46 layers) with exactly 8 layered min-sum
iterations (no early stop), as the reference benchmark
tests/benchmarks/phy/upper/channel_coding/ldpc/ldpc_decoder_benchmark.cpp does
(random +-10 LLR codeblocks, -I 8 -L 384, cb_len = max).  Inputs are resident in
HBM before the timed region.  Multi-GPU: codeblocks are independent, so every
rank decodes its own batch (weak scaling, no data-path collective); the timed
region is bracketed by barriers and the max time over ranks is reported.

cpu_baseline: the REFERENCE decoder itself (oracle/_ref, compiled from
/root/reference sources: AVX512 if the host has it, else AVX2) on a bounded
sample of the same workload, on the host cores of the same box, rank 0 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BG, Z, ITERS = 1, 384, 8
K_BITS = 22 * Z                 # information bits per codeblock (message incl. CRC)
N_LLRS = 66 * Z                 # LLRs per codeblock (full length)
OUT_BYTES = (K_BITS + 7) // 8
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md chip-level parameters (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=4096, help="codeblocks per rank per step")
    p.add_argument("--iters", type=int, default=ITERS)
    p.add_argument("--arith", default="simd", choices=["simd", "generic"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline sample duration")
    p.add_argument("--cpu-threads", type=int, default=16)
    return p.parse_args()


def cpu_baseline(args, llrs_host):
    """Times the reference CPU decoder on a bounded sample of the same workload."""
    try:
        import oracle  # test infrastructure: only used here as the CPU baseline
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "codeblocks/s", "error": "oracle unavailable: %s" % e}
    if oracle.REF is None:
        return {"value": None, "unit": "codeblocks/s", "error": "oracle/_ref/libsrsran_ref.so not built"}
    impl = b"avx512" if oracle.REF.srs_ref_has_impl(b"avx512") else b"avx2"
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    P = oracle.P
    sample = np.ascontiguousarray(llrs_host[:512])
    ns = sample.shape[0]
    # calibrate on a small sample, then decode ~cpu_seconds worth, cycling over the sample
    n0 = min(4 * threads, 256)
    t = oracle.REF.srs_ref_ldpc_decode_many(impl, BG, Z, args.iters, -1, sample.ctypes.data_as(P), N_LLRS, ns, n0,
                                            threads, None, None)
    n = int(max(n0, min(n0 / max(t, 1e-9) * args.cpu_seconds, 1 << 22)))
    t = oracle.REF.srs_ref_ldpc_decode_many(impl, BG, Z, args.iters, -1, sample.ctypes.data_as(P), N_LLRS, ns, n,
                                            threads, None, None)
    # single-thread rate on a shorter sample, for the per-core figure
    n1 = max(8, int(n / threads / 4))
    t1 = oracle.REF.srs_ref_ldpc_decode_many(impl, BG, Z, args.iters, -1, sample.ctypes.data_as(P), N_LLRS, ns, n1,
                                             1, None, None)
    return {
        "value": n / t,
        "unit": "codeblocks/s",
        "cores": threads,
        "kind": "reference",
        "impl": impl.decode(),
        "single_thread_value": n1 / t1,
        "sample": "%d BG1 Z=384 full-length codeblocks (cycling over 512 distinct ones), %d iterations, reference "
                  "ldpc_decoder_%s compiled from /root/reference, %d worker threads with one decoder each, %.1f s; "
                  "single thread: %d codeblocks in %.1f s" % (n, args.iters, impl.decode(), threads, t, n1, t1),
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    import srsran_project_amd as amd

    dec = amd.LdpcDecoder(args.arith, device=local_rank)
    cfg = amd.LdpcDecoderConfiguration(base_graph=BG, lifting_size=Z, nof_crc_bits=24, max_iterations=args.iters)

    # Synthetic input, as ldpc_decoder_benchmark.cpp:172: random (+-10) LLRs.
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    llrs = (torch.randint(0, 2, (args.batch, N_LLRS), device=dev, generator=g, dtype=torch.int8) * 20 - 10)
    out = torch.empty((args.batch, OUT_BYTES), dtype=torch.uint8, device=dev)
    its = torch.empty((args.batch,), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        dec.decode_batch(llrs, cfg, None, out=out, nof_iters=its, stream=stream)
    torch.cuda.synchronize(dev)

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        starts[s].record(stream)
        dec.decode_batch(llrs, cfg, None, out=out, nof_iters=its, stream=stream)
        ends[s].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([starts[s].elapsed_time(ends[s]) for s in range(args.steps)]))

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    total_cbs = args.batch * args.steps * world
    value = total_cbs / elapsed
    bytes_per_cb = N_LLRS + OUT_BYTES + 4  # LLRs in, packed message out, iteration count
    achieved_gbs = bytes_per_cb * args.batch / (kernel_ms * 1e-3) / 1e9

    traffic = None
    tpath = os.path.join(ROOT, "profiles", "r01_ldpc_decode_traffic.json")
    if os.path.exists(tpath):
        # HBM bytes per launch of this kernel on this workload, from rocprofv3
        # FETCH_SIZE / WRITE_SIZE in separate --pmc passes (tools/gpu_check.sh traffic)
        traffic = json.load(open(tpath)).get("hbm_bytes_per_launch")

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args, llrs[:512].cpu().numpy())
        line = {
            "metric": "LDPC decode codeblocks/s (BG1 Z=384, 8 min-sum iterations, full-length rate-1/3 codeblocks)",
            "value": value,
            "unit": "codeblocks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8",
            "data": "synthetic (random +-10 LLRs, as ldpc_decoder_benchmark.cpp)",
            "config": {
                "workload": "configs[1]: LDPC decode BG1 Z=384 8 iterations",
                "base_graph": BG,
                "lifting_size": Z,
                "max_iterations": args.iters,
                "codeblock_llrs": N_LLRS,
                "codeblocks_per_step_per_gpu": args.batch,
                "early_stop": False,
                "arith": args.arith,
                "parallelism": "codeblocks sharded over ranks" if world > 1 else "single GPU",
            },
            "info_throughput_gbps": value * K_BITS / 1e9,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "ldpc_decode_kernel",
                "kernel_ms": kernel_ms,
                "algorithmic_bytes_per_launch": bytes_per_cb * args.batch,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
