#!/usr/bin/env python3
"""bench.py -- MI355X PHY hot-path throughput (BASELINE.json configs).

Default workload (`--workload pipeline`, the BASELINE.json headline metric
"PDSCH+PUSCH codeblocks/s @ 100 MHz 273-PRB 4x4 MIMO", configs[3]): one step
runs every cell-slot of a batch through the full PDSCH transmit and PUSCH
receive chains -- see bench_pipeline.py.

`--workload ldpc` (configs[1], the headline of the decoder alone): one "step"
decodes one batch of BG1, Z=384 full-length codeblocks (66*384 = 25344 LLRs
each, rate 1/3, 46 layers) with exactly 8 layered min-sum iterations (no early
stop), as the reference benchmark
tests/benchmarks/phy/upper/channel_coding/ldpc/ldpc_decoder_benchmark.cpp does
(random +-10 LLR codeblocks, -I 8 -L 384, cb_len = max).

`--workload ofdm` (configs[2]): one step OFDM-modulates and then demodulates a
batch of slots of the 100 MHz numerology-1 carrier (273 PRB, 4096-point DFT,
normal CP): 4 antenna ports x `--slots` slots, cbf16 resource grids to complex
float baseband and back (ofdm_slot_modulator / ofdm_slot_demodulator).

`--workload sch_slot` (heterogeneous slots, not a BASELINE.json config): one step PDSCH-encodes and
PUSCH-decodes the transport blocks of `--slots-pipeline` cells x `--ues-per-cell` UEs with different PRB
shares, MCS and layer counts through the slot-level entry points -- see bench_slot.py.
`--workload pucch`: every PUCCH (Formats 0-4) of a slot of --slots-pipeline cells through the slot forms of
include/srsran_amd/pucch.h, UCI messages/s, with the reference pucch_processor_impl as the CPU baseline
(bench_pucch.py).
`--workload slot_pipeline`: the full PDSCH + PUSCH chains of such multi-UE cells (slot encoder, slot modulator
+ DM-RS, OFDM; OFDM, slot PUSCH processor) -- bench_slot.SlotPipeline.

Inputs are resident in HBM before the timed region.  Multi-GPU: `--gpus N`
starts N ranks itself (one process per GPU, before any GPU call), or runs under
torch.distributed.run; cells / codeblocks / slots are independent, so every
rank processes its own batch (weak scaling, no data-path collective; the
pipeline's optional `--ingest` adds the RCCL scatter / gather of slot inputs and
results, timed separately); the timed region is bracketed by barriers and the
max time over ranks is reported.

cpu_baseline: the REFERENCE implementation itself (oracle/_ref, compiled from
/root/reference sources: the AVX512 decoder if the host has it, else AVX2; the
generic DFT for OFDM since FFTW is not in the image) on a bounded sample of the
same workload, on the host cores of the same box, rank 0 only.
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md chip-level parameters (spec)

# LDPC headline workload
BG, Z, ITERS = 1, 384, 8
K_BITS = 22 * Z                 # information bits per codeblock (message incl. CRC)
N_LLRS = 66 * Z                 # LLRs per codeblock (full length)
OUT_BYTES = (K_BITS + 7) // 8

# OFDM workload: 100 MHz, 30 kHz SCS
OFDM_MU, OFDM_BW, OFDM_N, OFDM_PORTS = 1, 273, 4096, 4


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="pipeline", choices=["pipeline", "ldpc", "ofdm", "sch_slot",
                                                                       "slot_pipeline", "pucch"])
    p.add_argument("--batch", type=int, default=4096, help="ldpc: codeblocks per rank per step")
    p.add_argument("--slots", type=int, default=160, help="ofdm: slots per rank per step (x 4 ports)")
    p.add_argument("--slots-pipeline", type=int, default=64,
                   help="pipeline: cells (one slot each) per rank per step")
    p.add_argument("--iters", type=int, default=ITERS)
    p.add_argument("--arith", default="simd", choices=["simd", "generic"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline sample duration")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--snr-db", type=float, default=35.0, help="pipeline: PUSCH SNR of the headline line")
    p.add_argument("--low-snr-db", type=float, default=None,
                   help="pipeline: also report a line at this SNR, near the 256QAM R=0.93 decoding threshold where "
                        "the decoder runs ~4 iterations per codeblock (default per PUSCH layers, from "
                        "tools/snr_sweep.py: 31.0 dB for 4 layers, 23.8 dB for 2; < 0 disables)")
    p.add_argument("--mimo", default="4x4", choices=["4x4", "2x2"],
                   help="pipeline: 4x4 (headline: PDSCH 4 layers x 4 ports, PUSCH --ul-layers x 4 rx) or 2x2 "
                        "(configs[3]: PDSCH 2 layers x 2 ports, PUSCH 2 layers x 2 rx, reference-pinned ZF)")
    p.add_argument("--ul-layers", type=int, default=4, choices=[1, 2, 3, 4],
                   help="pipeline: PUSCH layers (4: MMSE 4x4, parity unpinned; 2: the reference-pinned ZF 2x4)")
    p.add_argument("--chest-td", default="average", choices=["average", "interpolate"],
                   help="pipeline: PUSCH DM-RS estimator time-domain strategy (average: the reference app's default, "
                        "du_low_config.h:68)")
    p.add_argument("--ingest", action="store_true",
                   help="pipeline, N > 1: rank 0 holds all cells' slot inputs; RCCL scatter / gather every step")
    p.add_argument("--no-probe", action="store_true",
                   help="pipeline: no live kernel probes in the timed steps (roofline from the alone decoder)")
    p.add_argument("--alone-probe", action="store_true",
                   help="pipeline: also time the LDPC decoder alone on pre-dematched rows (an extra launch form)")
    p.add_argument("--no-pinned", action="store_true",
                   help="pipeline: skip the reference-pinned sibling line (PUSCH 2 layers x 4 rx, ZF)")
    p.add_argument("--no-latency", action="store_true",
                   help="pipeline: skip the 1 / 8 cell latency figures; sch_slot: skip the per-UE launch timing")
    p.add_argument("--graph", action="store_true",
                   help="pipeline: replay each step as a HIP graph captured once (both streams, every launch)")
    p.add_argument("--ues-per-cell", type=int, default=8, help="sch_slot: UEs sharing each cell's 273 PRBs")
    p.add_argument("--mixed", action="store_true",
                   help="slot_pipeline: ~20%% UCI-on-PUSCH, ~10%% HARQ retransmission, ~3%% DFT-s-OFDM PDUs")
    return p.parse_args()


def load_traffic(name, kernel=None):
    """HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (tools/gpu_check.sh traffic, tools/pmc_summary.py), committed under profiles/;
    `kernel` picks one kernel of a multi-kernel summary."""
    tpath = os.path.join(ROOT, "profiles", name)
    if os.path.exists(tpath):
        d = json.load(open(tpath))
        if kernel is not None and kernel in d.get("kernels", {}):
            return d["kernels"][kernel].get("hbm_bytes_per_launch")
        return d.get("hbm_bytes_per_launch")
    return None


def timed(args, dist, world, dev, stream, step, probes=None):
    """Warmup, then K steps bracketed by barrier + synchronize; per-step HIP
    events on the launch stream.  Returns (elapsed_s max over ranks, mean event ms).
    On a CPU device (the gloo tests of the multi-rank path) the events are skipped.
    probes: optional dict {probe id: None} of live kernel probes (srsran_project_amd.profiling) armed over exactly
    the K timed steps; filled with (launches, mean ms, min ms, max ms) of each kernel family's launches in them."""
    import torch

    gpu = dev.type == "cuda"
    if probes and gpu:
        from srsran_project_amd import profiling
    sync = (lambda: torch.cuda.synchronize(dev)) if gpu else (lambda: None)
    for _ in range(args.warmup):
        step()
    sync()
    if gpu:
        starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
        ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    # Python's cyclic garbage collector off while timing, as timeit does (collected before the barrier, so the ranks
    # still start their clocks together): no collection pause inside the timed steps
    gc.collect()
    gc_was_enabled = gc.isenabled()
    gc.disable()
    try:
        if world > 1:
            dist.barrier()
        sync()
        if probes and gpu:
            for p in [q for q in probes if isinstance(q, int)]:
                profiling.arm(p, 64 * args.steps)
        t0 = time.perf_counter()
        for s in range(args.steps):
            if gpu:
                starts[s].record(stream)
            step()
            if gpu:
                ends[s].record(stream)
        sync()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    finally:
        if gc_was_enabled:
            gc.enable()
    if probes and gpu:
        for p in [q for q in probes if isinstance(q, int)]:
            probes[p] = profiling.read(p)
    if gpu:
        event_ms = float(np.mean([starts[s].elapsed_time(ends[s]) for s in range(args.steps)]))
    else:
        event_ms = elapsed * 1e3 / max(1, args.steps)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), event_ms


# ------------------------------------------------------------------ LDPC ----

def ldpc_cpu_baseline(args, llrs_host):
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


def run_ldpc(args, dist, world, rank, dev):
    import torch

    import srsran_project_amd as amd

    dec = amd.LdpcDecoder(args.arith, device=dev.index)
    cfg = amd.LdpcDecoderConfiguration(base_graph=BG, lifting_size=Z, nof_crc_bits=24, max_iterations=args.iters)
    # Synthetic input, as ldpc_decoder_benchmark.cpp:172: random (+-10) LLRs.
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    llrs = (torch.randint(0, 2, (args.batch, N_LLRS), device=dev, generator=g, dtype=torch.int8) * 20 - 10)
    out = torch.empty((args.batch, OUT_BYTES), dtype=torch.uint8, device=dev)
    its = torch.empty((args.batch,), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        dec.decode_batch(llrs, cfg, None, out=out, nof_iters=its, stream=stream)

    elapsed, kernel_ms = timed(args, dist, world, dev, stream, step)
    total_cbs = args.batch * args.steps * world
    value = total_cbs / elapsed
    bytes_per_cb = N_LLRS + OUT_BYTES + 4  # LLRs in, packed message out, iteration count
    achieved_gbs = bytes_per_cb * args.batch / (kernel_ms * 1e-3) / 1e9
    if rank != 0:
        return None
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = ldpc_cpu_baseline(args, llrs[:512].cpu().numpy())
    full_pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", "r03c_ldpc_full_pmc.json")
    if os.path.exists(pmc_path):
        row = json.load(open(pmc_path)).get("ldpc_decode_hr_kernel<0, 46, 1>", {})
        full_pmc = {"hbm_bytes": row.get("hbm_mb", 0.0) * 1e6 or None, "valu_busy": row.get("valu_busy")}
    return {
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
            "traffic": full_pmc.get("hbm_bytes"),
            "kernel": "ldpc_decode_hr_kernel<ARITH, 46, 1> (full-length BG1 Z=384 kernel)",
            "kernel_ms": kernel_ms,
            "algorithmic_bytes_per_launch": bytes_per_cb * args.batch,
            "limiter": "valu",
            "valu_busy_pmc": full_pmc.get("valu_busy"),
            "note": "HBM-far by design (8 layered iterations over LDS-resident soft bits); the limiter is VALU issue: "
                    "valu_busy_pmc = SQ_ACTIVE_INST_VALU x 4 / (1,024 SIMDs x kernel cycles) of this kernel on this "
                    "workload, traffic = PMC FETCH + WRITE bytes per launch (profiles/r03c_ldpc_full_pmc.json)",
        },
        "cpu_baseline": cpu,
    }


# ------------------------------------------------------------------ OFDM ----

def ofdm_cpu_baseline(args, grids_host):
    try:
        import oracle
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "symbols/s", "error": "oracle unavailable: %s" % e}
    if oracle.REF is None:
        return {"value": None, "unit": "symbols/s", "error": "oracle/_ref/libsrsran_ref.so not built"}
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    sample = np.ascontiguousarray(grids_host)
    ns = sample.shape[0]
    n0 = 2 * threads
    t = oracle.REF.srs_ref_ofdm_roundtrip_many(OFDM_MU, OFDM_BW, OFDM_N, sample.ctypes.data_as(oracle.P), ns, n0,
                                               threads)
    n = int(max(n0, min(n0 / max(t, 1e-9) * args.cpu_seconds, 1 << 20)))
    t = oracle.REF.srs_ref_ofdm_roundtrip_many(OFDM_MU, OFDM_BW, OFDM_N, sample.ctypes.data_as(oracle.P), ns, n,
                                               threads)
    return {
        "value": n * 14 / t,
        "unit": "symbols/s",
        "cores": threads,
        "kind": "reference",
        "impl": "ofdm_slot_modulator_impl + ofdm_slot_demodulator_impl, dft_processor_generic_impl",
        "sample": "%d slot-ports (14 symbols each) modulated then demodulated, 100 MHz mu=1 273 PRB 4096-point, "
                  "cycling over %d grids, %d worker threads with one modulator + demodulator each, %.1f s "
                  "(reference generic DFT: FFTW is not in the image)" % (n, ns, threads, t),
    }


def run_ofdm(args, dist, world, rank, dev):
    import torch

    import srsran_project_amd as amd

    rg = OFDM_BW * 12
    mod = amd.OfdmSlotModulator(amd.OfdmModulatorConfiguration(OFDM_MU, OFDM_BW, OFDM_N, 0, 1.0, 3.5e9),
                                device=dev.index)
    dem = amd.OfdmSlotDemodulator(amd.OfdmDemodulatorConfiguration(OFDM_MU, OFDM_BW, OFDM_N, 0, 1.0, 3.5e9, 0),
                                  device=dev.index)
    g = torch.Generator(device=dev)
    g.manual_seed(99 + rank)
    # QPSK-like cbf16 grid: +-0.707 in bf16 (0x3F35 / 0xBF35)
    bits = torch.randint(0, 2, (args.slots, OFDM_PORTS, 14, 2 * rg), device=dev, generator=g, dtype=torch.int16)
    grid = torch.where(bits == 0, torch.tensor(0x3F35, dtype=torch.int16, device=dev),
                       torch.tensor(0xBF35 - 0x10000, dtype=torch.int16, device=dev)).contiguous()
    stride = mod.max_slot_size()
    samples = torch.empty((args.slots, OFDM_PORTS, stride), dtype=torch.complex64, device=dev)
    back = torch.empty_like(grid)
    stream = torch.cuda.current_stream(dev)

    def step():
        mod.modulate_batch(grid, 0, out=samples, stream=stream)
        dem.demodulate_batch(samples, 0, grid=back, stream=stream)

    # per-kernel timing on the launch stream: modulator alone, demodulator alone
    elapsed, step_ms = timed(args, dist, world, dev, stream, step)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record(stream)
    for _ in range(args.steps):
        mod.modulate_batch(grid, 0, out=samples, stream=stream)
    ev[1].record(stream)
    for _ in range(args.steps):
        dem.demodulate_batch(samples, 0, grid=back, stream=stream)
    ev[2].record(stream)
    torch.cuda.synchronize(dev)
    mod_ms = ev[0].elapsed_time(ev[1]) / args.steps
    dem_ms = ev[1].elapsed_time(ev[2]) / args.steps

    nsym = args.slots * OFDM_PORTS * 14
    # algorithmic HBM bytes: grid (cbf16, 4 B/RE) + samples (cf32, 8 B) once each way
    samp = sum(mod.get_slot_size(s % (1 << OFDM_MU)) for s in range(args.slots))
    mod_bytes = OFDM_PORTS * (args.slots * 14 * rg * 4 + samp * 8)
    dem_bytes = nsym * (OFDM_N * 8 + rg * 4)
    mod_gbs = mod_bytes / (mod_ms * 1e-3) / 1e9
    dem_gbs = dem_bytes / (dem_ms * 1e-3) / 1e9
    value = nsym * args.steps * world / elapsed
    if rank != 0:
        return None
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = ofdm_cpu_baseline(args, grid[:8, 0].cpu().numpy().view(np.uint16))
    return {
        "metric": "OFDM modulate+demodulate symbols/s (100 MHz numerology-1, 273 PRB, 4096-point DFT)",
        "value": value,
        "unit": "symbols/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (random QPSK cbf16 resource grids)",
        "config": {
            "workload": "configs[2]: OFDM modulate+demodulate, 100 MHz numerology-1 (4096-pt FFT), batched slots",
            "numerology": OFDM_MU,
            "bw_rb": OFDM_BW,
            "dft_size": OFDM_N,
            "ports": OFDM_PORTS,
            "slots_per_step_per_gpu": args.slots,
            "symbols_per_step_per_gpu": nsym,
            "parallelism": "slots sharded over ranks" if world > 1 else "single GPU",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": (mod_bytes + dem_bytes) / ((mod_ms + dem_ms) * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (mod_bytes + dem_bytes) / ((mod_ms + dem_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "traffic": load_traffic("r01_ofdm_traffic.json"),
            "kernel": "ofdm_modulate_kernel<4096> + ofdm_demodulate_kernel<4096>",
            "modulate": {"ms": mod_ms, "bytes": mod_bytes, "GB/s": mod_gbs},
            "demodulate": {"ms": dem_ms, "bytes": dem_bytes, "GB/s": dem_gbs},
            "step_event_ms": step_ms,
        },
        "cpu_baseline": cpu,
    }


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N ranks of this script (one process per GPU) before anything touches
    the GPU, each with RANK / LOCAL_RANK / WORLD_SIZE and a 127.0.0.1 rendezvous, forward their output and exit
    with the worst return code. Rank 0 prints the JSON line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(sys.argv[0])] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("warning: --gpus %d but WORLD_SIZE %d; reporting the launched world" % (args.gpus, world),
              file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    if args.workload == "pipeline":
        from bench_pipeline import run_pipeline

        line = run_pipeline(args, dist, world, rank, dev, timed, HBM_PEAK_GBS,
                            load_traffic("r05_traffic.json", "ldpc_decode_hr_kernel"))
    elif args.workload == "sch_slot":
        from bench_slot import run_sch_slot

        line = run_sch_slot(args, dist, world, rank, dev, timed)
    elif args.workload == "slot_pipeline":
        from bench_slot import run_slot_pipeline

        line = run_slot_pipeline(args, dist, world, rank, dev, timed)
    elif args.workload == "pucch":
        from bench_pucch import run_pucch

        line = run_pucch(args, dist, world, rank, dev, timed)
    else:
        run = run_ldpc if args.workload == "ldpc" else run_ofdm
        line = run(args, dist, world, rank, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
