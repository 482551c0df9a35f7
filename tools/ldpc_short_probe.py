"""Times the LDPC decoder on short (high-rate) codeblocks to split the per-codeblock
fixed cost (input scan, soft-bit load, hard decision) from the per-iteration cost."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import srsran_project_amd as amd  # noqa: E402

Z, BG, N = 384, 1, 4096
dev = torch.device("cuda", 0)
dec = amd.LdpcDecoder("simd", device=0)
rng = np.random.default_rng(0)
full = rng.integers(-10, 11, (N, 66 * Z)).astype(np.int8)
short = full.copy()
short[:, 9000:] = 0
for name, x in (("full", full), ("short", short)):
    t = torch.from_numpy(x).to(dev)
    for it in (1, 2, 4, 8):
        cfg = amd.LdpcDecoderConfiguration(base_graph=BG, lifting_size=Z, nof_crc_bits=24, max_iterations=it)
        for crc in (None, amd.CrcGeneratorPoly.CRC24B):
            dec.decode_batch(t, cfg, crc)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                dec.decode_batch(t, cfg, crc)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 5
            print("%-5s it=%d crc=%-5s  %.3f ms  %.0f ns/CB" % (name, it, crc is not None, ms, ms * 1e6 / N), flush=True)
