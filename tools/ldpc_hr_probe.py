"""Times the high-rate LDPC decoder kernel (BG1 Z=384 rows of 24Z LLRs, the PUSCH 256QAM R~0.93 shape)
at fixed iteration counts (random LLRs never pass the CRC) to split the per-codeblock fixed cost from the
per-iteration cost, with and without the CRC early-stop check."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import srsran_project_amd as amd  # noqa: E402

Z, N = 384, 4544
dev = torch.device("cuda", 0)
dec = amd.LdpcDecoder("simd", device=0)
rng = np.random.default_rng(0)
x = torch.from_numpy(rng.integers(-10, 11, (N, 24 * Z)).astype(np.int8)).to(dev)
res = {}
for it in (1, 2, 3, 4, 6):
    cfg = amd.LdpcDecoderConfiguration(base_graph=1, lifting_size=Z, nof_crc_bits=24, max_iterations=it)
    for crc in (None, amd.CrcGeneratorPoly.CRC24B):
        dec.decode_batch(x, cfg, crc)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            dec.decode_batch(x, cfg, crc)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res[(it, crc is not None)] = ms
        print("it=%d crc=%-5s %.4f ms  %.1f ns/CB" % (it, crc is not None, ms, ms * 1e6 / N), flush=True)
for c in (False, True):
    its = np.array([1, 2, 3, 4, 6])
    ms = np.array([res[(i, c)] for i in its])
    slope, icpt = np.polyfit(its, ms, 1)
    print("crc=%s: per-iteration %.4f ms, fixed %.4f ms" % (c, slope, icpt))
