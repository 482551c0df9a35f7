"""Multi-GPU cell fan-out: one process per GPU, cells (sectors) sharded over the
ranks of one node, slot batches moved over RCCL (xGMI) only at the edges.

The reference runs every cell of a gNB in one process on CPU threads
(lib/phy/upper/upper_phy_factories.cpp builds one upper PHY per cell sector,
each with its own PDSCH / PUSCH processor pools). Cells share no data on the
PHY hot path, so here each rank owns a contiguous share of the cells and runs
the whole PDSCH + PUSCH chain of its cells on its own GPU with no data-path
collective (weak scaling). The optional slot ingest models a single fronthaul
entry point: rank 0 holds the slot inputs of every cell (uplink baseband and
downlink transport blocks), `scatter` fans each rank's share out, and `gather`
brings the decoded uplink transport blocks and CRC flags back to rank 0 --
one scatter / gather per slot batch, sized for the per-link xGMI bandwidth
(a whole batch per message, never per cell).

Works on any torch.distributed backend: "nccl" (RCCL) with GPU tensors in the
bench, "gloo" with CPU tensors in the multi-process tests.
"""


def cell_range(nof_cells, world, rank):
    """Contiguous, balanced share of nof_cells for `rank`: (first cell, number of cells)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("invalid rank %d of %d" % (rank, world))
    base, extra = divmod(nof_cells, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def padded_share(nof_cells, world):
    """Cells per rank in the scatter / gather messages (collectives need equal shapes): ceil(n / world)."""
    return -(-nof_cells // world)


class SlotFanout:
    """Scatter of per-cell slot inputs from rank 0 and gather of per-cell results to rank 0.

    Tensors are [cell][...] with the same trailing shape on every rank; rank 0 passes the full
    [nof_cells][...] tensor, every rank receives / sends its [cell_range count][...] share.
    """

    def __init__(self, dist, world, rank, nof_cells):
        self.dist, self.world, self.rank, self.nof_cells = dist, world, rank, nof_cells
        self.first, self.count = cell_range(nof_cells, world, rank)
        self.share = padded_share(nof_cells, world)

    def _chunks(self, full):
        import torch

        out = []
        for r in range(self.world):
            a, n = cell_range(self.nof_cells, self.world, r)
            c = full.new_zeros((self.share,) + tuple(full.shape[1:]))
            c[:n] = full[a:a + n]
            out.append(c)
        return out

    def scatter(self, full, out):
        """full: [nof_cells][...] on rank 0 (None elsewhere); out: [count][...] this rank's share."""
        import torch

        buf = out.new_empty((self.share,) + tuple(out.shape[1:]))
        if self.world == 1:
            out.copy_(full)
            return out
        chunks = self._chunks(full) if self.rank == 0 else None
        self.dist.scatter(buf, chunks, src=0)
        out.copy_(buf[:self.count])
        return out

    def gather(self, part, full):
        """part: [count][...] this rank's results; full: [nof_cells][...] filled on rank 0 (None elsewhere)."""
        import torch

        if self.world == 1:
            full.copy_(part)
            return full
        buf = part.new_zeros((self.share,) + tuple(part.shape[1:]))
        buf[:self.count] = part
        bufs = [torch.empty_like(buf) for _ in range(self.world)] if self.rank == 0 else None
        self.dist.gather(buf, bufs, dst=0)
        if self.rank == 0:
            for r in range(self.world):
                a, n = cell_range(self.nof_cells, self.world, r)
                full[a:a + n] = bufs[r][:n]
        return full
