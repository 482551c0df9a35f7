"""Mixed PUSCH slots for the slot-form and plug-in tests: one 273-PRB, four-port received grid shared by PDUs of
every kind the reference's pusch_processor_impl::process serves in one slot (uplink_processor_impl.cpp:270-326):

  uci     HARQ-ACK (5 bits) + CSI part 1 (12 bits) multiplexed on the UL-SCH, 4 rx ports
  tp      transform precoding (DFT-s-OFDM, low-PAPR DM-RS), 25 PRB, 4 rx ports
  harq    a HARQ process received on port 0 only at a low SNR: rv 0 (new data, kept) fails, rv 2 (new_data = false)
          decodes after combining with it
  plain   64QAM, 2 layers, 4 rx ports (the fused slot path)
  plain2  QPSK, 1 layer, 4 rx ports, its own DM-RS symbols (the fused slot path)

and, on request (kinds=...; they take the PRBs of tp / harq, so a slot holds them instead of those):

  csi2    HARQ-ACK (2 bits) + CSI part 1 (12 bits) + CSI part 2 sized by CSI part 1 (two fields, 8 sizes) on the
          UL-SCH, 16QAM, 25 PRB
  ucionly no codeword (tbs = 0): HARQ-ACK (1 bit) + CSI part 1 (20 bits), QPSK (no CSI part 2: the reference sizes a
          UCI-only PDU's CSI part 1 for "no CSI part 2" before the part 2 size is known, ulsch_info.cpp:96-123, so the
          two cannot share a PDU consistently)

Each UE's transmission comes from the reference's own transmit classes (oracle.pusch_proc.ue_transmit /
ue_transmit_tp); the grid is their sum plus AWGN (the strong UEs at SNR_DB, the HARQ UE scaled to HARQ_SNR_DB).
TEST INFRASTRUCTURE ONLY.
"""
import numpy as np

from oracle import pusch_proc as pp
from oracle.pdsch_mod import to_bf16

import srsran_project_amd as amd

NPRB = 273
NSUBC = 12 * NPRB
SNR_DB = 28.0
HARQ_SNR_DB = 8.0

BASE = dict(numerology=1, slot_index=0, rnti=1, bwp_start_rb=0, bwp_size_rb=NPRB, modulation=2,
            target_code_rate=679.0, rv=0, base_graph=1, new_data=1, n_id=0, nof_tx_layers=1, nof_rx_ports=4,
            dmrs_symbol_mask=(1 << 2) | (1 << 11), dmrs_type=1, scrambling_id=0, n_scid=0,
            nof_cdm_groups_without_data=2, rb_start=0, rb_count=NPRB, start_symbol_index=0, nof_symbols=14)

UES = [
    ("uci", dict(rnti=0x5001, n_id=7, scrambling_id=70, rb_start=0, rb_count=60, modulation=4, target_code_rate=490.0,
                 nof_harq_ack=5, nof_csi_part1=12, beta_offset_harq_ack=8.0, beta_offset_csi_part1=6.25,
                 alpha_scaling=1.0)),
    ("tp", dict(rnti=0x5002, n_id=8, rb_start=60, rb_count=25, modulation=4, target_code_rate=434.0,
                transform_precoding=1, n_rs_id=77)),
    ("harq", dict(rnti=0x5003, n_id=9, scrambling_id=90, rb_start=90, rb_count=60, modulation=4,
                  target_code_rate=658.0, nof_rx_ports=1)),
    ("plain", dict(rnti=0x5004, n_id=10, scrambling_id=100, n_scid=1, rb_start=150, rb_count=80, modulation=6,
                   target_code_rate=567.0, nof_tx_layers=2, dmrs_symbol_mask=(1 << 2) | (1 << 7) | (1 << 11))),
    ("plain2", dict(rnti=0x5005, n_id=11, scrambling_id=110, rb_start=230, rb_count=43, modulation=2,
                    target_code_rate=679.0, nof_cdm_groups_without_data=1, dmrs_symbol_mask=1 << 3,
                    start_symbol_index=1, nof_symbols=12)),
]


PART2_CSI2 = [([(1, 1), (4, 2)], [3, 1, 2, 11, 30, 0, 64, 7])]
UES_EXTRA = [
    ("csi2", dict(rnti=0x5006, n_id=12, scrambling_id=120, rb_start=60, rb_count=25, modulation=4,
                  target_code_rate=490.0, nof_harq_ack=2, nof_csi_part1=12, beta_offset_harq_ack=8.0,
                  beta_offset_csi_part1=6.25, beta_offset_csi_part2=5.0, alpha_scaling=1.0, csi_part2_size=PART2_CSI2)),
    ("ucionly", dict(rnti=0x5007, n_id=13, scrambling_id=130, rb_start=90, rb_count=10, modulation=2,
                     target_code_rate=679.0, nof_harq_ack=1, nof_csi_part1=20, beta_offset_harq_ack=8.0,
                     beta_offset_csi_part1=6.25, alpha_scaling=1.0)),
]


def _cplx(g):
    f = np.stack([((g & 0xFFFF) << 16).view(np.float32), ((g >> 16) << 16).view(np.float32)], -1)
    return (f[..., 0] + 1j * f[..., 1]).astype(np.complex128)


def _bf16(z):
    return np.ascontiguousarray(to_bf16(z.real.astype(np.float32)).astype(np.uint32)
                                | (to_bf16(z.imag.astype(np.float32)).astype(np.uint32) << 16))


def tbs_of(pdu):
    tp = pdu.get("transform_precoding", 0)
    nd = bin(pdu["dmrs_symbol_mask"]).count("1")
    ndmrs = 12 * nd if tp else 6 * nd * pdu["nof_cdm_groups_without_data"]
    return amd.tbs_calculator_calculate(pdu["nof_symbols"], ndmrs, 0, pdu["modulation"], pdu["target_code_rate"],
                                        pdu["nof_tx_layers"], 0, pdu["rb_count"])


def base_graph_of(tbs, rate):
    r = rate / 1024
    return 2 if (tbs <= 292 or (tbs <= 3824 and r <= 0.67) or r <= 0.25) else 1


def _chan(L, P, seed):
    rng = np.random.default_rng(seed)
    h = np.eye(L, P) + 0.25 * (rng.normal(size=(L, P)) + 1j * rng.normal(size=(L, P)))
    return (0.8 * h).astype(np.complex64)


def mixed_slot(slot_index, harq_rv, seed, kinds=None):
    """The received grid (uint32 [4][14][NSUBC]) of one slot, the PDU dicts (with tbs / base_graph / slot /
    HARQ-process rv and new_data), the transport blocks and UCI payloads each UE sent.  The HARQ UE sends the
    same transport block in every slot (its HARQ process), the others new ones."""
    kinds = kinds or [k for k, _ in UES]
    rng = np.random.default_rng(1000 + seed)
    z = np.zeros((4, 14, NSUBC), np.complex128)
    pdus, sent = [], []
    strong = None
    parts = []
    for u, (kind, over) in enumerate(UES + UES_EXTRA):
        if kind not in kinds:
            continue
        pdu = dict(BASE, **over, slot_index=slot_index)
        if kind == "harq":
            pdu.update(rv=harq_rv, new_data=int(harq_rv == 0))
        tbs = 0 if kind == "ucionly" else tbs_of(pdu)
        pdu["tbs"] = tbs
        pdu["base_graph"] = base_graph_of(tbs, pdu["target_code_rate"])
        tb_rng = np.random.default_rng(77 if kind == "harq" else 31 * seed + u)
        tb = tb_rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        uci = None
        if kind in ("uci", "csi2", "ucionly"):
            uci = (rng.integers(0, 2, pdu["nof_harq_ack"]).astype(np.uint8),
                   rng.integers(0, 2, pdu["nof_csi_part1"]).astype(np.uint8))
            if "csi_part2_size" in pdu:
                n2 = amd.uci_part2_get_size(uci[1], amd.uci_part2_description(pdu["csi_part2_size"]))
                uci = uci + (rng.integers(0, 2, n2).astype(np.uint8),)
        P = pdu["nof_rx_ports"]
        if kind == "tp":
            g, _ = pp.ue_transmit_tp(tb, pdu, NSUBC, channel=np.array([0.8, 0.3j, -0.5, 0.6 + 0.2j]))
        else:
            g, _ = pp.ue_transmit(tb, pdu, NSUBC, channel=_chan(pdu["nof_tx_layers"], P, 40 + u), uci=uci)
        zu = np.zeros_like(z)
        zu[:P] = _cplx(g)
        occ = np.abs(zu) > 0
        pw = float(np.mean(np.abs(zu[occ]) ** 2))
        parts.append((kind, zu, pw))
        if kind != "harq" and strong is None:
            strong = pw
        pdus.append(pdu)
        sent.append((tb, uci))
    sigma2 = (strong if strong is not None else 1.0) / 10 ** (SNR_DB / 10)
    for kind, zu, pw in parts:
        target = HARQ_SNR_DB if kind == "harq" else SNR_DB
        z += zu * np.sqrt(sigma2 * 10 ** (target / 10) / pw)
    z += np.sqrt(sigma2 / 2) * (rng.normal(size=z.shape) + 1j * rng.normal(size=z.shape))
    return _bf16(z), pdus, sent


def kind_of(pdu):
    if pdu.get("tbs", 1) == 0:
        return "ucionly"
    if "csi_part2_size" in pdu:
        return "csi2"
    if pdu.get("nof_harq_ack", 0) or pdu.get("nof_csi_part1", 0):
        return "uci"
    if pdu.get("transform_precoding", 0):
        return "tp"
    if pdu["nof_rx_ports"] == 1:
        return "harq"
    return "plain"
