"""CPU oracle of the PUSCH DM-RS channel estimator -- TEST INFRASTRUCTURE ONLY.

Restates, in numpy float32 (pinned against the reference's own
dmrs_pusch_estimator_impl + port_channel_estimator_average_impl compiled into
oracle/_ref by oracle/Makefile, tests/test_oracle_vs_ref.py, within a float
tolerance: sums are reassociated):
  pilots()            dmrs_pusch_estimator_impl.cpp:72-184 (pseudo-random sequence, CDM weights)
  estimate_port()     port_channel_estimator_average_impl.cpp:130-506 (LSE, CFO estimation and
                      compensation, pair averaging, FD smoothing, linear interpolation, TD strategy,
                      noise / RSRP / EPRE / SNR) with port_channel_estimator_helpers.cpp
                      (apply_fd_smoothing :213-260, virtual pilots :334-418, filter :58-100) and
                      time_alignment_estimator_dft_impl.cpp (:122-310).
Single hop (no frequency hopping), contiguous PRB allocation, DM-RS type 1.
Estimates are complex bf16 (uint32, real in the low half).
"""
import ctypes

import numpy as np

from . import REF, _ptr, prbs
from .pdsch_mod import to_bf16

NRE = 12
NSYMB = 14
MAX_RB = 275
MAX_V_PILOTS = 12
MAX_SINR_DB = 100.0
T_C = 1.0 / (480e3 * 4096)
MAX_DFT = 4096  # pow2(log2_ceil(MAX_RB * NRE))
RC_FILTER = np.array([
    -0.0641253, -0.0660711, -0.0611526, -0.0485918, -0.0281126, 0.0000000, 0.0348830, 0.0751249,
    0.1188406, 0.1637874, 0.2075139, 0.2475302, 0.2814857, 0.3073415, 0.3235207, 0.3290274,
    0.3235207, 0.3073415, 0.2814857, 0.2475302, 0.2075139, 0.1637874, 0.1188406, 0.0751249,
    0.0348830, 0.0000000, -0.0281126, -0.0485918, -0.0611526, -0.0660711, -0.0641253], np.float32)
f32 = np.float32


def symbol_start_epochs(numerology):
    """port_channel_estimator_average_impl.cpp:542-553 (normal CP)."""
    scs_hz = (15 << numerology) * 1000

    def cp_s(i):
        k = (144 >> numerology) + (16 if (i == 0 or i == 7 * (1 << numerology)) else 0)
        return k * 64 * T_C

    e = np.zeros(NSYMB, np.float32)
    e[0] = f32(cp_s(0) * scs_hz)
    for i in range(1, NSYMB):
        e[i] = f32(float(e[i - 1]) + cp_s(i) * scs_hz + 1.0)
    return e


def dmrs_re_offsets(type2, cdm):
    if not type2:
        return np.arange(0, NRE, 2) + cdm
    return np.array([0, 1, 6, 7]) + 2 * cdm


def pilots(slot_index, type2, nof_layers, scrambling_id, n_scid, symbols_mask, prb_lo, prb_hi):
    """complex64 [layers][nof_dmrs_symbols][npil] (dmrs_pusch_estimator_impl.cpp:72-184)."""
    nd = 4 if type2 else 6
    amp = f32(np.sqrt(0.5))
    syms = [l for l in range(NSYMB) if (symbols_mask >> l) & 1]
    npil = (prb_hi - prb_lo) * nd
    base = np.zeros((len(syms), npil), np.complex64)
    for d, l in enumerate(syms):
        c_init = ((NSYMB * slot_index + l + 1) * (2 * scrambling_id + 1) * (1 << 17) + (2 * scrambling_id + n_scid)) \
            % (1 << 31)
        c = prbs(c_init, 2 * prb_hi * nd)[2 * prb_lo * nd:]
        base[d] = np.where(c[0::2] == 0, amp, -amp) + 1j * np.where(c[1::2] == 0, amp, -amp)
    out = np.zeros((nof_layers, len(syms), npil), np.complex64)
    for v in range(nof_layers):
        out[v] = base
        if v % 2 == 1:  # w_f = {+1, -1}; w_t = +1 for layers < 4
            out[v][:, 1::2] *= -1
    return out, syms


def _filter(nof_rb, stride):
    """filter_type (port_channel_estimator_helpers.cpp:58-100): (coefficients, unused tail correction)."""
    nof_rb = min(nof_rb, 3)
    nof_coefs = nof_rb * 10 + 1
    half = nof_coefs // 2 // stride
    n_first = 31 // 2 - half * stride
    n = 2 * half + 1
    coefs = RC_FILTER[n_first:n_first + n * stride:stride][:n].astype(np.float32)
    total = f32(0)
    for c in coefs:
        total = f32(total + c)
    return (coefs * (f32(1) / total)).astype(np.float32)


def _unwrap(args):
    a = args.astype(np.float32).copy()
    width = f32(np.pi)
    k = f32(0)
    for i in range(a.size - 1):
        old, nxt = a[i], a[i + 1]
        a[i] = f32(a[i] + f32(2) * k * width)
        jump = f32(nxt - old)
        if abs(jump) > width:
            k = f32(k - np.copysign(f32(1), jump))
    a[-1] = f32(a[-1] + f32(2) * k * width)
    return a


def _v_pilots(base, is_start):
    """compute_v_pilots (port_channel_estimator_helpers.cpp:334-378)."""
    n = base.size
    absv = np.abs(base).astype(np.float32)
    argv = _unwrap(np.angle(base).astype(np.float32))
    idx = np.arange(n, dtype=np.float32)
    mean_x = f32(f32(n * (n - 1)) / f32(2) / f32(n))
    norm_x_sq = f32(f32((n - 1) * n * (2 * n - 1)) / f32(6))

    def fit(v):
        m = f32(np.mean(v, dtype=np.float64))
        s = f32(np.dot(v.astype(np.float64), idx.astype(np.float64)))
        s = f32(s - mean_x * m * f32(n))
        s = f32(s / f32(norm_x_sq - f32(n) * mean_x * mean_x))
        return s, f32(m - s * mean_x)

    sa, ia = fit(absv)
    sg, ig = fit(argv)
    off = -n if is_start else n
    i_v = (np.arange(n) + off).astype(np.float32)
    rho = (sa * i_v + ia).astype(np.float32)
    ph = (sg * i_v + ig + np.where(rho > 0, f32(0), f32(np.pi))).astype(np.float32)
    return (np.abs(rho) * (np.cos(ph) + 1j * np.sin(ph))).astype(np.complex64)


def fd_smoothing(x, nof_rb, stride, strategy):
    """apply_fd_smoothing (port_channel_estimator_helpers.cpp:213-260). strategy 0 none, 1 mean, 2 filter."""
    if strategy == 0:
        return x.copy()
    if strategy == 1:
        return np.full_like(x, np.complex64(np.mean(x.astype(np.complex128))))
    rc = _filter(nof_rb, stride)
    nv = min(MAX_V_PILOTS, rc.size // 2)
    if nof_rb == 1:
        nv = x.size
    enl = np.concatenate([_v_pilots(x[:nv], True), x, _v_pilots(x[-nv:], False)])
    y = np.convolve(enl.astype(np.complex128), rc.astype(np.float64), mode="same")
    return y[nv:nv + x.size].astype(np.complex64)


def interpolate(pilots_f, nof_re, offset, stride):
    """interpolator_linear_impl.cpp: known values at offset + stride * i, linear in between, held at the ends."""
    out = np.zeros(nof_re, np.complex64)
    pos = offset + stride * np.arange(pilots_f.size)
    out[:offset + 1] = pilots_f[0]
    for i in range(pilots_f.size - 1):
        a, b = pilots_f[i], pilots_f[i + 1]
        r = np.arange(stride, dtype=np.float32) / f32(stride)
        seg = (a + (b - a) * r).astype(np.complex64)
        lo = pos[i]
        hi = min(lo + stride, nof_re)
        out[lo:hi] = seg[:hi - lo]
    last = pos[-1]
    if last < nof_re:
        out[last:] = pilots_f[-1]
    return out


def _ta(filtered, type2, offsets, numerology):
    """estimate_time_alignment + time_alignment_estimator_dft_impl::estimate (contiguous allocation)."""
    slices = filtered.reshape(-1, filtered.shape[-1])
    npil = slices.shape[1]
    scs = (15 << numerology) * 1000
    if not type2:
        req, stride = npil, 2
        pos = np.arange(npil)
    else:
        # Generic mask path: REs of the pattern over the PRB range, relative to the lowest one.
        nprb = npil // 4
        pos = (np.arange(nprb)[:, None] * NRE + offsets[None, :]).reshape(-1) - offsets[0]
        req, stride = int(pos[-1]) + 1, 1
    req = req * MAX_DFT // (MAX_RB * NRE)
    n = 1 << int(np.ceil(np.log2(max(req, 1))))
    min_dft = 1 << int(np.ceil(np.log2(1.0 / (15000 * 16 * 64 * T_C))))
    n = max(min_dft, n)
    corr = np.zeros(n, np.float64)
    for s in slices:
        buf = np.zeros(n, np.complex128)
        buf[pos] = s
        t = np.fft.ifft(buf) * n  # unnormalised inverse DFT
        corr += np.abs(t) ** 2
    half_cp = (144 * 64 / (1 << (numerology + 1))) * T_C
    fs = n * scs * stride
    max_taps = int(np.floor(half_cp * fs))
    d = corr[:max_taps]
    a = corr[n - max_taps:]
    i_d, v_d = int(np.argmax(d)), d.max()
    i_a, v_a = int(np.argmax(a)), a.max()
    idx = i_d if v_d >= v_a else -(max_taps - i_a)
    frac = 0.0
    if n != MAX_DFT:
        taps = 5 if max_taps > 2 else 3
        pk = np.array([corr[(idx + i + n - taps // 2) % n] for i in range(taps)])
        if taps == 5:
            num = np.dot([-0.4, -0.2, 0.0, 0.2, 0.4], pk)
            den = np.dot([0.571429, -0.285714, -0.571429, -0.285714, 0.571429], pk)
            r = -num / den
        else:
            r = -0.5 * np.dot([-0.5, 0.0, 0.5], pk) / np.dot([0.5, -1.0, 0.5], pk)
        frac = 0.0 if (not np.isfinite(r) or abs(r) > 1) else r
    return (idx + frac) / fs


def estimate_port(rx_grid, pil, syms, type2, prb_lo, prb_hi, first_symbol, nof_symbols, scaling, fd, td, compensate_cfo,
                  numerology):
    """One rx port: rx_grid complex64 [14][nsubc]. td: 0 interpolate, 1 average.
    Returns (estimates complex64 [layers][14][nof_re] or None rows, stats dict)."""
    L, nds, npil = pil.shape
    ncdm = (L + 1) // 2
    nd = 4 if type2 else 6
    epochs = symbol_start_epochs(numerology)
    beta = f32(scaling)
    nof_lse = 1 if td == 1 else nds
    nof_re = (prb_hi - prb_lo) * NRE
    rx = np.zeros((ncdm, nds, npil), np.complex64)
    for g in range(ncdm):
        sc = (np.arange(prb_lo, prb_hi)[:, None] * NRE + dmrs_re_offsets(type2, g)[None, :]).reshape(-1)
        for d, l in enumerate(syms):
            rx[g, d] = rx_grid[l, sc]
    epre = f32(np.sum(np.abs(rx.astype(np.complex128)) ** 2))
    # LSE per layer / DM-RS symbol (preprocess_pilots_and_estimate_cfo, compensate_cfo_and_accumulate).
    prod = np.zeros((L, nds, npil), np.complex64)
    for v in range(L):
        prod[v] = rx[v // 2] * np.conj(pil[v])
    cfo = None
    if nds >= 2:
        acc = []
        for g in range(ncdm):
            a = 0j
            lay = range(2 * g, min(2 * g + 2, L))
            for v in lay:
                a += np.sum(prod[v, 1].astype(np.complex128) * np.conj(prod[v, 0].astype(np.complex128)))
            acc.append(f32(np.angle(a) / (2 * np.pi) / (float(epochs[syms[1]]) - float(epochs[syms[0]]))))
        cfo = f32(np.sum(np.array(acc, np.float64)) / ncdm)
    lse = prod.copy()
    if cfo is not None and compensate_cfo:
        for d, l in enumerate(syms):
            lse[:, d] *= np.complex64(np.exp(-2j * np.pi * float(epochs[l]) * float(cfo)))
    if td == 1:
        lse = lse.sum(axis=1, keepdims=True, dtype=np.complex128).astype(np.complex64)
    # Pair averaging (average_pairs): one DM-RS symbol -> layers of two-layer CDM groups; more -> all layers if L > 1.
    avg_layers = [v for v in range(L) if (nds == 1 and min(2 * (v // 2) + 2, L) - 2 * (v // 2) == 2)] \
        if nds == 1 else (list(range(L)) if L > 1 else [])
    for v in avg_layers:
        x = lse[v]
        n2 = (npil // 2) * 2
        av = ((x[:, 0:n2:2] + x[:, 1:n2:2]) / f32(2)).astype(np.complex64)
        x[:, 0:n2:2] = av
        x[:, 1:n2:2] = av
    total = f32(f32(1) / beta)
    if td == 1:
        total = f32(total / f32(nds))
    offset = int(dmrs_re_offsets(type2, 0)[0])
    stride = int(dmrs_re_offsets(type2, 0)[1] - dmrs_re_offsets(type2, 0)[0])
    filt = np.zeros((L, nof_lse, npil), np.complex64)
    freq = np.zeros((L, nof_lse, nof_re), np.complex64)
    rsrp = f32(0)
    for v in range(L):
        # the interpolator offset / stride come from the layer's RE pattern (configure_interpolator)
        offs = dmrs_re_offsets(type2, v // 2)
        off_v, stride_v = int(offs[0]), int(offs[1] - offs[0])
        for s in range(nof_lse):
            x = (lse[v, s] * total).astype(np.complex64)
            filt[v, s] = fd_smoothing(x, prb_hi - prb_lo, stride_v, fd)
            p = f32(np.sum(np.abs(filt[v, s].astype(np.complex128)) ** 2))
            rsrp = f32(rsrp + p * (beta * beta * f32(nds) / f32(nof_lse)))
            freq[v, s] = interpolate(filt[v, s], nof_re, off_v, stride_v)
    del offset, stride
    # Time-domain strategy -> estimates for the allocation's symbols.
    est = np.zeros((L, NSYMB, nof_re), np.complex64)
    dmrs_set = set(syms)
    last = first_symbol + nof_symbols
    for v in range(L):
        for l in range(first_symbol, last):
            if td == 1:
                e = freq[v, 0]
            else:
                before = max([d for d in syms if first_symbol <= d < l], default=-1)
                after = min([d for d in syms if l <= d < last], default=-1)
                e = None
                if before == -1:
                    second = min([d for d in syms if after + 1 <= d < last], default=-1)
                    if second == -1:
                        e = freq[v, 0]
                    else:
                        before, after = after, second
                if e is None and after == -1:
                    second_last = max([d for d in syms if first_symbol <= d < before], default=-1)
                    if second_last == -1:
                        e = freq[v, nds - 1]
                    else:
                        after, before = before, second_last
                if e is None:
                    w = f32(f32(l - before) / f32(after - before))
                    i = len([d for d in syms if first_symbol <= d < before])
                    e = (freq[v, i] + (freq[v, i + 1] - freq[v, i]) * w).astype(np.complex64)
            est[v, l] = e
    del dmrs_set
    # Noise (estimate_noise) per CDM group.
    noise = f32(0)
    for g in range(ncdm):
        lay = list(range(2 * g, min(2 * g + 2, L)))
        sc_est = {v: (filt[v].astype(np.complex128).sum(axis=0) * float(f32(beta / f32(nof_lse)))) for v in lay}
        energy = 0.0
        for d, l in enumerate(syms):
            pred = sum(sc_est[v] * pil[v, d] for v in lay)
            if compensate_cfo and cfo is not None:
                pred = pred * np.exp(2j * np.pi * float(epochs[l]) * float(cfo))
            energy += np.sum(np.abs(rx[g, d] - pred) ** 2)
        energy = f32(energy)
        noise = f32(noise + (energy if np.isfinite(energy) and energy != 0 else f32(0)))
    ta = _ta(filt, type2, dmrs_re_offsets(type2, 0), numerology)
    return est, dict(epre=epre, rsrp=rsrp, noise=noise, cfo=cfo, ta=ta, npil=npil * nds, ncdm=ncdm)


def pusch_chest(grid, slot_index, type2, nof_layers, scrambling_id, n_scid, scaling, symbols_mask, prb_lo, prb_hi,
                first_symbol, nof_symbols, fd=2, td=1, compensate_cfo=True, numerology=1, estimates=None):
    """grid uint32 [ports][14][nsubc]. Returns (estimates uint32 [ports][layers][14][nsubc], stats per port).
    DM-RS type 1 only: with the type-2 pattern the reference's linear interpolator (stride 1 over 4 pilots
    per RB) reads past its input (interpolator_linear_impl.cpp:103-113), which has no defined result."""
    if type2:
        raise ValueError("PUSCH channel estimation restated for DM-RS type 1 only")
    P, _, nsubc = grid.shape
    u = grid.astype(np.uint32)
    cg = ((u & 0xFFFF) << 16).view(np.float32) + 1j * ((u >> 16) << 16).view(np.float32)
    pil, syms = pilots(slot_index, type2, nof_layers, scrambling_id, n_scid, symbols_mask, prb_lo, prb_hi)
    out = np.zeros((P, nof_layers, NSYMB, nsubc), np.uint32) if estimates is None else estimates.copy()
    stats = []
    scs_hz = (15 << numerology) * 1000
    for p in range(P):
        est, st = estimate_port(cg[p].astype(np.complex64), pil, syms, type2, prb_lo, prb_hi, first_symbol,
                                nof_symbols, scaling, fd, td, compensate_cfo, numerology)
        npil_total, ncdm = st["npil"], st["ncdm"]
        rsrp = f32(st["rsrp"] / f32(npil_total * nof_layers))
        epre = f32(st["epre"] / f32(npil_total))
        nvar = f32(st["noise"] / f32(npil_total * ncdm - 1))
        nvar = max(f32(rsrp / f32(10 ** (MAX_SINR_DB / 10))), nvar)
        datarp = f32(rsrp * f32(nof_layers) / f32(scaling) / f32(scaling))
        snr = f32(datarp / nvar) if np.isfinite(nvar) and nvar != 0 else f32(0)
        cfo = st["cfo"]
        lo, hi = prb_lo * NRE, prb_hi * NRE
        for v in range(nof_layers):
            for l in range(first_symbol, first_symbol + nof_symbols):
                e = est[v, l]
                row = out[p, v, l].copy()
                row[lo:hi] = to_bf16(e.real.astype(np.float32)).astype(np.uint32) | \
                    (to_bf16(e.imag.astype(np.float32)).astype(np.uint32) << 16)
                # the CFO phase is applied to the whole OFDM symbol (do_compute, :184-193), stale REs included
                re, im = row & 0xFFFF, row >> 16
                if compensate_cfo and cfo is not None:
                    # sc_prod on the bf16 estimate (second rounding)
                    ef = ((re << 16).view(np.float32) + 1j * (im << 16).view(np.float32)).astype(np.complex64)
                    ef = (ef * np.complex64(np.exp(2j * np.pi * float(symbol_start_epochs(numerology)[l])
                                                   * float(cfo)))).astype(np.complex64)
                    re = to_bf16(ef.real.astype(np.float32)).astype(np.uint32)
                    im = to_bf16(ef.imag.astype(np.float32)).astype(np.uint32)
                out[p, v, l] = re | (im << 16)
        stats.append(dict(noise_var=nvar, epre=epre, snr=snr, rsrp=rsrp, time_alignment_s=st["ta"],
                          cfo_hz=(np.nan if cfo is None else float(cfo) * scs_hz)))
    return out, stats


# ---- the reference itself -------------------------------------------------------------------------------------------
_c = ctypes
if REF is not None and hasattr(REF, "srs_ref_pusch_chest"):
    REF.srs_ref_pusch_chest.restype = _c.c_int
    REF.srs_ref_pusch_chest.argtypes = ([_c.c_void_p] + [_c.c_uint] * 4 + [_c.c_int, _c.c_uint, _c.c_uint, _c.c_int,
                                                                         _c.c_float, _c.c_uint, _c.c_void_p,
                                                                         _c.c_uint, _c.c_uint, _c.c_int, _c.c_int,
                                                                         _c.c_int] + [_c.c_void_p] * 7)
    REF.srs_ref_pusch_chest_many.restype = _c.c_double
    REF.srs_ref_pusch_chest_many.argtypes = [_c.c_void_p, _c.c_uint, _c.c_uint, _c.c_int, _c.c_uint, _c.c_uint,
                                             _c.c_void_p, _c.c_uint, _c.c_uint, _c.c_uint, _c.c_uint]


if REF is not None and hasattr(REF, "srs_ref_low_papr"):
    REF.srs_ref_low_papr.restype = None
    REF.srs_ref_low_papr.argtypes = [_c.c_void_p, _c.c_uint, _c.c_uint, _c.c_uint]


def ref_low_papr(M, u, v=0):
    """The reference's low_papr_sequence_generator_impl::generate(sequence, u, v, 0, 1): complex64 [M]."""
    out = np.zeros(M, np.complex64)
    REF.srs_ref_low_papr(_ptr(out), M, u, v)
    return out


def ref_pusch_chest(grid, slot_index, type2, nof_layers, scrambling_id, n_scid, scaling, symbols_mask, prb_lo, prb_hi,
                    first_symbol, nof_symbols, fd=2, td=1, compensate_cfo=True, numerology=1, estimates=None):
    g = np.ascontiguousarray(grid, dtype=np.uint32)
    P, _, nsubc = g.shape
    crbs = np.zeros(nsubc // NRE, np.uint8)
    crbs[prb_lo:prb_hi] = 1
    est = np.zeros((P, nof_layers, NSYMB, nsubc), np.uint32) if estimates is None else estimates.copy()
    nv, ep, sn = (np.zeros(P, np.float32) for _ in range(3))
    rs = np.zeros(P * nof_layers, np.float32)
    ta = np.zeros(P * nof_layers, np.float64)
    cf = np.zeros(P * nof_layers, np.float32)
    r = REF.srs_ref_pusch_chest(_ptr(g), P, nsubc, numerology, slot_index, int(type2), nof_layers, scrambling_id,
                                int(n_scid), float(scaling), symbols_mask, _ptr(crbs), first_symbol, nof_symbols, fd,
                                td, int(compensate_cfo), _ptr(est), _ptr(nv), _ptr(ep), _ptr(sn), _ptr(rs), _ptr(ta),
                                _ptr(cf))
    if r != 0:
        raise RuntimeError("reference estimator did not notify")
    stats = [dict(noise_var=nv[p], epre=ep[p], snr=sn[p], rsrp=rs[p * nof_layers], time_alignment_s=ta[p * nof_layers],
                  cfo_hz=float(cf[p * nof_layers])) for p in range(P)]
    return est, stats
