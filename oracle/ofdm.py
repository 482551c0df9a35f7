"""CPU restatement of srsRAN's OFDM modulator / demodulator (TS 38.211 Section 5.3
and 5.4) -- TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke() and the
cpu_baseline legs of the benches may use it; the product never does).

numpy, complex128: the DFT is computed exactly (np.fft), so this is the
"true" value the reference's float32 DFT approximates; tests compare both the
reference (oracle/_ref, pinned in tests/test_oracle_vs_ref.py) and the GPU path
against it within stated float tolerances.

Reference:
  lib/phy/lower/modulation/ofdm_modulator_impl.cpp:56-106    symbol modulation (grid halves, IDFT, scale*phase, CP)
  lib/phy/lower/modulation/ofdm_demodulator_impl.cpp:95-145  symbol demodulation (window, DFT, scale*phase, window comp)
  lib/phy/lower/modulation/phase_compensation_lut.h:45-75     phase compensation per symbol of a subframe
  include/srsran/ran/cyclic_prefix.h:93-104                   CP length in units of kappa
  include/srsran/ran/phy_time_unit.h:100-110                  to_samples
  include/srsran/adt/bf16.h:39-80                             float <-> bfloat16 (round half to even)
  Resource grids are complex bf16 [symbol][subcarrier] (lib/phy/support/resource_grid_impl.h:50).
"""
import math

import numpy as np

NRE = 12


def nsymb_per_slot(extended_cp):
    return 12 if extended_cp else 14


def sampling_rate_hz(numerology, dft_size):
    return 15000 * (1 << numerology) * dft_size


def cp_length(symbol, numerology, dft_size, extended_cp=False):
    """CP samples of symbol `symbol` (index within the subframe)."""
    if extended_cp:
        kappa = 512 >> numerology
    else:
        kappa = 144 >> numerology
        if symbol == 0 or symbol == 7 * (1 << numerology):
            kappa += 16
    num = kappa * 64 * sampling_rate_hz(numerology, dft_size)
    den = 15000 * 2048 * 64
    assert num % den == 0, "incompatible sampling rate"
    return num // den


def symbol_size(symbol, numerology, dft_size, extended_cp=False):
    return cp_length(symbol, numerology, dft_size, extended_cp) + dft_size


def slot_size(slot, numerology, dft_size, extended_cp=False):
    ns = nsymb_per_slot(extended_cp)
    return sum(symbol_size(ns * slot + s, numerology, dft_size, extended_cp) for s in range(ns))


def phase_lut(numerology, dft_size, center_freq_hz, is_tx, extended_cp=False):
    """complex64 coefficient per symbol of a subframe (phase_compensation_lut.h)."""
    srate = float(sampling_rate_hz(numerology, dft_size))
    sign_two_pi = (-1.0 if is_tx else 1.0) * 2.0 * math.pi
    out = []
    offset = 0
    for s in range((1 << numerology) * nsymb_per_slot(extended_cp)):
        offset += cp_length(s, numerology, dft_size, extended_cp)
        start = float(offset) / srate
        ph = sign_two_pi * center_freq_hz * start
        out.append(complex(math.cos(ph), math.sin(ph)))
        offset += dft_size
    return np.array(out, dtype=np.complex64)


def bf16_to_float(u16):
    return (np.asarray(u16, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def float_to_bf16(x):
    """to_bf16 (bf16.h:39): add 0x7fff + lsb, keep the high half."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFFFFFF
    return (u >> 16).astype(np.uint16)


def grid_to_complex(grid_u16):
    """cbf16 grid (uint16 [..., 2*n] interleaved re/im) -> complex128 [..., n]."""
    f = bf16_to_float(grid_u16).astype(np.float64)
    return f[..., 0::2] + 1j * f[..., 1::2]


def complex_to_grid(z):
    z = np.asarray(z)
    out = np.empty(z.shape[:-1] + (2 * z.shape[-1],), np.uint16)
    out[..., 0::2] = float_to_bf16(z.real.astype(np.float32))
    out[..., 1::2] = float_to_bf16(z.imag.astype(np.float32))
    return out


def _coef(lut, symbol, scale):
    c = np.complex64(lut[symbol]) * np.float32(scale)  # cf_t * float, in float
    return complex(np.complex64(c))


def modulate_slot(grid_u16, slot, numerology, bw_rb, dft_size, scale, center_freq_hz, extended_cp=False):
    """ofdm_slot_modulator::modulate for one port.  grid_u16: uint16 [nsymb, 2*rg]
    (cbf16).  Returns complex128 time samples [slot_size]."""
    rg = bw_rb * NRE
    N = dft_size
    ns = nsymb_per_slot(extended_cp)
    lut = phase_lut(numerology, N, center_freq_hz, True, extended_cp)
    X = grid_to_complex(grid_u16)
    out = []
    for s in range(ns):
        l = ns * slot + s
        cp = cp_length(l, numerology, N, extended_cp)
        x = np.zeros(N, np.complex128)
        x[N - rg // 2:] = X[s, :rg // 2]
        x[:rg // 2] = X[s, rg // 2:rg]
        y = np.fft.ifft(x) * N  # INVERSE, unnormalised (FFTW_BACKWARD convention)
        y = y * _coef(lut, l, scale)
        out.append(np.concatenate([y[N - cp:], y]))
    return np.concatenate(out)


def demodulate_slot(samples, slot, numerology, bw_rb, dft_size, scale, center_freq_hz, window_offset=0,
                    extended_cp=False, as_bf16=True):
    """ofdm_slot_demodulator::demodulate for one port.  samples: complex [slot_size].
    Returns the cbf16 grid uint16 [nsymb, 2*rg] (or complex128 before rounding)."""
    rg = bw_rb * NRE
    N = dft_size
    ns = nsymb_per_slot(extended_cp)
    lut = phase_lut(numerology, N, center_freq_hz, False, extended_cp)
    samples = np.asarray(samples, np.complex128)
    if window_offset:
        omega = np.float32(np.float32(window_offset) * np.float32(2.0 * math.pi) / np.float32(N))
        ang = (omega * np.arange(N, dtype=np.float32)).astype(np.float32)
        wcomp = (np.cos(ang).astype(np.float32) + 1j * np.sin(ang).astype(np.float32))
    grid = np.zeros((ns, rg), np.complex128)
    pos = 0
    for s in range(ns):
        l = ns * slot + s
        cp = cp_length(l, numerology, N, extended_cp)
        win = samples[pos + cp - window_offset:pos + cp - window_offset + N]
        Y = np.fft.fft(win) * _coef(lut, l, scale)
        if window_offset:
            Y = Y * wcomp
        grid[s, :rg // 2] = Y[N - rg // 2:]
        grid[s, rg // 2:] = Y[:rg // 2]
        pos += cp + N
    return complex_to_grid(grid) if as_bf16 else grid


def random_grid(rng, nsymb, rg, amp=1.0):
    """Random cbf16 grid (QPSK-like plus noise), uint16 [nsymb, 2*rg]."""
    z = (rng.choice([-1.0, 1.0], (nsymb, rg)) + 1j * rng.choice([-1.0, 1.0], (nsymb, rg))) * (amp / math.sqrt(2))
    z = z + (rng.normal(0, 0.1, (nsymb, rg)) + 1j * rng.normal(0, 0.1, (nsymb, rg)))
    return complex_to_grid(z)
