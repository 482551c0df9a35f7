"""CPU restatement of srsRAN's channel equalizer (ZF / MMSE) -- TEST
INFRASTRUCTURE ONLY (tests/ and bench cpu_baseline legs; never the product).

numpy float64 on the bf16 inputs (exact arithmetic, the value the reference's
float32 code approximates).  Reference:
  lib/phy/upper/equalization/channel_equalizer_generic_impl.cpp:290-378  dispatch,
      max noise variance for 2 layers, is_supported (:240-270)
  lib/phy/upper/equalization/channel_equalizer_generic_impl.cpp:122-170  1-layer port reduction
  lib/phy/upper/equalization/equalize_zf_1xn.h:131-170   ZF 1 x N (scalar path semantics)
  lib/phy/upper/equalization/equalize_zf_2xn.h:185-250   ZF 2 x N (scalar path semantics)
MMSE with one layer is the ZF equalizer (channel_equalizer_generic_impl.cpp:348).
Layouts: symbols cbf16 [port][re]; estimates cbf16 [layer][port][re]
(dynamic_ch_est_list.h dims {re, rx_port, tx_layer}); outputs [re][layer].
"""
import numpy as np

from .ofdm import bf16_to_float


def cbf16_to_complex(u16):
    f = bf16_to_float(u16).astype(np.float64)
    return f[..., 0::2] + 1j * f[..., 1::2]


def _isnormal(x):
    x = np.asarray(x, dtype=np.float64)
    with np.errstate(invalid="ignore"):
        return np.isfinite(x) & (np.abs(x) >= np.finfo(np.float32).tiny)


def is_supported(algorithm, nof_ports, nof_layers):
    if nof_ports not in (1, 2, 4) or nof_ports < nof_layers:
        return False
    if algorithm == "zf":
        return nof_layers in (1, 2)
    return nof_layers == 1


def equalize(symbols_u16, est_u16, noise_vars, tx_scaling, nof_layers):
    """symbols_u16: uint16 [ports, 2*nof_re]; est_u16: uint16 [layers, ports, 2*nof_re];
    noise_vars: float [ports].  Returns (eq complex128 [nof_re, layers], nvar float64 [nof_re, layers])."""
    y = cbf16_to_complex(symbols_u16)           # [P, R]
    h = cbf16_to_complex(est_u16)               # [L, P, R]
    nv = np.asarray(noise_vars, dtype=np.float64)
    P, R = y.shape
    eq = np.zeros((R, nof_layers), np.complex128)
    out_nv = np.full((R, nof_layers), np.inf)
    if nof_layers == 1:
        valid_port = _isnormal(nv) & (nv > 0)
        hn = np.abs(h[0]) ** 2                  # [P, R]
        ok = _isnormal(hn) & valid_port[:, None]
        ch_mod_sq = np.sum(np.where(ok, hn, 0.0), axis=0)
        nvar_acc = np.sum(np.where(ok, hn * nv[:, None], 0.0), axis=0)
        re_out = np.sum(np.where(ok, y * np.conj(h[0]), 0.0), axis=0)
        d = tx_scaling * ch_mod_sq
        good = _isnormal(d) & _isnormal(nvar_acc)
        with np.errstate(divide="ignore", invalid="ignore"):
            eq[:, 0] = np.where(good, re_out / d, 0)
            out_nv[:, 0] = np.where(good, nvar_acc / d / d, np.inf)
        return eq, out_nv
    assert nof_layers == 2
    noise = float(np.max(nv))
    if not (_isnormal(noise) and noise >= 0):
        return eq, out_nv
    n0 = np.sum(np.abs(h[0]) ** 2, axis=0)
    n1 = np.sum(np.abs(h[1]) ** 2, axis=0)
    xi = np.sum(np.conj(h[0]) * h[1], axis=0)
    m0 = np.sum(np.conj(h[0]) * y, axis=0)
    m1 = np.sum(np.conj(h[1]) * y, axis=0)
    d = tx_scaling * (n0 * n1 - np.abs(xi) ** 2)
    good = _isnormal(d)
    with np.errstate(divide="ignore", invalid="ignore"):
        eq[:, 0] = np.where(good, (n1 * m0 - xi * m1) / d, 0)
        eq[:, 1] = np.where(good, (n0 * m1 - np.conj(xi) * m0) / d, 0)
        out_nv[:, 0] = np.where(good, noise * n1 / (tx_scaling * d), np.inf)
        out_nv[:, 1] = np.where(good, noise * n0 / (tx_scaling * d), np.inf)
    return eq, out_nv


PIVOT_REL = 2.0 ** -20  # equalizer_device.h: a Cholesky pivot below 2^-20 x its diagonal entry is singular


def is_supported_mimo(algorithm, nof_ports, nof_layers):
    """Topologies of the MI355X equalizer: the reference's (is_supported) plus the L-layer solves the open
    reference asserts for (ZF 3x4 / 4x4, MMSE 2xN / 3x4 / 4x4, channel_equalizer_generic_impl.cpp:197-247)."""
    return nof_ports in (1, 2, 4) and 1 <= nof_layers <= min(4, nof_ports) and algorithm in ("zf", "mmse")


def equalize_mimo(symbols_u16, est_u16, noise_vars, tx_scaling, nof_layers, algorithm):
    """fp64 restatement of equalizer_device.h equalize_mimo -- PARITY UNPINNED (no open reference): y = ts H x + n,
    sigma^2 = the largest port noise variance (channel_equalizer_generic_impl.cpp:304).
      zf:   x = (H^H H)^-1 H^H y / ts, nv_l = sigma^2 [(H^H H)^-1]_ll / ts^2
      mmse: A = ts^2 H^H H + sigma^2 I, u = A^-1 ts H^H y, d = diag(A^-1), mu = 1 - sigma^2 d,
            x = u / mu, nv = sigma^2 d / mu (unbiased MMSE; equal to ZF for one layer).
    Invalid sigma^2 (not a positive normal number for MMSE, not normal and >= 0 for ZF), a Gram / A matrix with a
    Cholesky pivot not above 2^-20 times its diagonal entry (singular in float32 terms): zero symbols and
    infinite variances; likewise mu_l <= 2^-20 (no signal on the layer).
    Returns (eq complex128 [R, L], nv float64 [R, L], kappa [R]: condition number of the solve, x 1/min(mu) for
    MMSE -- the float32 error amplification the GPU tolerance scales with)."""
    y = cbf16_to_complex(symbols_u16)           # [P, R]
    h = cbf16_to_complex(est_u16)               # [L, P, R]
    P, R = y.shape
    L = nof_layers
    eq = np.zeros((R, L), np.complex128)
    out_nv = np.full((R, L), np.inf)
    kappa = np.ones(R)
    sigma = float(np.max(np.asarray(noise_vars, np.float64)))
    mmse = algorithm == "mmse"
    noise_ok = _isnormal(sigma) and (sigma > 0 if mmse else sigma >= 0)
    if not noise_ok:
        return eq, out_nv, kappa
    H = np.transpose(h, (2, 1, 0))              # [R, P, L]
    G = np.einsum("rpi,rpk->rik", np.conj(H), H)
    b = np.einsum("rpi,rp->ri", np.conj(H), y.T)
    ts = float(tx_scaling)
    A = ts * ts * G + sigma * np.eye(L) if mmse else G
    rhs = ts * b if mmse else b
    finite = np.all(np.isfinite(A.reshape(R, -1)), axis=1)
    A_ok = np.where(finite[:, None, None], A, np.eye(L))
    # positive definiteness as the Cholesky pivots see it
    def _chol_ok(M):
        # the GPU's singularity rule: every Cholesky pivot a normal number above 2^-20 times its diagonal entry
        C = np.linalg.cholesky(M)
        piv = np.real(np.diagonal(C, axis1=-2, axis2=-1)) ** 2
        diag = np.real(np.diagonal(M, axis1=-2, axis2=-1))
        return np.all(_isnormal(piv) & (piv > PIVOT_REL * diag), axis=-1)

    try:
        good = finite & _chol_ok(A_ok)
    except np.linalg.LinAlgError:  # some RE is not positive definite: decide RE by RE
        good = np.zeros(R, bool)
        for r in np.nonzero(finite)[0]:
            try:
                good[r] = bool(_chol_ok(A_ok[r]))
            except np.linalg.LinAlgError:
                good[r] = False
    A_ok = np.where(good[:, None, None], A_ok, np.eye(L))
    Ainv = np.linalg.inv(A_ok)
    u = np.einsum("rik,rk->ri", Ainv, rhs)
    d = np.real(np.diagonal(Ainv, axis1=1, axis2=2))
    kappa = np.where(good, np.linalg.cond(A_ok), 1.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        if mmse:
            mu = 1.0 - sigma * d
            good = good & np.all(mu > PIVOT_REL, axis=1)  # mu_l (SINR / (1 + SINR)) above 2^-20, as the GPU
            x = u / mu
            nv = sigma * d / mu
            kappa = kappa / np.clip(np.min(mu, axis=1), 1e-30, None)
        else:
            x = u / ts
            nv = sigma * d / (ts * ts)
    eq[good] = x[good]
    out_nv[good] = nv[good]
    return eq, out_nv, np.where(good, kappa, 1.0)


def random_channel(rng, nof_re, nof_ports, nof_layers, snr_db=20.0):
    """Rayleigh channel, QPSK per layer, AWGN: returns (symbols uint16 [P, 2R], est uint16
    [L, P, 2R], noise_var float32 [P], tx complex [R, L])."""
    from .ofdm import float_to_bf16

    def to_cbf16(z):
        out = np.empty(z.shape[:-1] + (2 * z.shape[-1],), np.uint16)
        out[..., 0::2] = float_to_bf16(z.real.astype(np.float32))
        out[..., 1::2] = float_to_bf16(z.imag.astype(np.float32))
        return out

    h = (rng.normal(size=(nof_layers, nof_ports, nof_re)) + 1j * rng.normal(size=(nof_layers, nof_ports, nof_re)))
    h /= np.sqrt(2)
    x = (rng.choice([-1.0, 1.0], (nof_layers, nof_re)) + 1j * rng.choice([-1.0, 1.0], (nof_layers, nof_re)))
    x /= np.sqrt(2)
    nvar = 10 ** (-snr_db / 10)
    noise = (rng.normal(size=(nof_ports, nof_re)) + 1j * rng.normal(size=(nof_ports, nof_re))) * np.sqrt(nvar / 2)
    y = np.einsum("lpr,lr->pr", h, x) + noise
    return to_cbf16(y), to_cbf16(h), np.full(nof_ports, nvar, np.float32), x.T
