"""Shared PUSCH channel-estimation test cases: synthetic received grids
(a frequency-selective, slowly rotating channel times random QPSK-like data
plus noise, the shapes of the reference's dmrs_pusch_estimator vector tests:
tests/unittests/phy/upper/signal_processors/dmrs_pusch_estimator_test_data.h,
whose .dat files are not in the reference tree) and the estimator settings."""
import numpy as np

from oracle.pdsch_mod import to_bf16

# (name, ports, nof_prb, rb_start, rb_count, layers, dmrs mask, first, nsym, fd, td, cfo, scaling, noise)
CASES = [
    ("1x1_52prb_filter_avg", 1, 52, 0, 52, 1, (1 << 2) | (1 << 11), 0, 14, 2, 1, True, 1.0, 0.05),
    ("2x2_part_filter_avg", 2, 52, 4, 36, 2, (1 << 2) | (1 << 11), 0, 14, 2, 1, True, 1.0, 0.05),
    ("4x4_273prb_filter_avg", 4, 273, 0, 273, 4, (1 << 2) | (1 << 11), 0, 14, 2, 1, True, 1.0, 0.02),
    ("2x4_interp", 2, 52, 0, 52, 4, (1 << 2) | (1 << 7) | (1 << 11), 0, 14, 2, 0, True, 1.0, 0.05),
    ("1rb", 1, 25, 3, 1, 1, 1 << 2, 0, 14, 2, 1, True, 1.0, 0.05),
    ("mean_nocfo_1dmrs", 2, 52, 0, 52, 2, 1 << 3, 1, 13, 1, 1, False, 1.0, 0.05),
    ("none_interp_4rx", 4, 106, 10, 90, 2, (1 << 2) | (1 << 7) | (1 << 11), 0, 14, 0, 0, True, 1.0, 0.05),
    ("3layers_interp", 2, 52, 0, 52, 3, (1 << 2) | (1 << 3), 0, 14, 2, 0, True, 1.0, 0.05),
    ("scaled_2rb", 1, 24, 5, 2, 1, (1 << 2) | (1 << 9), 2, 10, 2, 1, True, 1.41, 0.1),
]


def bf16_grid(c):
    return (to_bf16(c.real.astype(np.float32)).astype(np.uint32)
            | (to_bf16(c.imag.astype(np.float32)).astype(np.uint32) << 16))


def make_grid(ports, nof_prb, noise, seed):
    rng = np.random.default_rng(seed)
    nsubc = 12 * nof_prb
    k = np.arange(nsubc)
    g = np.zeros((ports, 14, nsubc), np.complex64)
    for p in range(ports):
        h = (0.8 + 0.3j) * np.exp(-2j * np.pi * k * (3 + p) / 4096) * (1 + 0.2 * np.cos(k / 200 + p))
        for l in range(14):
            d = (rng.choice([-1, 1], nsubc) + 1j * rng.choice([-1, 1], nsubc)) * 0.7
            g[p, l] = h * np.exp(1j * 0.01 * l) * d + noise * (rng.normal(size=nsubc) + 1j * rng.normal(size=nsubc))
    return bf16_grid(g)


def case_args(case, seed=0):
    name, P, nprb, lo, cnt, L, mask, first, ns, fd, td, cfo, scaling, noise = case
    grid = make_grid(P, nprb, noise, seed)
    kw = dict(slot_index=3 + seed, type2=False, nof_layers=L, scrambling_id=77 + seed, n_scid=seed % 2,
              scaling=scaling, symbols_mask=mask, prb_lo=lo, prb_hi=lo + cnt, first_symbol=first, nof_symbols=ns,
              fd=fd, td=td, compensate_cfo=cfo, numerology=1)
    return grid, kw


def stale_estimates(grid_shape, nof_layers, seed=2):
    """Finite stale contents of an estimate buffer (the reference rotates them by the CFO phase)."""
    rng = np.random.default_rng(seed)
    shape = (grid_shape[0], nof_layers) + tuple(grid_shape[1:])
    return bf16_grid((rng.normal(size=shape) + 1j * rng.normal(size=shape)).astype(np.complex64))


def to_cf(u):
    u = np.asarray(u, np.uint32)
    return ((u & 0xFFFF) << 16).view(np.float32) + 1j * ((u >> 16) << 16).view(np.float32)


def assert_estimates_close(got, want, what=""):
    """bf16 estimates: equal up to the two bf16 roundings of a float-reassociated value (the estimate, then
    the CFO-rotated estimate): 2^-6 relative of the larger magnitude of the pair, plus 1e-6 absolute."""
    same = np.asarray(got, np.uint32) == np.asarray(want, np.uint32)
    a, b = to_cf(got), to_cf(want)
    with np.errstate(invalid="ignore", over="ignore"):
        tol = 2.0 ** -6 * np.maximum(np.abs(a), np.abs(b)) + 1e-6
        bad = ~same & ~(np.abs(a - b) <= tol)
    assert not bad.any(), "%s: %d of %d estimates differ (max %.3e)" % (what, bad.sum(), bad.size,
                                                                       np.abs(a - b)[bad].max())


def assert_stats_close(got, want, what=""):
    for p, (x, y) in enumerate(zip(got, want)):
        for k in ("noise_var", "epre", "rsrp", "snr"):
            assert np.isclose(float(x[k]), float(y[k]), rtol=2e-3, atol=1e-12), (what, p, k, x[k], y[k])
        tx, ty = float(x["time_alignment_s"]), float(y["time_alignment_s"])
        assert abs(tx - ty) <= 2e-3 * abs(ty) + 2e-9, (what, p, "ta", tx, ty)
        cx, cy = float(x["cfo_hz"]), float(y["cfo_hz"])
        assert (np.isnan(cx) and np.isnan(cy)) or np.isclose(cx, cy, rtol=2e-3, atol=1e-2), (what, p, "cfo", cx, cy)
