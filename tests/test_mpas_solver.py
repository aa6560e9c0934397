"""The MPAS vertical solver ("physics" mpas, oracle/mpas_oracle.c ora_mpas_*): the oracle
against a NumPy restatement of the same statements, and the property the restored
back substitution exists for -- the acoustic step's new rw_p solves the tridiagonal
system (a_tri, b_tri, c_tri) that vert_imp factors (dynamics_tasks.rg:566-591,
:1660-1677 with the quirks Q16-Q21 fixed)."""
import numpy as np
import pytest

import oracle as O

from helpers import make_state

EPSSM = 0.1
RESM = (1.0 - EPSSM) / (1.0 + EPSSM)


def rows(st, name, n):
    return st[name][:n]


def vert_imp_numpy(st, dts):
    """b_tri with cofwt(k-1) (Q16) and the LU recurrence of this call (Q17), on top of the
    reference coefficients (the oracle's ora_atm_compute_vert_imp_coefs)"""
    ref = st.copy()
    O.Oracle(ref).atm_compute_vert_imp_coefs(dts)
    n, L = st.nCells, st.L
    rdzw, cofrz = ref["rdzw"], ref["cofrz"]
    zz, cofwz, coftz, cofwt, cofwr = (rows(ref, f, n) for f in ("zz", "cofwz", "coftz", "cofwt", "cofwr"))
    a, c = rows(ref, "a_tri", n).copy(), rows(ref, "c_tri", n).copy()
    b = rows(ref, "b_tri", n).copy()
    alpha, gamma = rows(ref, "alpha_tri", n).copy(), rows(ref, "gamma_tri", n).copy()
    for k in range(1, L):
        b[:, k] = 1.0 + cofwz[:, k] * (coftz[:, k] * rdzw[k] * zz[:, k] + coftz[:, k] * rdzw[k - 1] * zz[:, k - 1]) - \
            coftz[:, k] * (cofwt[:, k] * rdzw[k] - cofwt[:, k - 1] * rdzw[k - 1]) + cofwr[:, k] * ((cofrz[k] - cofrz[k - 1]))
    gamma[:, 0] = 0.0
    for k in range(1, L):
        alpha[:, k] = 1.0 / (b[:, k] - a[:, k] * gamma[:, k - 1])
        gamma[:, k] = c[:, k] * alpha[:, k]
    return ref, a, b, c, alpha, gamma


@pytest.mark.parametrize("L", [5, 56])
def test_mpas_vert_imp_numpy(x1_2562, L):
    st = make_state(x1_2562, L, "random")
    got = st.copy()
    O.Oracle(got).mpas_vert_imp_coefs(240.0)
    ref, a, b, c, alpha, gamma = vert_imp_numpy(st, 240.0)
    n = st.nCells
    for name, v in (("a_tri", a), ("b_tri", b), ("c_tri", c), ("alpha_tri", alpha), ("gamma_tri", gamma)):
        assert np.array_equal(got[name][:n, :L], v[:, :L]), name
    for name in ("cofwz", "coftz", "cofwt", "cofwr", "cofrz"):
        assert np.array_equal(got[name], ref[name]), name


def acoustic_numpy(st, dts, small_step):
    """ora_mpas_acoustic_step restated over all cells at once (statement for statement);
    returns the new state and, per cell, the explicit right-hand side x and the solution
    z of the tridiagonal system before the Rayleigh damping"""
    s = st.copy()
    n, nE, L = st.nCells, st.nEdges, st.L
    rcv = 287.0 / (7.0 * 287.0 / 2.0 - 287.0)
    c2 = 7.0 * 287.0 / 2.0 * rcv
    g = 9.80616
    coe = s["cellsOnEdge"][:nE]
    c1, cc2 = coe[:, 0], coe[:, 1]
    rtp, rpp, zz, ex = s["rtheta_pp"], s["rho_pp"], s["zz"], s["exner"]
    spec_e = s["specZoneMaskEdge"][:nE, 0]
    invdc = s["invDcEdge"][:nE, 0]
    for k in range(L):
        if small_step != 0:
            pgrad = ((rtp[cc2, k] - rtp[c1, k]) * invdc) / (0.5 * (zz[cc2, k] + zz[c1, k]))
            pgrad = s["cqu"][:nE, k] * 0.5 * c2 * (ex[c1, k] + ex[cc2, k]) * pgrad
            pgrad = pgrad + 0.5 * s["zxu"][:nE, k] * g * (rpp[c1, k] + rpp[cc2, k])
            s["ru_p"][:nE, k] = s["ru_p"][:nE, k] + dts * (s["tend_u"][:nE, k] - (1.0 - spec_e) * pgrad)
            s["ruAvg"][:nE, k] = s["ruAvg"][:nE, k] + s["ru_p"][:nE, k]
        else:
            s["ru_p"][:nE, k] = dts * s["tend_u"][:nE, k]
            s["ruAvg"][:nE, k] = s["ru_p"][:nE, k]
    s["rtheta_pp_old"][:n, :L] = 0.0 if small_step == 0 else s["rtheta_pp"][:n, :L]
    if small_step == 0:
        s["wwAvg"][:n, :L + 1] = 0.0
        s["rw_p"][:n, :L + 1] = 0.0
        s["rho_pp"][:n, :L] = 0.0
        s["rtheta_pp"][:n, :L] = 0.0
    assert np.all(s["specZoneMaskCell"][:n, 0] == 0.0)  # (the specified zone branch is not exercised)
    rtp0, rpp0, rwp0 = s["rtheta_pp"][:n, :L].copy(), s["rho_pp"][:n, :L].copy(), s["rw_p"][:n, :L + 1].copy()
    rs, ts = np.zeros((n, L)), np.zeros((n, L))
    ne = s["nEdgesOnCell"][:n, 0]
    tm = s["theta_m"]
    for i in range(10):
        on = i < ne
        e = s["edgesOnCell"][:n, i]
        e1, e2 = s["cellsOnEdge"][e, 0], s["cellsOnEdge"][e, 1]
        for k in range(L):
            flux = s["edgesOnCellSign"][:n, i] * dts * s["dvEdge"][e, 0] * s["ru_p"][e, k] * s["invAreaCell"][:n, 0]
            rs[:, k] = np.where(on, rs[:, k] - flux, rs[:, k])
            ts[:, k] = np.where(on, ts[:, k] - flux * 0.5 * (tm[e2, k] + tm[e1, k]), ts[:, k])
    cofrz, rdzw, fzm, fzp = s["cofrz"], s["rdzw"], s["fzm"], s["fzp"]
    coftz = s["coftz"][:n]
    for k in range(L):
        rs[:, k] = rpp0[:, k] + dts * s["tend_rho"][:n, k] + rs[:, k] - cofrz[k] * RESM * (rwp0[:, k + 1] - rwp0[:, k])
        ts[:, k] = rtp0[:, k] + dts * s["tend_theta"][:n, k] + ts[:, k] - \
            RESM * rdzw[k] * (coftz[:, k + 1] * rwp0[:, k + 1] - coftz[:, k] * rwp0[:, k])
    ww = s["wwAvg"][:n]
    for k in range(1, L):
        ww[:, k] = ww[:, k] + 0.5 * (1.0 - EPSSM) * rwp0[:, k]
    z = rwp0.copy()
    zzc, cofwz, cofwr, cofwt = s["zz"][:n], s["cofwz"][:n], s["cofwr"][:n], s["cofwt"][:n]
    w = s["w"][:n]
    for k in range(1, L):
        z[:, k] = rwp0[:, k] + dts * w[:, k] - cofwz[:, k] * ((zzc[:, k] * ts[:, k] - zzc[:, k - 1] * ts[:, k - 1]) +
                                                            RESM * (zzc[:, k] * rtp0[:, k] - zzc[:, k - 1] * rtp0[:, k - 1])) - \
            cofwr[:, k] * ((rs[:, k] + rs[:, k - 1]) + RESM * (rpp0[:, k] + rpp0[:, k - 1])) + \
            cofwt[:, k] * (ts[:, k] + RESM * rtp0[:, k]) + cofwt[:, k - 1] * (ts[:, k - 1] + RESM * rtp0[:, k - 1])
    x = z.copy()
    a, alpha, gamma = s["a_tri"][:n], s["alpha_tri"][:n], s["gamma_tri"][:n]
    for k in range(1, L):
        z[:, k] = (z[:, k] - a[:, k] * z[:, k - 1]) * alpha[:, k]
    for k in range(L - 1, -1, -1):
        z[:, k] = z[:, k] - gamma[:, k] * z[:, k + 1]
    sol = z.copy()
    rws, rw, dss, rz = s["rw_save"][:n], s["rw"][:n], s["dss"][:n], s["rho_zz"][:n]
    for k in range(1, L):
        d = rws[:, k] - rw[:, k]
        z[:, k] = (z[:, k] + d - dts * dss[:, k] * (fzm[k] * zzc[:, k] + fzp[k] * zzc[:, k - 1]) *
                   (fzm[k] * rz[:, k] + fzp[k] * rz[:, k - 1]) * w[:, k]) / (1.0 + dts * dss[:, k]) - d
    for k in range(1, L):
        ww[:, k] = ww[:, k] + 0.5 * (1.0 + EPSSM) * z[:, k]
    s["rw_p"][:n, :L + 1] = z
    for k in range(L):
        s["rho_pp"][:n, k] = rs[:, k] - cofrz[k] * (z[:, k + 1] - z[:, k])
        s["rtheta_pp"][:n, k] = ts[:, k] - rdzw[k] * (coftz[:, k + 1] * z[:, k + 1] - coftz[:, k] * z[:, k])
    return s, x, sol


def mpas_state(x1_2562, L):
    from mpasdyn import mesh as M
    st = make_state(M.zero_based(x1_2562), L, "random")
    st["specZoneMaskCell"][...] = 0.0
    O.Oracle(st).mpas_vert_imp_coefs(240.0)
    return st


@pytest.mark.parametrize("L", [5, 56])
@pytest.mark.parametrize("small_step", [0, 1])
def test_mpas_acoustic_numpy(x1_2562, L, small_step):
    st = mpas_state(x1_2562, L)
    got = st.copy()
    O.Oracle(got).mpas_acoustic_step(240.0, small_step)
    want, _, _ = acoustic_numpy(st, 240.0, small_step)
    for name in ("ru_p", "ruAvg", "rw_p", "wwAvg", "rho_pp", "rtheta_pp", "rtheta_pp_old"):
        assert np.array_equal(got[name], want[name]), name


@pytest.mark.parametrize("L", [5, 56])
def test_mpas_acoustic_solves_tridiagonal(x1_2562, L):
    """the new rw_p (before the Rayleigh term) satisfies a z(k-1) + b z(k) + c z(k+1) = x(k)
    on the interior interfaces, z(0) and z(L) held: the back substitution (Q21) is what
    makes this hold, the reference's forward sweep alone does not"""
    st = mpas_state(x1_2562, L)
    _, x, z = acoustic_numpy(st, 240.0, 1)
    n = st.nCells
    a, b, c = st["a_tri"][:n], st["b_tri"][:n], st["c_tri"][:n]
    k = np.arange(1, L)
    res = a[:, k] * z[:, k - 1] + b[:, k] * z[:, k] + c[:, k] * z[:, k + 1] - x[:, k]
    scale = np.abs(b[:, k] * z[:, k]).max() + np.abs(x[:, k]).max()
    assert np.abs(res).max() <= 1e-12 * scale
    # the forward sweep alone (the reference's step) leaves a residual
    if L > 2:
        y = x.copy()
        for kk in range(1, L):
            y[:, kk] = (y[:, kk] - a[:, kk] * y[:, kk - 1]) * st["alpha_tri"][:n, kk]
        y[:, L] = z[:, L]
        r2 = a[:, k] * y[:, k - 1] + b[:, k] * y[:, k] + c[:, k] * y[:, k + 1] - x[:, k]
        assert np.abs(r2).max() > 1e3 * np.abs(res).max()


def test_mpas_srk3_runs(x1_2562):
    """the MPAS-form step runs and stays finite on the literal x1.2562 state (every other
    task is the reference's)"""
    from mpasdyn import mesh as M
    st = make_state(M.zero_based(x1_2562), 5, "random")
    O.Oracle(st).mpas_srk3(720.0, 1)
    for name in ("rw_p", "rho_pp", "rtheta_pp", "ru_p", "u", "w"):
        assert np.isfinite(st[name]).all(), name


@pytest.mark.parametrize("rk_step", [0, 2])
def test_mpas_recover_numpy(x1_2562, rk_step):
    """ora_mpas_recover against NumPy: ru = ru_save + ru_p (Q24), rw/wwAvg/w of the
    interior interfaces, w(L) = 0, exner = (zz rgas/p0 (rtheta_p + rtheta_base))^rcv, and
    the lower-boundary flux added to w(0) once per edge"""
    from mpasdyn import mesh as M
    st = make_state(M.zero_based(x1_2562), 5, "random")
    st["bdyMaskCell"][...] = 0
    got = st.copy()
    O.Oracle(got).mpas_recover(3, rk_step, 240.0)
    n, nE, L = st.nCells, st.nEdges, st.L
    rho_zz = st["rho_p_save"][:n, :L] + st["rho_pp"][:n, :L] + st["rho_base"][:n, :L]
    assert np.array_equal(got["rho_zz"][:n, :L], rho_zz)
    ru = st["ru_save"][:nE, :L] + st["ru_p"][:nE, :L]
    assert np.array_equal(got["ru"][:nE, :L], ru)
    c1, c2 = st["cellsOnEdge"][:nE, 0], st["cellsOnEdge"][:nE, 1]
    rzf = got["rho_zz"]
    assert np.array_equal(got["u"][:nE, :L], 2.0 * ru / (rzf[c1, :L] + rzf[c2, :L]))
    rw = st["rw_save"][:n, 1:L] + st["rw_p"][:n, 1:L]
    assert np.array_equal(got["rw"][:n, 1:L], rw) and np.array_equal(got["rw"][:n, 0], st["rw"][:n, 0])
    assert (got["w"][:n, L] == 0.0).all()
    if rk_step == 2:
        rtp = got["rtheta_p"][:n, :L]
        ex = (st["zz"][:n, :L] * (287.0 / 1.0e5) * (rtp + st["rtheta_base"][:n, :L])) ** (287.0 / (7.0 * 287.0 / 2.0 - 287.0))
        assert np.allclose(got["exner"][:n, :L], ex, rtol=1e-14, atol=0)
    # w(0): the boundary flux of every edge once, over the cf-weighted density
    cf1, cf2, cf3 = st["cf1"][0], st["cf2"][0], st["cf3"][0]
    ne = st["nEdgesOnCell"][:n, 0]
    w0 = np.zeros(n)
    for i in range(10):
        e = st["edgesOnCell"][:n, i]
        flux = cf1 * got["ru"][e, 0] + cf2 * got["ru"][e, 1] + cf3 * got["ru"][e, 2]
        term = st["edgesOnCell_sign"][:n, i] * (st["zb_cell"][:n, 0, i] + np.copysign(1.0, flux) * st["zb3_cell"][:n, 0, i]) * flux
        w0 = np.where(i < ne, w0 + term, w0)
    w0 = w0 / (cf1 * rzf[:n, 0] + cf2 * rzf[:n, 1] + cf3 * rzf[:n, 2])
    assert np.array_equal(got["w"][:n, 0], w0)
