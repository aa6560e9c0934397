"""Jablonowski-Williamson baroclinic-wave initial state, mpas mode.

Restates `init_atm_case_jw` (vertical_init/init_atm_cases.rg:24-743) for 0-based (mpas-mode)
meshes with its undefined behaviour fixed the way MPAS-A's init_atm_case_jw (MPAS-Model
src/core_init_atmosphere/mpas_init_atm_cases.F, not vendored) defines it:
  * the reference's 1-based loop bounds and swapped `cr[{k, i}]` indices (:251, :266, :419,
    :447) read as the cell-and-level points they mean; `kiteAreasOnVertex[vertexDegree]`
    (:100) as every kite;
  * the height coordinate from level 0: zw(k) = k dz, sh(k) = (k dz / zt)^1.5,
    ah(k) = 1 - cos(pi/2 k dz / zt)^6 (:163-171);
  * dry (qv = 0, :126-137), no rebalancing and no wind perturbation (u_pert = 0, :552-555),
    no Rayleigh layer (xnutr = 0, :140);
  * the 2-D latitude table (:257-360) is omitted: nothing after it reads its results.
Host-side, one-time (like the other precompute of build_state.py); the hot path then runs
from this state.  Fields written: the vertical grid (rdzw, rdzu, fzm, fzp, cf1..cf3), zgrid,
zz, zxu, dss, pressure_base, rho_base, rtheta_base, exner_base, exner, pressure_p,
rho_p, rho_zz, theta_m, rtheta_p, surface_pressure, u, ru, v, rw, w, zb_cell, zb3_cell,
rho, theta, fVertex, cqu (1: dry), and the mesh coefficients defc_a, defc_b,
coeffs_reconstruct (build_state.mpas_mesh_coefficients)."""
import numpy as np

from .build_state import OMEGA, SPHERE_RADIUS

RGAS = 287.0
CP = 3.5 * RGAS
GRAVITY = 9.80616
P0 = 1.0e5
U0, T0B, T0, DELTA_T, DTDZ, ETA_T = 35.0, 250.0, 288.0, 4.8e5, 0.005, 0.2
ZT = 45000.0


def vertical_grid(L):
    """:158-205: the JW height coordinate (0-based levels) -> dict of 1-D arrays"""
    dz = ZT / L
    k = np.arange(L + 1, dtype=np.float64)
    zw = k * dz
    sh = (k * dz / ZT) ** 1.5
    ah = 1.0 - np.cos(0.5 * np.pi * k * dz / ZT) ** 6
    dzw = zw[1:] - zw[:-1]
    dzu = np.zeros(L + 1)
    rdzu = np.zeros(L + 1)
    fzm = np.zeros(L + 1)
    fzp = np.zeros(L + 1)
    dzu[1:L] = 0.5 * (dzw[1:] + dzw[:-1])
    rdzu[1:L] = 1.0 / dzu[1:L]
    fzp[1:L] = 0.5 * dzw[1:] / dzu[1:L]
    fzm[1:L] = 0.5 * dzw[:-1] / dzu[1:L]
    rdzw = np.zeros(L + 1)
    rdzw[:L] = 1.0 / dzw
    cof1 = (2.0 * dzu[1] + dzu[2]) / (dzu[1] + dzu[2]) * dzw[0] / dzu[1]
    cof2 = dzu[1] / (dzu[1] + dzu[2]) * dzw[0] / dzu[2]
    return dict(zw=zw, sh=sh, ah=ah, dzw=dzw, dzu=dzu, rdzu=rdzu, rdzw=rdzw, fzm=fzm, fzp=fzp,
                cf1=fzp[1] + cof1, cf2=fzm[1] - cof1 - cof2, cf3=cof2)


def _jw_temperature(eta, phi):
    """:331-352: the JW temperature at eta levels (columns x levels), dry"""
    etav = (eta - 0.252) * np.pi / 2.0
    teta = T0 * eta ** (RGAS * DTDZ / GRAVITY)
    teta = np.where(eta >= ETA_T, teta, teta + DELTA_T * np.abs(ETA_T - eta) ** 5)
    s, c = np.sin(phi)[:, None], np.cos(phi)[:, None]
    return teta + 0.75 * eta * np.pi * U0 / RGAS * np.sin(etav) * np.sqrt(np.cos(etav)) * (
        (-2.0 * s ** 6 * (c ** 2 + 1.0 / 3.0) + 10.0 / 63.0) * 2.0 * U0 * np.cos(etav) ** 1.5
        + (1.6 * c ** 3 * (s ** 2 + 2.0 / 3.0) - np.pi / 4.0) * SPHERE_RADIUS * OMEGA)


def _hydrostatic(phi, pb, rb, zz, g, L):
    """:366-432 the hydrostatic iteration per column -> (pressure_p, rho_p, temperature):
    libmpasdyn's host threads (mpas_jw_hydrostatic, the same arithmetic in the same order)
    when the library is built, else the NumPy statement below"""
    try:
        from . import lib
        so = lib.load()
    except Exception:  # noqa: BLE001 -- host-side init only: NumPy computes the same values
        so = None
    nC = pb.shape[0]
    pb, rb, zz = (np.ascontiguousarray(x, dtype=np.float64) for x in (pb, rb, zz))
    if so is not None and nC > 0:
        import ctypes
        import os
        pp, rr, tt = np.empty_like(pb), np.empty_like(pb), np.empty_like(pb)
        vec = [np.ascontiguousarray(g[n], dtype=np.float64) for n in ("dzw", "dzu", "fzm", "fzp")]
        lat = np.ascontiguousarray(phi, dtype=np.float64)
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        rc = so.mpas_jw_hydrostatic(nC, L, ptr(lat), ptr(pb), ptr(rb), ptr(zz), *[ptr(v) for v in vec], ptr(pp),
                                    ptr(rr), ptr(tt), min(16, os.cpu_count() or 1))
        if rc != 0:
            raise RuntimeError(f"mpas_jw_hydrostatic failed ({rc})")
        return pp, rr, tt
    dzw, dzu, fzm, fzp = g["dzw"], g["dzu"], g["fzm"], g["fzp"]
    # level-major rows (the k loop is the slow axis), chunks of columns that stay in cache;
    # the recurrence ppi(k+1) = ppi(k) - t(k) is np.subtract.accumulate (sequential roundings)
    pp, rr, tt = np.zeros_like(pb), np.zeros_like(pb), np.zeros_like(pb)
    cdz = (dzu[1:L] * GRAVITY)[:, None]
    fzp1, fzm1 = fzp[1:L][:, None], fzm[1:L][:, None]
    CH = 16384
    for c0 in range(0, nC, CH):
        sl = slice(c0, min(c0 + CH, nC))
        pbT, rbT, zzT = np.ascontiguousarray(pb[sl].T), np.ascontiguousarray(rb[sl].T), np.ascontiguousarray(zz[sl].T)
        ppT = np.zeros_like(pbT)
        rrT = np.zeros_like(pbT)
        acc = np.empty_like(ppT)
        for _ in range(10):
            ttT = np.ascontiguousarray(_jw_temperature(((pbT + ppT) / P0).T, phi[sl]).T)
            for _ in range(25):
                rrT = (ppT / (RGAS * zzT) - rbT * (ttT - T0B)) / ttT
                acc[0] = P0 - 0.5 * dzw[0] * GRAVITY * (1.25 * (rrT[0] + rbT[0]) - 0.25 * (rrT[1] + rbT[1]))
                acc[0] -= pbT[0]
                acc[1:] = cdz * (rrT[:-1] * fzp1 + rrT[1:] * fzm1)
                ppi = np.subtract.accumulate(acc, axis=0)
                ppT = 0.2 * ppi + 0.8 * ppT
        pp[sl], rr[sl], tt[sl] = ppT.T, rrT.T, ttT.T
    return pp, rr, tt


def init_atm_case_jw(m, st, perturb=False):
    """Fill the JW state into HostState st (built by build_state(m, L, "physical") on a
    0-based mesh m).  perturb: add the test case's zonal-wind perturbation (1 m/s Gaussian
    of radius a/10 at 20E 40N, Jablonowski & Williamson 2006; MPAS-A's
    init_atm_case_jw with config_init_case = 2) -- the reference's own branch is dead
    (u_pert = 0, :552-555).  Returns st."""
    nC, nE, nV, L = m.nCells, m.nEdges, m.nVertices, st.L
    if L < 3:
        raise ValueError("the JW state needs nVertLevels >= 3 (cf1..cf3 use three levels)")
    cOE = np.asarray(m.cellsOnEdge)
    if cOE.min() != 0:
        raise ValueError("init_atm_case_jw expects a 0-based (mpas-mode) mesh: mesh.zero_based(m)")
    g = vertical_grid(L)
    for name in ("rdzw", "rdzu", "fzm", "fzp"):
        st[name] = g[name]
    for name in ("cf1", "cf2", "cf3"):
        a = np.zeros(L + 1)
        a[0] = g[name]
        st[name] = a
    phi = np.asarray(m.latCell, dtype=np.float64)
    etavs = (1.0 - 0.252) * np.pi / 2.0
    # :147-152 surface height of the JW geopotential
    s, c = np.sin(phi), np.cos(phi)
    hx = U0 / GRAVITY * np.cos(etavs) ** 1.5 * (
        (-2.0 * s ** 6 * (c ** 2 + 1.0 / 3.0) + 10.0 / 63.0) * U0 * np.cos(etavs) ** 1.5
        + (1.6 * c ** 3 * (s ** 2 + 2.0 / 3.0) - np.pi / 4.0) * SPHERE_RADIUS * OMEGA)
    zgrid = (1.0 - g["ah"])[None, :] * (g["sh"][None, :] * (ZT - hx[:, None]) + hx[:, None]) + \
        (g["ah"] * g["sh"] * ZT)[None, :]
    zz = (g["zw"][1:] - g["zw"][:-1])[None, :] / (zgrid[:, 1:] - zgrid[:, :-1])
    st["zgrid"][:nC] = zgrid
    st["zz"][:nC, :L] = zz
    dc = st["dcEdge"][:nE, 0]
    c1, c2 = cOE[:, 0], cOE[:, 1]
    st["zxu"][:nE, :L] = 0.5 * (zgrid[c2, :L] - zgrid[c1, :L] + zgrid[c2, 1:] - zgrid[c1, 1:]) / dc[:, None]
    st["dss"][:nC] = 0.0
    # :366-432 base state and the hydrostatic iteration, per column
    ztemp = 0.5 * (zgrid[:, 1:] + zgrid[:, :-1])
    pb = P0 * np.exp(-GRAVITY * ztemp / (RGAS * T0B))
    ex_b = (pb / P0) ** (RGAS / CP)
    rb = pb / (RGAS * T0B * zz)
    tb = T0B / ex_b
    pp, rr, tt = _hydrostatic(phi, pb, rb, zz, g, L)
    dzw, dzu, fzm, fzp = g["dzw"], g["dzu"], g["fzm"], g["fzp"]
    exner = ((pb + pp) / P0) ** (RGAS / CP)
    theta_m = tt / exner
    rho_zz = rb + rr
    st["pressure_base"][:nC, :L] = pb
    st["rho_base"][:nC, :L] = rb
    st["rtheta_base"][:nC, :L] = rb * tb
    st["exner_base"][:nC, :L] = ex_b
    st["exner"][:nC, :L] = exner
    st["pressure_p"][:nC, :L] = pp
    st["rho_p"][:nC, :L] = rr
    st["rho_zz"][:nC, :L] = rho_zz
    st["theta_m"][:nC, :L] = theta_m
    st["rtheta_p"][:nC, :L] = theta_m * rr + rb * (theta_m - tb)
    st["surface_pressure"][:nC, 0] = 0.5 * dzw[0] * GRAVITY * (
        1.25 * (rr[:, 0] + rb[:, 0]) - 0.25 * (rr[:, 1] + rb[:, 1])) + pp[:, 0] + pb[:, 0]
    # :513-569 the zonal jet through the edges' vertex latitudes (no perturbation)
    vOE = np.asarray(m.verticesOnEdge)
    lat1, lat2 = np.asarray(m.latVertex)[vOE[:, 0]], np.asarray(m.latVertex)[vOE[:, 1]]
    dv = st["dvEdge"][:nE, 0]
    flux = (0.5 * (lat2 - lat1) - 0.125 * (np.sin(4.0 * lat2) - np.sin(4.0 * lat1))) * SPHERE_RADIUS / dv
    ptot = pb + pp
    ev = (0.5 * (ptot[c1] + ptot[c2]) / P0 - 0.252) * np.pi / 2.0
    u = U0 * flux[:, None] * np.cos(ev) ** 1.5
    if perturb:
        lat_e, lon_e = np.asarray(m.latEdge), np.asarray(m.lonEdge)
        lat_c, lon_c = 2.0 * np.pi / 9.0, np.pi / 9.0
        r = np.arccos(np.clip(np.sin(lat_c) * np.sin(lat_e) + np.cos(lat_c) * np.cos(lat_e) * np.cos(lon_e - lon_c),
                              -1.0, 1.0))
        u = u + (1.0 * np.exp(-(r * 10.0) ** 2) * np.cos(np.asarray(m.angleEdge)))[:, None]
    st["u"][:nE, :L] = u
    st["ru"][:nE, :L] = 0.5 * (rho_zz[c1] + rho_zz[c2]) * u
    st["fVertex"][:nV, 0] = 2.0 * OMEGA * np.sin(np.asarray(m.latVertex))
    # :580-600 zb / zb3 of the terrain-following coordinate, seen from each cell (the
    # per-cell copies atm_compute_signs makes, dynamics_tasks.rg:87-107)
    area = 1.0 / st["invAreaCell"][:nC, 0]
    z_edge = 0.5 * (zgrid[c1] + zgrid[c2])  # (nE, L+1)
    zb = np.stack([(z_edge - zgrid[c1]) * (dv / area[c1])[:, None],
                   (z_edge - zgrid[c2]) * (dv / area[c2])[:, None]], axis=2)  # (nE, L+1, 2)
    eoc = st["edgesOnCell"][:nC]
    ne = st["nEdgesOnCell"][:nC, 0]
    cells = np.arange(nC)
    zbc = np.zeros((nC, L + 1, 10))
    for i in range(eoc.shape[1]):
        on = i < ne
        e = np.where(on, eoc[:, i], 0)
        side = np.where(cOE[e, 0] == cells, 0, 1)
        zbc[:, :, i] = np.where(on[:, None], zb[e, :, :][np.arange(nC), :, side], 0.0)
    st["zb_cell"][:nC] = zbc
    st["zb3_cell"][:nC] = 0.0
    # :602-618 rw from the terrain slope, w
    ru = st["ru"][:nE]
    rw = np.zeros((nC, L + 1))
    zzf = st["zz"][:nC]
    for k in range(1, L):
        fl = fzm[k] * ru[:, k] + fzp[k] * ru[:, k - 1]
        np.add.at(rw[:, k], c2, (fzm[k] * zzf[c2, k] + fzp[k] * zzf[c2, k - 1]) * zb[:, k, 1] * fl)
        np.subtract.at(rw[:, k], c1, (fzm[k] * zzf[c1, k] + fzp[k] * zzf[c1, k - 1]) * zb[:, k, 0] * fl)
    st["rw"][:nC] = rw
    w = np.zeros((nC, L + 1))
    for k in range(1, L):
        w[:, k] = rw[:, k] / (fzp[k] * rho_zz[:, k - 1] + fzm[k] * rho_zz[:, k])
    st["w"][:nC] = w
    # :620-636 v from weightsOnEdge over edgesOnEdge
    eoe = st["edgesOnEdge_ECP"][:nE]
    woe = st["weightsOnEdge"][:nE]
    neoe = st["nEdgesOnEdge"][:nE, 0]
    v = np.zeros((nE, L + 1))
    for i in range(int(neoe.max()) if nE else 0):
        on = i < neoe
        v += np.where(on[:, None], woe[:, i, None] * st["u"][np.where(on, eoe[:, i], 0)], 0.0)
    st["v"][:nE] = v
    st["rho"][:nC, :L] = rho_zz * zz
    st["theta"][:nC, :L] = theta_m
    st["cqu"][:nE, :L] = 1.0
    # the mesh coefficients MPAS-A's init computes and the reference never writes (Q2):
    # Smagorinsky deformation weights and the cell-centre velocity reconstruction
    from .build_state import mpas_mesh_coefficients
    mpas_mesh_coefficients(m, st)
    return st


# the 3-D fields init_atm_case_jw writes (the rest of the state stays 0)
JW_FIELDS = ("zgrid", "zz", "zxu", "dss", "pressure_base", "rho_base", "rtheta_base", "exner_base", "exner",
             "pressure_p", "rho_p", "rho_zz", "theta_m", "rtheta_p", "surface_pressure", "u", "ru", "v", "rw", "w",
             "zb_cell", "zb3_cell", "rho", "theta", "cqu", "coeffs_reconstruct")


def jw_state(m0, L, perturb=False, subset=False, extra_names=()):
    """build_state(physical) + init_atm_case_jw for a 0-based mesh m0.  subset: a HostState
    with only the mesh fields, JW_FIELDS and `extra_names` (large meshes; the others are the
    zeros a fresh context holds)"""
    from .build_state import build_state
    if subset:
        st = build_state(m0, L, "physical", vertical=False, mesh_only=True, extra_names=JW_FIELDS + tuple(extra_names))
    else:
        st = build_state(m0, L, "physical", vertical=False)
    return init_atm_case_jw(m0, st, perturb=perturb)
