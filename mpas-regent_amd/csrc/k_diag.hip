// k_diag.hip -- the operators the reference defines next to the RK3 loop but does not run
// inside it, for gfx950:
//   atm_recover_large_step_variables_work  dynamics_tasks.rg:1766-1872 (commented out of
//                                          atm_srk3, rk_timestep.rg:460, Q7)
//   mpas_reconstruct_2d                    dynamics_tasks.rg:1893-1948 (atm_core_init,
//                                          atm_core.rg:33; commented out of atm_srk3 :487)
//   summarize_timestep                     rk_timestep.rg:29-359 (called at :492 with every
//                                          print flag false: a no-op on the path)
// Same column mapping as the rest of the library: one wavefront per cell/edge column.
#include "mpas_dev.h"
#include "mpas_halo.h"

namespace mpas {

// ---------------------------------------------------------------- recover_large_step
struct RecK {
    double invNs, dt, rgas_p0, rgas, rcv;
    int rk_step;
    double coef_divdamp;  // (DAMP: the stage's last atm_divergence_damping_3d, option mdamp)
};

// :1788-1820 (the loop over cells and levels 0..nVertLevels-1), and the "garbage cell"
// rho_zz = 1.0 of :1790-1792 (our zero slot).  MPASV (option physics = 1, oracle
// ora_mpas_recover): w(0) = 0, w(L) = 0, rw/wwAvg/w of the interior interfaces only,
// exner = (zz rgas/p0 (rtheta_p + rtheta_base))^rcv
// the MPAS form of k_recover_cells for one lane, every level stored: levels 1..L-1 the
// recovered values (:1800-1820 with Q24 fixed), w(0) = w(L) = 0, rw / wwAvg at levels 0 and L
// the values they hold (wwAvg: just loaded; rw: its keep tails), every other field at level L
// its keep tail, the padding levels 0.0 (mpas_dev.h keep tails)
// NAVG (atm_srk3 option ntu, a stage before the last): wwAvg is dead -- the next stage's first
// acoustic substep sets it (:1625-1630) before any task reads it -- and is neither read nor stored
template <int LP, bool NAVG = false>
__device__ __forceinline__ void recover_cells_mpas(const DevState& S, const RecK& a, int c, int k, double zz,
                                                   double zz_m, double fzm, double fzp, double rps, double rpp,
                                                   double rb, double ww, double rws, double rwp, double rtps,
                                                   double rtpp, double rtb, double rtd, double exb) {
    const int L = S.L;
    auto kL = [&](int f) { return keepv<LP>(S, f, KC, c); };
    const double rho_p = rps + rpp;
    const double rho_zz = rho_p + rb;
    double wwAvg = ww;
    wwAvg *= a.invNs;
    wwAvg += rws;
    const double rw = rws + rwp;
    const double w = rw / (fzm * zz + fzp * zz_m);
    // (NAVG, a stage before the last: rho_p is dead too -- only setup reads it, and the last stage's
    // recover rewrites it first; rtheta_p after stage 1 likewise -- vert_imp, its reader, runs at the
    // start of stage 1 only)
    if (!NAVG) colk(fw(S, F_rho_p), c) = KEEPW(rho_p, kL(F_rho_p));
    colk(fw(S, F_rho_zz), c) = KEEPW(rho_zz, kL(F_rho_zz));
    if (!NAVG) colk(fw(S, F_wwAvg), c) = (k == 0 || k == L) ? ww : PADW(wwAvg);
    colk(fw(S, F_rw), c) = KEEPW0(rw, keepv<LP>(S, F_rw, KC, c, true), kL(F_rw));
    colk(fw(S, F_w), c) = (k == 0 || k >= L) ? 0.0 : w;
    if (a.rk_step == 2) {
        const double rtheta_p = rtps + rtpp - a.dt * rho_zz * rtd;
        colk(fw(S, F_rtheta_p), c) = KEEPW(rtheta_p, kL(F_rtheta_p));
        colk(fw(S, F_theta_m), c) = KEEPW((rtheta_p + rtb) / rho_zz, kL(F_theta_m));
        const double exner = pow(zz * a.rgas_p0 * (rtheta_p + rtb), a.rcv);
        colk(fw(S, F_exner), c) = KEEPW(exner, kL(F_exner));
        colk(fw(S, F_pressure_p), c) = KEEPW(zz * a.rgas * (exner * rtheta_p + rtb * (exner - exb)), kL(F_pressure_p));
    } else {
        const double rtheta_p = rtps + rtpp;
        if (!(NAVG && a.rk_step == 1)) colk(fw(S, F_rtheta_p), c) = KEEPW(rtheta_p, kL(F_rtheta_p));
        colk(fw(S, F_theta_m), c) = KEEPW((rtheta_p + rtb) / rho_zz, kL(F_theta_m));
    }
}

template <int LP, bool MPASV, bool NAVG = false>
__global__ __launch_bounds__(256) void k_recover_cells(DevState S, RecK a) {
    static_assert(!NAVG || MPASV, "the dead averages: the MPAS forms (the reference semantics never recover)");
    ColMap<LP> m(S, KC);
    const int L = S.L, k = m.k, c = m.ent;
    if (m.blk == 0 && (int)threadIdx.x < L) fw(S, F_rho_zz)[(size_t)S.nCells * LP + lpos(LP, threadIdx.x)] = 1.0;
    if (c >= S.nCO) return;
    const bool kl = k < L;
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double zz = col_rd<LP>(fd(S, F_zz), c, k, L), zz_m = lvl_dn<LP>(zz, k);
    const double rps = colk(fd(S, F_rho_p_save), c), rpp = colk(fd(S, F_rho_pp), c), rb = colk(fd(S, F_rho_base), c);
    const double ww = NAVG ? 0.0 : colk(fd(S, F_wwAvg), c), rws = colk(fd(S, F_rw_save), c), rwp = colk(fd(S, F_rw_p), c);
    const double rtps = colk(fd(S, F_rtheta_p_save), c), rtpp = colk(fd(S, F_rtheta_pp), c);
    const double rtb = colk(fd(S, F_rtheta_base), c);
    const double rtd = a.rk_step == 2 ? colk(fd(S, F_rt_diabatic_tend), c) : 0.0;
    const double exb = a.rk_step == 2 ? colk(fd(S, F_exner_base), c) : 0.0;
    if (MPASV && k == L) keep_put<LP>(S, F_w, KC, c, 0.0);  // (w's level L changes: its keep tail too)
    if (MPASV) {  // every level of every column written (level L / 0 with their kept values, the
                  // padding with zeros: keep tails, mpas_dev.h) -- no partially written line
        recover_cells_mpas<LP, NAVG>(S, a, c, k, zz, zz_m, fzm, fzp, rps, rpp, rb, ww, rws, rwp, rtps, rtpp, rtb, rtd, exb);
        return;
    }
    if (!kl) return;
    const double rho_p = rps + rpp;
    const double rho_zz = rho_p + rb;
    double wwAvg = ww;
    wwAvg *= a.invNs;
    wwAvg += rws;
    const double rw = rws + rwp;
    const double w = rw / (fzm * zz + fzp * zz_m);  // (:1805 sets w = 0.0 first)
    colk(fw(S, F_rho_p), c) = rho_p;
    colk(fw(S, F_rho_zz), c) = rho_zz;
    if (!MPASV || k > 0) {
        colk(fw(S, F_wwAvg), c) = wwAvg;
        colk(fw(S, F_rw), c) = rw;
        if (k == 0) keep_put0<LP>(S, F_rw, KC, c, rw);  // (rw's level 0 changes: its keep tail too)
    }
    colk(fw(S, F_w), c) = (MPASV && k == 0) ? 0.0 : w;
    if (a.rk_step == 2) {
        const double rtheta_p = rtps + rtpp - a.dt * rho_zz * rtd;
        colk(fw(S, F_rtheta_p), c) = rtheta_p;
        colk(fw(S, F_theta_m), c) = (rtheta_p + rtb) / rho_zz;
        const double exner = MPASV ? pow(zz * a.rgas_p0 * (rtheta_p + rtb), a.rcv)
                                   : zz * a.rgas_p0 * pow((rtheta_p + rtb), a.rcv);  // Q24 literal
        colk(fw(S, F_exner), c) = exner;
        colk(fw(S, F_pressure_p), c) = zz * a.rgas * (exner * rtheta_p + rtb * (exner - exb));
    } else {
        const double rtheta_p = rtps + rtpp;
        colk(fw(S, F_rtheta_p), c) = rtheta_p;
        colk(fw(S, F_theta_m), c) = (rtheta_p + rtb) / rho_zz;
    }
}

// :1830-1837: ruAvg, ru (Q24: ru_save * ru_p; MPASV: ru_save + ru_p), u from the new rho_zz
// NAVG (see recover_cells_mpas): ruAvg is dead -- the next stage's first substep sets it
// (k_acoustic_ru FIRST) -- and is neither read nor stored
// DAMP (option mdamp, the MPAS forms): the stage's last atm_divergence_damping_3d (:1742-1762) applied
// here to the ru_p this kernel reads -- divdamp_body's expression on the same values (rtheta_pp,
// rtheta_pp_old, theta_m of the acoustic step: this launch runs before k_recover_cells, which rewrites
// theta_m; OLD0: rtheta_pp_old = 0 after a stage's first substep), so the same bits -- and rho_zz of
// the edge's cells formed as k_recover_cells forms it ((rho_p_save + rho_pp) + rho_base; the garbage
// cell's 1.0, :1790-1792).  The damped ru_p is stored unless NAVG (a stage before the last: the next
// stage's first substep sets ru_p from tend_u)
template <int LP, bool MPASV, bool NAVG = false, bool DAMP = false, bool OLD0 = false>
__global__ __launch_bounds__(256) void k_recover_edges(DevState S, RecK a) {
    static_assert(!NAVG || MPASV, "the dead averages: the MPAS forms");
    static_assert(!DAMP || MPASV, "the damping in recover: the MPAS forms");
    ColMap<LP> m(S, KE);
    const int L = S.L, k = m.k, e = m.ent;
    if (e >= S.nEO || (!MPASV && k >= L)) return;
    const int cell1 = fi(S, F_cellsOnEdge)[(size_t)e * 2], cell2 = fi(S, F_cellsOnEdge)[(size_t)e * 2 + 1];
    double rz1, rz2, rup;
    const double ra = NAVG ? 0.0 : colk(fd(S, F_ruAvg), e), rus = colk(fd(S, F_ru_save), e);
    if constexpr (DAMP) {
        double ps1, ps2, pp1, pp2, rb1, rb2, r1, r2, ro1 = 0.0, ro2 = 0.0, t1, t2;
        gather2s<LP>(fd(S, F_rho_p_save), cell1, cell2, k, ps1, ps2);
        gather2s<LP>(fd(S, F_rho_pp), cell1, cell2, k, pp1, pp2);
        gather2s<LP>(fd(S, F_rho_base), cell1, cell2, k, rb1, rb2);
        gather2s<LP>(fd(S, F_rtheta_pp), cell1, cell2, k, r1, r2);
        if (!OLD0) gather2s<LP>(fd(S, F_rtheta_pp_old), cell1, cell2, k, ro1, ro2);
        gather2s<LP>(fd(S, F_theta_m), cell1, cell2, k, t1, t2);
        const int sh1 = fi(S, F_isShared)[cell1], sh2 = fi(S, F_isShared)[cell2];
        const double spec = fd(S, F_specZoneMaskEdge)[e];
        const double ru0 = colk(fd(S, F_ru_p), e);
        const double rp1 = ps1 + pp1, rp2 = ps2 + pp2;
        rz1 = (cell1 == S.nCells) ? 1.0 : rp1 + rb1;
        rz2 = (cell2 == S.nCells) ? 1.0 : rp2 + rb2;
        const double divCell1 = -(r1 - ro1), divCell2 = -(r2 - ro2);
        rup = (k < L && !(sh1 && sh2)) ? ru0 + a.coef_divdamp * (divCell2 - divCell1) * (1.0 - spec) / (t1 + t2) : ru0;
        if (!NAVG) colk(fw(S, F_ru_p), e) = k < L ? rup : PADW(ru0);
    } else {
        const double* rz = fd(S, F_rho_zz);
        rz1 = colk(rz, cell1);
        rz2 = colk(rz, cell2);
        rup = colk(fd(S, F_ru_p), e);
    }
    double ruAvg = ra;
    ruAvg *= a.invNs;
    ruAvg += rus;
    const double ru = MPASV ? rus + rup : rus * rup;
    if (MPASV) {  // (every level written: level L with the values it holds -- ruAvg just loaded, ru / u
                  // their keep tails -- the padding with zeros; mpas_dev.h keep tails)
        if (!NAVG) colk(fw(S, F_ruAvg), e) = KEEPW(ruAvg, ra);
        colk(fw(S, F_ru), e) = KEEPW(ru, keepv<LP>(S, F_ru, KE, e));
        colk(fw(S, F_u), e) = KEEPW(2 * ru / (rz1 + rz2), keepv<LP>(S, F_u, KE, e));
        return;
    }
    colk(fw(S, F_ruAvg), e) = ruAvg;
    colk(fw(S, F_ru), e) = ru;
    colk(fw(S, F_u), e) = 2 * ru / (rz1 + rz2);
}

// One slot's two terms: a = level-0 flux term (lanes 0..2 of ru, level 0 of zb/zb3), b = this
// level's term.
template <int LP, bool MPASV>
__device__ __forceinline__ void recover_w_slot(double r, double z, double z3, double sg, int k, double fzm,
                                               double fzp, double cf1, double cf2, double cf3, double& a,
                                               double& b) {
    const double r_m = lvl_dn<LP>(r, k);
    const double r0 = __shfl(r, 0, LP), r1 = __shfl(r, 1, LP), r2 = __shfl(r, 2, LP);
    const double zb0 = __shfl(z, 0, LP), zb30 = __shfl(z3, 0, LP);
    const double flux = (cf1 * r0 + cf2 * r1 + cf3 * r2);
    a = sg * (zb0 + copysign(1.0, flux) * zb30) * flux;
    const double flux2 = MPASV ? fzm * r + fzp * r_m : fzm * r * (fzp * r_m);  // (ref: Q24 literal)
    b = sg * (z + copysign(1.0, flux2) * z3) * flux2;
}

// :1839-1870: the w recovery from (rho*omega)_p over the cell's edges, then the division.
// The level-0 term (cf1..cf3 flux) is added to w(cell, 0) at every one of the nVertLevels
// level iterations of the cell; lane 0 replays that sequence in the reference's order.
// MPASV: the level-0 term once per edge, flux2 = fzm ru(k) + fzp ru(k-1) (Q24).
// (rz, w: rho_zz and w of the column as k_recover_cells stored them, read back)
template <int LP, bool MPASV>
__device__ __forceinline__ void recover_w_col(const DevState& S, int c, int k, double rz, double w) {
    const int L = S.L;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* sgn = fd(S, F_edgesOnCell_sign) + (size_t)c * 10;
    int e_[NF];
    double sg_[NF];
    row_ld(eoc, e_);
    row_ld(sgn, sg_);
    const double *ru = fd(S, F_ru), *zb = fd(S, F_zb_cell), *zb3 = fd(S, F_zb3_cell);
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double cf1 = fd(S, F_cf1)[0], cf2 = fd(S, F_cf2)[0], cf3 = fd(S, F_cf3)[0];
    const double w_in = w;  // (level L: stored back as loaded -- the column's lines written whole)
    const double rz_m = lvl_dn<LP>(rz, k), rz1 = __shfl(rz, 1, LP), rz2 = __shfl(rz, 2, LP);
    // the first NF slots: loads issued unconditionally, in pairs (every lane is active);
    // slots NF..9 (cells with more edges) one at a time under wave-uniform guards
    double r_[NF], z_[NF], z3_[NF], a_[10], b_[10];
#pragma unroll
    for (int i = 0; i < NF; i += 2) {
        gather2s<LP>(ru, e_[i], e_[i + 1], k, r_[i], r_[i + 1]);
        gather2<LP>(zb, c * 10 + i, zb3, c * 10 + i, k, z_[i], z3_[i]);
        gather2<LP>(zb, c * 10 + i + 1, zb3, c * 10 + i + 1, k, z_[i + 1], z3_[i + 1]);
    }
#pragma unroll
    for (int i = 0; i < NF; i++)
        recover_w_slot<LP, MPASV>(r_[i], z_[i], z3_[i], sg_[i], k, fzm, fzp, cf1, cf2, cf3, a_[i], b_[i]);
#pragma unroll
    for (int i = NF; i < 10; i++) {
        a_[i] = b_[i] = 0.0;
        if (i < ne) {
            const double r = colk(ru, eoc[i]), z = colk(zb, c * 10 + i), z3 = colk(zb3, c * 10 + i);
            recover_w_slot<LP, MPASV>(r, z, z3, sgn[i], k, fzm, fzp, cf1, cf2, cf3, a_[i], b_[i]);
        }
    }
    if (k == 0 && MPASV) {
#pragma unroll
        for (int i = 0; i < 10; i++)
            if (i < ne) w = w + a_[i];
        w = w / (cf1 * rz + cf2 * rz1 + cf3 * rz2);
    } else if (k == 0) {
#pragma unroll
        for (int i = 0; i < 10; i++)  // level iteration 0
            if (i < ne) {
                w += a_[i];
                w += b_[i];
            }
        for (int kk = 1; kk < L; kk++)  // level iterations 1..nVertLevels-1
#pragma unroll
            for (int i = 0; i < 10; i++)
                if (i < ne) w += a_[i];
        w /= (cf1 * rz + cf2 * rz1 + cf3 * rz2);
    } else {
#pragma unroll
        for (int i = 0; i < 10; i++)
            if (i < ne) w += b_[i];
        w /= (fzm * rz + fzp * rz_m);
    }
    colk(fw(S, F_w), c) = k < L ? w : PADW(w_in);
}
template <int LP, bool MPASV>
__global__ __launch_bounds__(256) void k_recover_w(DevState S) {
    ColMap<LP> m(S, KC);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO) return;
    if (fi(S, F_bdyMaskCell)[c] > kRelaxZone) return;
    double rz, w;
    col_rd2<LP>(fd(S, F_rho_zz), fd(S, F_w), c, k, L, rz, w);
    recover_w_col<LP, MPASV>(S, c, k, rz, w);
}

// (option mdamp: the cell part and the w recovery in one kernel -- ru is ready once the edge kernel
// runs first -- was measured slower, 1.58 -> 1.83 ms for the two stage-0/1 recovers: the fused
// kernel's registers halve its occupancy; profiles/r06/mdamp/kbench_recover_cw_tried.json)

template <int LP>
static hipError_t recover_lp(const DevState& S, hipStream_t st, int ns, int rk_step, double dt, int navg,
                             int damp, double damp_dts) {
    RecK a;
    a.invNs = 1 / (double)ns;
    a.dt = dt;
    a.rgas = kRgas;
    a.rgas_p0 = kRgas / 100000;
    a.rcv = kRgas / (kCp - kRgas);
    a.rk_step = rk_step;
    a.coef_divdamp = damp ? divdamp_coef(damp_dts) : 0.0;
    const int nCB = col_blocks<LP>(S, KC);
    const bool na = navg && S.physics;  // (option ntu: the averages of a stage before the last are dead)
    if (damp && !S.physics) return hipErrorInvalidValue;
    if (damp) {  // (option mdamp) the edges first, with the stage's last damping; then the cells and w
        auto kd = [&](const DevState& X) {
            const int nb = col_blocks<LP>(X, KE);
            if (!nb) return;
            if (na && damp == 2) k_recover_edges<LP, true, true, true, true><<<nb, 256, 0, st>>>(X, a);
            else if (na) k_recover_edges<LP, true, true, true, false><<<nb, 256, 0, st>>>(X, a);
            else if (damp == 2) k_recover_edges<LP, true, false, true, true><<<nb, 256, 0, st>>>(X, a);
            else k_recover_edges<LP, true, false, true, false><<<nb, 256, 0, st>>>(X, a);
        };
        if (damp == 2) HALO_RUN(S, st, kd, F_rho_p_save, F_rho_pp, F_rho_base, F_rtheta_pp, F_theta_m);
        else HALO_RUN(S, st, kd, F_rho_p_save, F_rho_pp, F_rho_base, F_rtheta_pp, F_rtheta_pp_old, F_theta_m);
        HALO_WROTE(S, F_ru, F_u);
        if (!na) HALO_WROTE(S, F_ruAvg, F_ru_p);
        if (nCB && na) k_recover_cells<LP, true, true><<<nCB, 256, 0, st>>>(S, a);
        else if (nCB) k_recover_cells<LP, true><<<nCB, 256, 0, st>>>(S, a);
        HALO_WROTE(S, F_rho_zz, F_rw, F_w, F_theta_m, F_exner, F_pressure_p);
        if (!na) HALO_WROTE(S, F_wwAvg, F_rho_p);
        if (!(na && rk_step == 1)) HALO_WROTE(S, F_rtheta_p);
        auto kw = [&](const DevState& X) {
            const int nb = col_blocks<LP>(X, KC);
            if (nb) k_recover_w<LP, true><<<nb, 256, 0, st>>>(X);
        };
        HALO_RUN(S, st, kw, F_ru);
        HALO_WROTE(S, F_w);
        return hipGetLastError();
    }
    if (nCB && na) k_recover_cells<LP, true, true><<<nCB, 256, 0, st>>>(S, a);
    else if (nCB && S.physics) k_recover_cells<LP, true><<<nCB, 256, 0, st>>>(S, a);
    else if (nCB) k_recover_cells<LP, false><<<nCB, 256, 0, st>>>(S, a);
    HALO_WROTE(S, F_rho_zz, F_rw, F_w, F_theta_m, F_exner, F_pressure_p);
    if (!na) HALO_WROTE(S, F_wwAvg, F_rho_p);
    if (!(na && rk_step == 1)) HALO_WROTE(S, F_rtheta_p);
    auto ke = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KE);
        if (nb && na) k_recover_edges<LP, true, true><<<nb, 256, 0, st>>>(X, a);
        else if (nb && X.physics) k_recover_edges<LP, true><<<nb, 256, 0, st>>>(X, a);
        else if (nb) k_recover_edges<LP, false><<<nb, 256, 0, st>>>(X, a);
    };
    HALO_RUN(S, st, ke, F_rho_zz);
    HALO_WROTE(S, F_ru, F_u);
    if (!na) HALO_WROTE(S, F_ruAvg);
    auto kw = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (nb && X.physics) k_recover_w<LP, true><<<nb, 256, 0, st>>>(X);
        else if (nb) k_recover_w<LP, false><<<nb, 256, 0, st>>>(X);
    };
    HALO_RUN(S, st, kw, F_ru);
    HALO_WROTE(S, F_w);
    return hipGetLastError();
}
hipError_t launch_recover_large_step(const DevState& S, hipStream_t st, int ns, int rk_step, double dt, int navg,
                                     int damp, double damp_dts) {
    MPAS_LP_DISPATCH(S.LP, recover_lp, S, st, ns, rk_step, dt, navg, damp, damp_dts);
}

// ---------------------------------------------------------------- damping coefficients
// atm_compute_damping_coefs (dynamics_tasks.rg:274-300; atm_core_init, atm_core.rg:41):
// dss of levels 0..L-1 from the layer's mid height; pow(x, 2.0) as x * x
template <int LP>
__global__ __launch_bounds__(256) void k_damping(DevState S, double zd, double xnutr, double pii) {
    ColMap<LP> m(S, KC);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO) return;
    const double zg = col_rd<LP>(fd(S, F_zgrid), c, k, L);
    const double zg_up = lvl_up<LP>(zg, k), zt = __shfl(zg, L, LP);
    const double md = fd(S, F_meshDensity)[c];
    double dss = 0.0;
    const double z = 0.5 * (zg + zg_up);
    if (z > zd) {
        const double sn = sin(0.5 * pii * (z - zd) / (zt - zd));
        dss = xnutr * (sn * sn);
        dss /= pow(md, (0.25 * 1.0));
    }
    if (k < L || k > L) colk(fw(S, F_dss), c) = PADW(dss);
}
template <int LP>
static hipError_t damping_lp(const DevState& S, hipStream_t st, double zd, double xnutr) {
    const int nb = col_blocks<LP>(S, KC);
    if (nb) k_damping<LP><<<nb, 256, 0, st>>>(S, zd, xnutr, acos(-1.0));
    HALO_WROTE(S, F_dss);
    return hipGetLastError();
}
hipError_t launch_damping_coefs(const DevState& S, hipStream_t st, double zd, double xnutr) {
    MPAS_LP_DISPATCH(S.LP, damping_lp, S, st, zd, xnutr);
}

// ---------------------------------------------------------------- init_coupled_diagnostics
// atm_init_coupled_diagnostics (dynamics_tasks.rg:651-726; atm_core.rg:31): three phases
// with the data flow's barriers -- rho_zz /= zz (cells), ru from u and the new rho_zz
// (edges), then rw (the w part, minus the slope flux of ru over the cell's edges) and the
// thermodynamic diagnostics (cells)
template <int LP>
__global__ __launch_bounds__(256) void k_icd_rho(DevState S) {
    ColMap<LP> m(S, KC);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO || k >= L) return;
    double* rz = fw(S, F_rho_zz);
    const double zz = colk(fd(S, F_zz), c);
    colk(rz, c) = colk(rz, c) / zz;
}
template <int LP>
__global__ __launch_bounds__(256) void k_icd_ru(DevState S) {
    ColMap<LP> m(S, KE);
    const int L = S.L, k = m.k, e = m.ent;
    if (e >= S.nEO || k >= L) return;
    const int cell1 = fi(S, F_cellsOnEdge)[(size_t)e * 2], cell2 = fi(S, F_cellsOnEdge)[(size_t)e * 2 + 1];
    const double* rz = fd(S, F_rho_zz);
    const double r1 = colk(rz, cell1), r2 = colk(rz, cell2);
    colk(fw(S, F_ru), e) = 0.5 * colk(fd(S, F_u), e) * (r1 + r2);
}
template <int LP>
__global__ __launch_bounds__(256) void k_icd_cells(DevState S, double rgas_p0, double rgas, double rcv) {
    ColMap<LP> m(S, KC);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO) return;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* sgn = fd(S, F_edgesOnCellSign) + (size_t)c * 10;
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double rz = col_rd<LP>(fd(S, F_rho_zz), c, k, L), zz = col_rd<LP>(fd(S, F_zz), c, k, L);
    const double rz_m = lvl_dn<LP>(rz, k), zz_m = lvl_dn<LP>(zz, k);
    const double w = colk(fd(S, F_w), c);
    const double *ru = fd(S, F_ru), *zb = fd(S, F_zb_cell), *zb3 = fd(S, F_zb3_cell);
    double rw = 0.0;
    if (k > 0) rw = w * (fzp * rz_m + fzm * rz) * (fzp * zz_m + fzm * zz);
    const double zfac = fzp * zz_m + fzm * zz;
    for (int i = 0; i < ne; i++) {  // every lane takes part (the shuffle below)
        const double r = colk(ru, eoc[i]);
        const double r_m = lvl_dn<LP>(r, k);
        const double flux = fzm * r + fzp * r_m;
        const double z = colk(zb, c * 10 + i), z3 = colk(zb3, c * 10 + i);
        const double t = sgn[i] * (z + copysign(1.0, flux) * z3) * flux * zfac;
        rw = (k > 0) ? rw - t : rw;
    }
    if (k >= L) return;
    colk(fw(S, F_rw), c) = rw;
    const double rb = colk(fd(S, F_rho_base), c), tb = colk(fd(S, F_theta_base), c), tm = colk(fd(S, F_theta_m), c);
    const double rho_p = rz - rb;
    const double rtheta_base = tb * rb;
    const double rtheta_p = tm * rho_p + rb * (tm - tb);
    const double exner = pow(zz * rgas_p0 * (rtheta_p + rtheta_base), rcv);
    const double exner_base = pow(zz * rgas_p0 * (rtheta_base), rcv);
    colk(fw(S, F_rho_p), c) = rho_p;
    colk(fw(S, F_rtheta_base), c) = rtheta_base;
    colk(fw(S, F_rtheta_p), c) = rtheta_p;
    colk(fw(S, F_exner), c) = exner;
    colk(fw(S, F_exner_base), c) = exner_base;
    colk(fw(S, F_pressure_p), c) = zz * rgas * (exner * rtheta_p + rtheta_base * (exner - exner_base));
    colk(fw(S, F_pressure_base), c) = zz * rgas * exner_base * rtheta_base;
}
template <int LP>
static hipError_t icd_lp(const DevState& S, hipStream_t st) {
    const int nCB = col_blocks<LP>(S, KC);
    if (nCB) k_icd_rho<LP><<<nCB, 256, 0, st>>>(S);
    HALO_WROTE(S, F_rho_zz);
    auto ke = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KE);
        if (nb) k_icd_ru<LP><<<nb, 256, 0, st>>>(X);
    };
    HALO_RUN(S, st, ke, F_rho_zz);
    HALO_WROTE(S, F_ru);
    auto kc = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (nb) k_icd_cells<LP><<<nb, 256, 0, st>>>(X, kRgas / 100000, kRgas, kRgas / (kCp - kRgas));
    };
    HALO_RUN(S, st, kc, F_ru);
    HALO_WROTE(S, F_rw, F_rho_p, F_rtheta_base, F_rtheta_p, F_exner, F_exner_base, F_pressure_p, F_pressure_base);
    return hipGetLastError();
}
hipError_t launch_init_coupled_diagnostics(const DevState& S, hipStream_t st) {
    MPAS_LP_DISPATCH(S.LP, icd_lp, S, st);
}

// ---------------------------------------------------------------- reconstruct_2d
template <int LP>
__global__ __launch_bounds__(256) void k_reconstruct(DevState S, int on_a_sphere) {
    ColMap<LP> m(S, KC);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO) return;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* cr = fd(S, F_coeffs_reconstruct) + (size_t)c * 30;
    const double* u = fd(S, F_u);
    int e_[NF];
    double co_[3 * NF], u_[NF];
    row_ld(eoc, e_);
    row_ld(cr, co_);
#pragma unroll
    for (int i = 0; i < NF; i++) u_[i] = colk(u, e_[i]);
    const double clat = fd(S, X_cosLatCell)[c], slat = fd(S, X_sinLatCell)[c];
    const double clon = fd(S, X_cosLonCell)[c], slon = fd(S, X_sinLonCell)[c];
    // (every level written: level L with its kept value, the padding with zeros -- keep tails)
    auto kL = [&](int f) { return keepv<LP>(S, f, KC, c); };
    double X = 0.0, Y = 0.0, Z = 0.0;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        X = add_if(i < ne, X, co_[3 * i + 0] * u_[i]);
        Y = add_if(i < ne, Y, co_[3 * i + 1] * u_[i]);
        Z = add_if(i < ne, Z, co_[3 * i + 2] * u_[i]);
    }
    for (int i = NF; i < ne; i++) {
        const double ue = colk(u, eoc[i]);
        X += cr[3 * i + 0] * ue;
        Y += cr[3 * i + 1] * ue;
        Z += cr[3 * i + 2] * ue;
    }
    colk(fw(S, F_uReconstructX), c) = KEEPW(X, kL(F_uReconstructX));
    colk(fw(S, F_uReconstructY), c) = KEEPW(Y, kL(F_uReconstructY));
    colk(fw(S, F_uReconstructZ), c) = KEEPW(Z, kL(F_uReconstructZ));
    if (on_a_sphere) {
        colk(fw(S, F_uReconstructZonal), c) = KEEPW(-X * slon + Y * clon, kL(F_uReconstructZonal));
        colk(fw(S, F_uReconstructMeridional), c) = KEEPW(-(X * clon + Y * slon) * slat + Z * clat,
                                                         kL(F_uReconstructMeridional));
    } else {
        colk(fw(S, F_uReconstructZonal), c) = KEEPW(X, kL(F_uReconstructZonal));
        colk(fw(S, F_uReconstructMeridional), c) = KEEPW(Y, kL(F_uReconstructMeridional));
    }
}
template <int LP>
static hipError_t reconstruct_lp(const DevState& S, hipStream_t st, int on_a_sphere) {
    auto run = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (nb) k_reconstruct<LP><<<nb, 256, 0, st>>>(X, on_a_sphere);
    };
    HALO_RUN(S, st, run, F_u);
    HALO_WROTE(S, F_uReconstructX, F_uReconstructY, F_uReconstructZ, F_uReconstructZonal, F_uReconstructMeridional);
    return hipGetLastError();
}
hipError_t launch_reconstruct_2d(const DevState& S, hipStream_t st, int on_a_sphere) {
    MPAS_LP_DISPATCH(S.LP, reconstruct_lp, S, st, on_a_sphere);
}

// ---------------------------------------------------------------- output diagnostics
// dynamics_tasks.rg:729-746: rho = rho_zz * zz, pressure = pressure_base + pressure_p over
// cells x levels 0..nVertLevels-1 (the theta statement is commented out there); under the
// MPAS dynamics (physics = 2) also MPAS-A's surface pressure, the hydrostatic extrapolation
// init_atm_case_jw uses (init_atm_cases.rg:519-520)
template <int LP>
__global__ __launch_bounds__(256) void k_output_diag(DevState S) {
    ColMap<LP> m(S, KC);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO) return;
    double rz, zz, pb, pp;
    gather2<LP>(fd(S, F_rho_zz), c, fd(S, F_zz), c, k, rz, zz);  // (every lane: gather2)
    gather2<LP>(fd(S, F_pressure_base), c, fd(S, F_pressure_p), c, k, pb, pp);
    if (S.physics == 2) {  // the MPAS dynamics: surface pressure (ora_mpas_surface_pressure)
        const double q = colk(fd(S, F_qtot), c);
        const double rq = rz * (1.0 + q), rq1 = lvl_up<LP>(rq, k);
        const double dz0 = 1.0 / fd(S, F_rdzw)[0];
        if (k == 0) colk(fw(S, F_surface_pressure), c) = 0.5 * dz0 * kGravity * (1.25 * rq - 0.25 * rq1) + pp + pb;
    }
    if (k == L) return;
    colk(fw(S, F_rho), c) = PADW(rz * zz);
    colk(fw(S, F_pressure), c) = PADW(pb + pp);
}
template <int LP>
static hipError_t output_diag_lp(const DevState& S, hipStream_t st) {
    const int nb = col_blocks<LP>(S, KC);
    if (nb) k_output_diag<LP><<<nb, 256, 0, st>>>(S);
    HALO_WROTE(S, F_rho, F_pressure);
    if (S.physics == 2) HALO_WROTE(S, F_surface_pressure);
    return hipGetLastError();
}
hipError_t launch_output_diagnostics(const DevState& S, hipStream_t st) {
    MPAS_LP_DISPATCH(S.LP, output_diag_lp, S, st);
}

// ---------------------------------------------------------------- summarize_timestep
// Sequential semantics made parallel.  The points of a field are numbered in the
// reference's loop order, idx = entity * nVertLevels + k; every thread scans one
// contiguous chunk in that order and the chunks combine in order:
//   FirstExt  "if (x < best) ..." from 1e20 (or > from -1e20): the first point holding the
//             extreme, NaN never taken;
//   Fold      acc = min(acc, x) with min(a,b) = a < b ? a : b from acc = 0.0: a NaN makes
//             acc NaN and the next point then replaces it, so the result is the extreme
//             of the points after the last NaN with ties going to the LATER point (the
//             0.0 start counts only when there is no NaN), or NaN if the last point is one.
struct FirstExt {
    double v;
    long i;
};
struct Fold {
    long nan;  // index of the last NaN, -1 if none
    double v;
    long i;    // -1: no point after the last NaN yet
};
struct SumPart {
    FirstExt mn, mx, spd;
    Fold fmn, fmx;
    int has_nan;
};

__device__ __forceinline__ void fe_take(FirstExt& a, const FirstExt& b, bool is_min) {
    // b follows a (b's points come after a's): b wins only if strictly better
    if (b.i < 0) return;
    if (a.i < 0 || (is_min ? (b.v < a.v) : (b.v > a.v))) a = b;
}
__device__ __forceinline__ void fold_take(Fold& a, const Fold& b, bool is_min) {
    if (b.nan >= 0) {  // everything in a is before b's last NaN
        a = b;
        return;
    }
    if (b.i < 0) return;
    if (a.i < 0 || (is_min ? !(a.v < b.v) : !(a.v > b.v))) {  // ties to the later point
        a.v = b.v;
        a.i = b.i;
    }
}
__device__ __forceinline__ void part_init(SumPart& p) {
    p.mn = {1.0e20, -1};
    p.mx = {-1.0e20, -1};
    p.spd = {-1.0e20, -1};
    p.fmn = {-1, 0.0, -1};
    p.fmx = {-1, 0.0, -1};
    p.has_nan = 0;
}
__device__ __forceinline__ void part_take(SumPart& a, const SumPart& b) {
    fe_take(a.mn, b.mn, true);
    fe_take(a.mx, b.mx, false);
    fe_take(a.spd, b.spd, false);
    fold_take(a.fmn, b.fmn, true);
    fold_take(a.fmx, b.fmx, false);
    a.has_nan |= b.has_nan;
}

// which = 0: w over the owned cells; 1: u (and the wind speed with v) over the owned edges
template <int LP>
__global__ __launch_bounds__(256) void k_sum_scan(DevState S, int which, long chunk, SumPart* parts) {
    const long n = (long)(which == 0 ? S.nCO : S.nEO) * S.L;
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    const double* x = fd(S, which == 0 ? F_w : F_u);
    const double* y = fd(S, F_v);
    SumPart p;
    part_init(p);
    for (long idx = t * chunk; idx < n && idx < (t + 1) * chunk; idx++) {
        const long ent = idx / S.L, k = idx - ent * S.L;
        const double xv = x[ent * LP + lpos(LP, k)];
        if (xv < p.mn.v) p.mn = {xv, idx};
        if (xv > p.mx.v) p.mx = {xv, idx};
        if (which == 1) {
            const double yv = y[ent * LP + lpos(LP, k)];
            const double spd = sqrt(xv * xv + yv * yv);
            if (spd > p.spd.v) p.spd = {spd, idx};
        }
        if (isnan(xv)) {
            p.has_nan = 1;
            p.fmn = {idx, xv, -1};
            p.fmx = {idx, xv, -1};
        } else {
            if (p.fmn.i < 0 || !(p.fmn.v < xv)) p.fmn.v = xv, p.fmn.i = idx;
            if (p.fmx.i < 0 || !(p.fmx.v > xv)) p.fmx.v = xv, p.fmx.i = idx;
        }
    }
    parts[t] = p;
}

// one block: combine the chunk partials in order and finish the printed records
__global__ __launch_bounds__(256) void k_sum_final(DevState S, int which, const SumPart* parts, int nparts,
                                                   double* out) {
    __shared__ SumPart sh[256];
    const int t = threadIdx.x;
    const int per = (nparts + 255) / 256;
    SumPart p;
    part_init(p);
    for (int j = t * per; j < nparts && j < (t + 1) * per; j++) part_take(p, parts[j]);
    sh[t] = p;
    __syncthreads();
    for (int s = 1; s < 256; s <<= 1) {
        if ((t % (2 * s)) == 0 && t + s < 256) part_take(sh[t], sh[t + s]);
        __syncthreads();
    }
    if (t != 0) return;
    p = sh[0];
    const double pi_const = 2.0 * asin(1.0);
    const int L = S.L;
    const double* lat = fd(S, which == 0 ? F_lat : F_latEdge);
    const double* lon = fd(S, which == 0 ? F_lon : F_lonEdge);
    auto rec = [&](double* r, const FirstExt& e, bool level_k_latlon) {
        const long ent = e.i >= 0 ? e.i / L : -1, k = e.i >= 0 ? e.i % L : -1;
        double la = 0.0, lo = 0.0;
        if (ent >= 0 && (!level_k_latlon || k == 0)) {  // 2-D mesh data at level > 0 reads 0 (Q2)
            la = lat[ent];
            lo = lon[ent];
        }
        r[0] = e.v;
        r[1] = (double)ent;
        r[2] = (double)k;
        la *= 180.0 / pi_const;
        lo *= 180.0 / pi_const;
        if (lo > 180.0) lo -= 360.0;
        r[3] = la;
        r[4] = lo;
    };
    auto fold_end = [&](const Fold& f, bool is_min) {
        const long n = (long)(which == 0 ? S.nCO : S.nEO) * L;
        if (f.nan >= 0 && f.nan == n - 1) return f.v;  // the last point is NaN
        if (f.nan >= 0) return f.v;                    // extreme after the last NaN
        // no NaN: the 0.0 start precedes every point; ties go to the later point
        if (f.i < 0) return 0.0;
        return is_min ? ((0.0 < f.v) ? 0.0 : f.v) : ((0.0 > f.v) ? 0.0 : f.v);
    };
    double* o = out + (which == 0 ? 0 : 10);
    rec(o, p.mn, false);
    rec(o + 5, p.mx, true);
    if (which == 1) rec(out + 20, p.spd, false);
    out[25 + which] = p.has_nan ? 1.0 : 0.0;
    out[27 + 2 * which] = fold_end(p.fmn, true);
    out[28 + 2 * which] = fold_end(p.fmx, false);
}

template <int LP>
static hipError_t summarize_lp(const DevState& S, hipStream_t st, void* scratch, double* out) {
    constexpr int T = 64 * 256;  // chunk scanners
    SumPart* parts = (SumPart*)scratch;
    for (int which = 0; which < 2; which++) {
        const long n = (long)(which == 0 ? S.nCO : S.nEO) * S.L;
        const long chunk = (n + T - 1) / T;
        k_sum_scan<LP><<<T / 256, 256, 0, st>>>(S, which, chunk > 0 ? chunk : 1, parts);
        k_sum_final<<<1, 256, 0, st>>>(S, which, parts, T, out);
    }
    return hipGetLastError();
}
size_t summarize_scratch_bytes() { return (size_t)64 * 256 * sizeof(SumPart); }
hipError_t launch_summarize(const DevState& S, hipStream_t st, void* scratch, double* out) {
    MPAS_LP_DISPATCH(S.LP, summarize_lp, S, st, scratch, out);
}

}  // namespace mpas
