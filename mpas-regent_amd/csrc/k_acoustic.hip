// k_acoustic.hip -- atm_advance_acoustic_step_work (dynamics_tasks.rg:1546-1705), gfx950.
//
// One wavefront per cell column (lane k = level k).  Everything except the vertical
// recurrence of rw_p is level-parallel: the small-step initialisation, the horizontal
// flux gather over edgesOnCell (ru_p at the edge, theta_m at cellsOnEdge), rs/ts, and
// the final rho_pp/rtheta_pp/wwAvg updates.
//
// The recurrence (Q20: rw_p(k) reads rw_p, rho_pp, rtheta_pp of level k-1 AFTER their
// update; Q19: rs(k-1) = ts(k-1) = 0; Q21: no back substitution) is, with those k-1
// values affine in rw_p(k-1), a first-order linear recurrence
//        x_k = G_k * x_{k-1} + H_k,   x_0 = rw_p(0) (not updated)
// solved by an inclusive affine prefix scan over the lanes with wavefront shuffles
// (log2(LP) steps).  The scan reassociates fp64, so this path agrees with the oracle
// to rounding (tests/test_gpu_parity.py states the tolerance).  The EXACT=true
// variant evaluates the literal expression level by level (lane k-1 -> lane k
// broadcast) and is bit-identical to the oracle; it is the reference for the scan.
#include "k_cols.h"
#include "mpas_dev.h"
#include "mpas_halo.h"

#include <type_traits>

namespace mpas {

// FIRST: small_step == 0, where rho_pp, rtheta_pp, rw_p and wwAvg start from 0 (:1615-1636):
// their columns are not read at all (4 of the 19 own columns).
// MPASV: the MPAS vertical solver (option "physics" = 1, oracle ora_mpas_acoustic_step):
// rs/ts of every level, the explicit rw_p part from ts(k-1), rs(k-1) and the old
// rho_pp/rtheta_pp of level k-1 (Q19, Q20), the tridiagonal solve up (forward sweep) and
// down (the back substitution the reference leaves commented out, Q21), the Rayleigh
// term, then rho_pp/rtheta_pp; tend_rt = tend_theta (Q8).  Both sweeps are first-order
// linear recurrences: an affine prefix scan over the wavefront, upward then downward
// (EXACT: level by level in the reference's order).  The ru_p update (Q18) runs before,
// in k_acoustic_ru.
//
// MODE (reference semantics, no halo, option "fusedamp"; launch_acoustic): 0 plain; 1 also
// stores this substep's div = -(rtheta_pp - rtheta_pp_old) (:1755) per cell in X_dvA; 2
// also applies the PREVIOUS substep's atm_divergence_damping_3d (:1742-1762, coefficient
// coef_prev, its div in X_dvB) to every ru_p it reads -- the same expression on the same
// values as the damping kernel, so the same bits -- and writes the damped ru_p of the
// edges this cell owns (X_eown; the lowest (cell, slot) listing an edge) to X_rupB, all
// levels (level L copied, padding 0); the edges no cell lists are written by blocks of
// their own (X_orph, acoustic_orph_body).  The damping launch between two substeps disappears: its ru_p
// read-modify-write and its cell gathers (theta_m is gathered here anyway).
// t12 = theta_m(cell1) + theta_m(cell2) (the same value as t2 + t1: X_tme)
template <int LP>
__device__ __forceinline__ double damp_edge(double rup, double d1, double d2, double t12, double spec, double coef,
                                            bool on) {
    return on ? rup + coef * (d2 - d1) * (1.0 - spec) / t12 : rup;  // (:1757-1759 order)
}

// MODE 2, the edges no cell lists (X_orph): the damping alone, into the new buffer.  Its own
// blocks -- a launch of their own (k_acoustic_orph) or the tail of a combined grid: with this
// store on a path of the cell kernel, the compiler could no longer prove the cell kernel's
// mesh rows unclobbered and loaded them as vector loads after its first gathers (18 more
// VGPRs, a second memory round trip)
template <int LP, bool TME>
__device__ __forceinline__ void acoustic_orph_body(const DevState& S, double coefp, int ob) {
    const int L = S.L, k = (int)(threadIdx.x % LP);
    const int j = col_of<LP>(ob);
    if (j >= S.n_orph) return;
    const int e = fi(S, X_orph)[j];
    const int c1 = fi(S, F_cellsOnEdge)[(size_t)e * 2], c2 = fi(S, F_cellsOnEdge)[(size_t)e * 2 + 1];
    const double *dvi = fd(S, X_dvB), *tmf = fd(S, F_theta_m);
    const double ru = colk(fd(S, F_ru_p), e), d1 = colk(dvi, c1), d2 = colk(dvi, c2);
    const double t12 = TME ? colk(fd(S, X_tme), e) : colk(tmf, c1) + colk(tmf, c2);
    const int sh1 = fi(S, F_isShared)[c1], sh2 = fi(S, F_isShared)[c2];
    const bool on = (k < L) & !(sh1 & sh2);
    colk(fw(S, X_rupB), e) = PADW(damp_edge<LP>(ru, d1, d2, t12, fd(S, F_specZoneMaskEdge)[e], coefp, on));
}
template <int LP, bool TME>
__global__ __launch_bounds__(256) void k_acoustic_orph(DevState S, double coefp) {
    acoustic_orph_body<LP, TME>(S, coefp, (int)blockIdx.x);
}

// TME (atm_srk3, option "tmedge"): theta_m(cell2) + theta_m(cell1) of each edge comes from
// X_tme, which the stage's dyn_tend edge kernel formed (theta_m is not written in between):
// one gathered column per edge instead of two -- the same sums
// SML (atm_srk3, option "fusesml"; a stage's first substep): the stage's set_smlstep first;
// 1 from its slope fluxes, 2 (fast path) from their sum per level, X_smlS, formed once per step
// by k_sml_flux: u_tend, zb_cell and zb3_cell do not change within a step (reference semantics)
template <int LP, bool EXACT, bool SELF, bool FIRST, bool MPASV, int MODE, bool TME, int SML>
__device__ __forceinline__ void acoustic_body(const DevState& S, double dts, int small_step, double epssm, double resm,
                                              double coefp, int ncb, Blk bk, int wold = 1, int ddx = 0) {
    static_assert(!(MPASV && MODE), "the deferred damping is the reference semantics' (physics 0)");
    static_assert(!SML || (FIRST && !MPASV), "set_smlstep precedes a stage's first substep (reference semantics)");
    static_assert(SML != 2 || !EXACT, "the flux sum reassociates: fast path only");
    const int L = S.L, k = (int)(threadIdx.x % LP);
    int blk = bk.b;
    blk = xcd_block_n(S.xcd, blk, ncb);  // (ncb: the cell blocks, bk.n or fewer)
    const int c = col_of<LP>(blk) + S.lo[KC];
    if (c >= S.nCO) return;
    const size_t p = (size_t)c * LP + lpos(LP, k);
    double* rtp_f = fw(S, F_rtheta_pp);
    double* rpp_f = fw(S, F_rho_pp);
    double* rwp_f = fw(S, F_rw_p);
    double* ww_f = fw(S, F_wwAvg);
    const bool kl = k < L;
    // ---- every load of the column and of its edge gathers first, ahead of the first
    // store (which could alias them for the compiler)
    const double spec = fd(S, F_specZoneMaskCell)[c];
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* sgn = fd(S, F_edgesOnCellSign) + (size_t)c * 10;
    const int *cc1 = fi(S, X_ce_c1) + (size_t)c * 10, *cc2 = fi(S, X_ce_c2) + (size_t)c * 10;
    const double* cdv = fd(S, X_ce_dv) + (size_t)c * 10;
    const double invA = fd(S, F_invAreaCell)[c];
    const double *ru_p = fd(S, F_ru_p), *tm_f = fd(S, F_theta_m);
    const int *coth = fi(S, X_ce_oth) + (size_t)c * 10, *cs1 = fi(S, X_ce_s1) + (size_t)c * 10;
    int e_[NF], c1_[NF], c2_[NF], o_[NF], s1_[NF];
    double sgn_[NF], cdv_[NF], rup_[NF], t1_[NF], t2_[NF], ts_[NF];  // ts_: theta_m(cell2) + theta_m(cell1)
    const int ne = SELF ? cell_rec<true>(S, c, e_, o_, s1_) : cell_rec<false>(S, c, e_, c1_, c2_);
    row_ld(sgn, sgn_);
    row_ld(cdv, cdv_);
    // (gather2 / col_rd2: two columns per load instruction)
    double rtp, rpp, rwp, ww, tm, tend_rho, w, coftz, zz, rz, cofwt, cofwz, cofwr, a_tri, alpha, rws, rw, dss;
    if constexpr (FIRST) {
        rtp = rpp = rwp = ww = 0.0;
    } else {
        col_rd2<LP>(rtp_f, rpp_f, c, k, L, rtp, rpp);
        col_rd2<LP>(rwp_f, ww_f, c, k, L, rwp, ww);
    }
    col_rd2<LP>(fd(S, F_theta_m), fd(S, F_tend_rho), c, k, L, tm, tend_rho);
    // SML: the point's cprMask byte with the column loads (tested after a lane condition it
    // was loaded under a divergent branch and waited for there)
    const uint8_t cpr = SML ? ((const uint8_t*)S.f[F_cprMask])[p] : 0;
    static_assert(NF % 2 == 0, "slot pairs");
#pragma unroll
    for (int i = 0; i < NF; i += 2) {
        gather2s<LP>(ru_p, e_[i], e_[i + 1], k, rup_[i], rup_[i + 1]);
        if constexpr (TME) {
            gather2s<LP>(fd(S, X_tme), e_[i], e_[i + 1], k, ts_[i], ts_[i + 1]);
        } else {
            cell_pair2<LP, SELF>(tm_f, c1_, c2_, o_, s1_, tm, i, k, t1_[i], t2_[i], t1_[i + 1], t2_[i + 1]);
            ts_[i] = t2_[i] + t1_[i];
            ts_[i + 1] = t2_[i + 1] + t1_[i + 1];
        }
    }
    int own = 0;
    if constexpr (MODE == 2) {  // the previous substep's damping on this cell's edges
        const double* dvi = fd(S, X_dvB);
        const int* sh = fi(S, F_isShared);
        const double* spz = fd(S, F_specZoneMaskEdge);
        own = fi(S, X_eown)[c];
        const double dv_c = SELF ? colk(dvi, c) : 0.0;
        double d1_[NF], d2_[NF];
#pragma unroll
        for (int i = 0; i < NF; i += 2)
            cell_pair2<LP, SELF>(dvi, c1_, c2_, o_, s1_, dv_c, i, k, d1_[i], d2_[i], d1_[i + 1], d2_[i + 1]);
        // the isShared flags of every slot's two cells loaded up front and combined without
        // short-circuit evaluation: `kl && ... && !(sh[x1] && sh[x2])` put each slot's loads
        // under a lane-divergent branch with a full wait inside (six round trips per wave)
        // (specZoneMaskEdge too: sunk into the `on` branch, its load waited there)
        int sh1_[NF], sh2_[NF];
        double spz_[NF];
#pragma unroll
        for (int i = 0; i < NF; i++) {
            const int x1 = SELF ? (s1_[i] ? c : o_[i]) : c1_[i], x2 = SELF ? (s1_[i] ? o_[i] : c) : c2_[i];
            sh1_[i] = sh[x1];
            sh2_[i] = sh[x2];
            // (the edge's mask: wave-uniform at LP = 64, one column per wave)
            spz_[i] = LP == 64 ? uniform_d(spz[e_[i]]) : spz[e_[i]];
        }
#pragma unroll
        for (int i = 0; i < NF; i++) {
            const bool on = kl & (e_[i] < S.nEdges) & !(sh1_[i] & sh2_[i]);
            rup_[i] = damp_edge<LP>(rup_[i], d1_[i], d2_[i], ts_[i], spz_[i], coefp, on);
        }
    }
    // (rup_ / ts_ at k >= L: unused, the flux sum below selects on kl)
    col_rd2<LP>(fd(S, F_w), fd(S, F_coftz), c, k, L, w, coftz);
    col_rd2<LP>(fd(S, F_zz), fd(S, F_rho_zz), c, k, L, zz, rz);
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    int wst = 0;  // SML: set_smlstep's w store (1: the new w, 2: the padding's 0.0), made below
    if constexpr (SML == 2) {  // (X_smlS: k_sml_flux's sum of the slope fluxes)
        double wn = w - colk(fd(S, X_smlS), c);
        wn *= (fzm * zz + fzp * lvl_dn<LP>(zz, k));
        const bool rz_ok = fi(S, F_bdyMaskCell)[c] <= kRelaxZone;
        wst = ((k <= L) & rz_ok & (cpr != 0)) ? 1 : ((k > L) & rz_ok) ? 2 : 0;
        if (wst == 1) w = wn;
    } else if constexpr (SML == 1) {
        // the stage's atm_set_smlstep_pert_variables_work (:1503-1528, k_set_smlstep's
        // expressions) on this column, just before the substep reads w: the points of cpr
        // (cprMask) within the relaxation zone get w -= sum of the slope fluxes of u_tend,
        // w *= the zz average; the acoustic step then works on that w
        const double* ut_f = fd(S, F_u_tend);
        const double *zb = fd(S, F_zb_cell), *zb3 = fd(S, F_zb3_cell);
        const double* sgnc = fd(S, F_edgesOnCell_sign) + (size_t)c * 10;
        double ut_[NF], utm_[NF], zb_[NF], zb3_[NF], sgs_[NF];
        row_ld(sgnc, sgs_);
#pragma unroll
        for (int i = 0; i < NF; i += 2) gather2s<LP>(ut_f, e_[i], e_[i + 1], k, ut_[i], ut_[i + 1]);
#pragma unroll
        for (int i = 0; i < NF; i++) {
            ut_[i] = ldz(k <= L, ut_[i]);
            gather2<LP>(zb, c * 10 + i, zb3, c * 10 + i, k, zb_[i], zb3_[i]);  // (one 16-B load)
        }
#pragma unroll
        for (int i = 0; i < NF; i++) utm_[i] = lvl_dn<LP>(ut_[i], k);
        // (exact: the terms subtracted from w one by one, :1512-1521; fast path: summed first
        // in k_sml_flux's order, then subtracted -- the same bits as SML = 2 and k_set_smlstep's
        // fast path)
        double wn = w, sum = 0.0;
#pragma unroll
        for (int i = 0; i < NF; i++) {
            double flux = sgs_[i] * (fzm * ut_[i] + fzp * utm_[i]);
            const double t = (zb_[i] + copysign(1.0, ut_[i]) * zb3_[i]) * flux;
            if constexpr (EXACT) wn = sub_if(i < ne, wn, t);
            else sum = add_if(i < ne, sum, t);
        }
        for (int i = NF; i < ne; i++) {
            int iEdge = eoc[i];
            double ut = col_rd<LP>(ut_f, iEdge, k, L);
            double ut_m = lvl_dn<LP>(ut, k);
            double flux = sgnc[i] * (fzm * ut + fzp * ut_m);
            size_t q = ((size_t)c * 10 + i) * LP + lpos(LP, k);
            if constexpr (EXACT) wn -= (zb[q] + copysign(1.0, ut) * zb3[q]) * flux;
            else sum += (zb[q] + copysign(1.0, ut) * zb3[q]) * flux;
        }
        if constexpr (!EXACT) wn = w - sum;
        wn *= (fzm * zz + fzp * lvl_dn<LP>(zz, k));
        const bool rz_ok = fi(S, F_bdyMaskCell)[c] <= kRelaxZone;
        wst = ((k <= L) & rz_ok & (cpr != 0)) ? 1 : ((k > L) & rz_ok) ? 2 : 0;
        if (wst == 1) w = wn;
    }
    // the w tendency: the state w in the reference and under physics = 1 (Q8), tend_w under
    // the MPAS dynamics (physics = 2); the implicit Rayleigh term reads the state w
    const double tw = (MPASV && S.physics == 2) ? col_rd<LP>(fd(S, F_tend_w), c, k, L) : w;
    col_rd2<LP>(fd(S, F_cofwt), fd(S, F_cofwz), c, k, L, cofwt, cofwz);
    col_rd2<LP>(fd(S, F_cofwr), fd(S, F_a_tri), c, k, L, cofwr, a_tri);
    // (ddx, atm_srk3 with option smlsum: rw_save - rw, the step uses only their difference, from
    // X_Dd -- formed once per step, the same value: one column read instead of two)
    double dd;
    if (!MPASV && ddx) {
        col_rd2<LP>(fd(S, F_alpha_tri), fd(S, X_Dd), c, k, L, alpha, dd);
        dss = col_rd<LP>(fd(S, F_dss), c, k, L);
    } else {
        col_rd2<LP>(fd(S, F_alpha_tri), fd(S, F_rw_save), c, k, L, alpha, rws);
        col_rd2<LP>(fd(S, F_rw), fd(S, F_dss), c, k, L, rw, dss);
        dd = rws - rw;
    }
    double gam = 0.0, tend_th = 0.0;
    if constexpr (MPASV) col_rd2<LP>(fd(S, F_gamma_tri), fd(S, F_tend_theta), c, k, L, gam, tend_th);
    const double tt = MPASV ? tend_th : tm;  // tend_rt: the reference reads theta_m (Q8)
    const double cofrz = fd(S, F_cofrz)[k], rdzw = fd(S, F_rdzw)[k];
    // ---- the stores of the values formed above (the previous substep's damped ru_p on the
    // edges this cell owns, set_smlstep's w), after the column's last load: made where they
    // were formed, they let no later load move above them (the compiler cannot tell they do not
    // alias), and the second batch of column loads waited for the first batch's consumers
    if constexpr (MODE == 2) {
        double* rup_out = fw(S, X_rupB);
#pragma unroll
        for (int i = 0; i < NF; i++)
            if ((own >> i) & 1) colk(rup_out, e_[i]) = PADW(rup_[i]);  // (level L: the value read)
    }
    if constexpr (SML != 0) {
        if (wst == 1) {
            colk(fw(S, F_w), c) = w;
            if (k == L) keep_put<LP>(S, F_w, KC, c, w);  // (w's level L changes: its keep tail too)
        } else if (wst == 2) {
            colk(fw(S, F_w), c) = 0.0;  // (the padding's content: the column's last line written whole)
        }
    }

    // :1615-1636
    const double rtpo = (small_step == 0) ? 0 : rtp;
    // wold bit 1 (atm_srk3 option ntu, MODE != 0: the last substep of a stage before the step's last):
    // this substep's rho_pp, rtheta_pp, rw_p and wwAvg are dead -- the next stage's first substep sets
    // them (:1615-1636) before any task reads them, and the damping reads this substep's div (X_dvA)
    const bool nst = MODE != 0 && (wold & 2);
    // (level L: the kept value, keep tails in mpas_dev.h -- every line of the column whole)
    if (MODE == 0 || (wold & 1)) colk(fw(S, F_rtheta_pp_old), c) = KEEPW(rtpo, keepv<LP>(S, F_rtheta_pp_old, KC, c));
    // MODE 1/2: this substep's div (:1755) for the damping applied by the next substep
    auto store_div = [&](double rtp_new) {
        if constexpr (MODE != 0) colk(fw(S, X_dvA), c) = kl ? -(rtp_new - rtpo) : 0.0;
    };
    if (small_step == 0) {
        ww = 0;
        rwp = 0;
        if (kl) {
            rpp = 0;
            rtp = 0;
        }
    }

    if (spec != 0.0) {  // :1698-1703 (column-uniform branch)
        if (kl) {
            rpp = rpp + dts * tend_rho;
            rtp = rtp + dts * tt;
            rwp = rwp + dts * tw;
            ww = ww + 0.5 * (1.0 + epssm) * rwp;
        }
        if (!nst) {
            colk(rpp_f, c) = KEEPW(rpp, keepv<LP>(S, F_rho_pp, KC, c));
            colk(rtp_f, c) = KEEPW(rtp, keepv<LP>(S, F_rtheta_pp, KC, c));
            colk(rwp_f, c) = PADW(rwp);
            if (!(MPASV && (wold & 2))) colk(ww_f, c) = PADW(ww);  // (MPASV, wold bit 1: wwAvg dead)
        }
        store_div(rtp);
        return;
    }

    // ---- horizontal flux (:1644-1652), accumulated in the reference's order
    double rs = 0, ts = 0;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        double flux = sgn_[i] * dts * cdv_[i] * rup_[i] * invA;
        rs = sub_if(i < ne && kl, rs, flux);
        ts = sub_if(i < ne && kl, ts, flux * 0.5 * ts_[i]);
    }
    for (int i = NF; i < ne; i++) {
        double rpe = colk(ru_p, eoc[i]);
        if constexpr (MODE == 2) {
            const int e = eoc[i], x1 = cc1[i], x2 = cc2[i];
            const int sh1 = fi(S, F_isShared)[x1], sh2 = fi(S, F_isShared)[x2];
            const bool on = kl & (e < S.nEdges) & !(sh1 & sh2);
            rpe = damp_edge<LP>(rpe, colk(fd(S, X_dvB), x1), colk(fd(S, X_dvB), x2), colk(tm_f, x1) + colk(tm_f, x2),
                                fd(S, F_specZoneMaskEdge)[e], coefp, on);
            if ((own >> i) & 1) colk(fw(S, X_rupB), e) = PADW(rpe);
        }
        double flux = sgn[i] * dts * cdv[i] * ldz(kl, rpe) * invA;
        rs = sub_if(kl, rs, flux);
        ts = sub_if(kl, ts, flux * 0.5 * (ldz(kl, colk(tm_f, cc2[i])) + ldz(kl, colk(tm_f, cc1[i]))));
    }
    // ---- rs, ts (:1657-1658) from the OLD rw_p
    const double rwp_p = lvl_up<LP>(rwp, k), coftz_p = lvl_up<LP>(coftz, k);
    rs = rpp + dts * tend_rho + rs - cofrz * resm * (rwp_p - rwp);
    ts = rtp + dts * tt + ts - resm * rdzw * (coftz_p * rwp_p - coftz * rwp);

    if constexpr (MPASV) {  // the MPAS-A order (mpas_oracle.c ora_mpas_acoustic_step)
        const double ts_m = lvl_dn<LP>(ts, k), rs_m = lvl_dn<LP>(rs, k);
        const double rtp_m = lvl_dn<LP>(rtp, k), rpp_m = lvl_dn<LP>(rpp, k);
        const double zz_m = lvl_dn<LP>(zz, k), rz_m = lvl_dn<LP>(rz, k), cofwt_m = lvl_dn<LP>(cofwt, k);
        const bool in = k >= 1 && k < L;  // the interior interfaces
        const double rwold = rwp;
        if (in) ww = ww + 0.5 * (1.0 - epssm) * rwold;
        double x = rwold;
        if (in)
            x = rwold + dts * tw - cofwz * ((zz * ts - zz_m * ts_m) + resm * (zz * rtp - zz_m * rtp_m)) -
                cofwr * ((rs + rs_m) + resm * (rpp + rpp_m)) + cofwt * (ts + resm * rtp) + cofwt_m * (ts_m + resm * rtp_m);
        // up: y(k) = (x(k) - a(k) y(k-1)) alpha(k), 1 <= k < L; y(0) = rw_p(0)
        double y = x;
        if constexpr (EXACT) {
            for (int kk = 1; kk < L; kk++) {
                const double yp = __shfl(y, kk - 1, LP);
                y = (k == kk) ? (x - a_tri * yp) * alpha : y;
            }
        } else {
            double G = in ? -a_tri * alpha : 0.0, H = in ? x * alpha : x;
#pragma unroll
            for (int off = 1; off < LP; off <<= 1) {
                const double Gp = __shfl_up(G, off, LP), Hp = __shfl_up(H, off, LP);
                if (k >= off) {
                    H = G * Hp + H;
                    G = G * Gp;
                }
            }
            y = H;
        }
        // down: z(k) = y(k) - gamma(k) z(k+1), k = L-1 .. 0; z(L) = rw_p(L)
        double z = y;
        if constexpr (EXACT) {
            for (int kk = L - 1; kk >= 0; kk--) {
                const double zn = __shfl(z, kk + 1, LP);
                z = (k == kk) ? y - gam * zn : z;
            }
        } else {
            double G = k < L ? -gam : 0.0, H = k <= L ? y : 0.0;
#pragma unroll
            for (int off = 1; off < LP; off <<= 1) {
                const double Gp = __shfl_down(G, off, LP), Hp = __shfl_down(H, off, LP);
                if (k + off < LP) {
                    H = G * Hp + H;
                    G = G * Gp;
                }
            }
            z = H;
        }
        double r = (k == L) ? rwold : z;
        if (in) {  // implicit Rayleigh damping of w
            const double d = dd;
            r = (z + d - dts * dss * (fzm * zz + fzp * zz_m) * (fzm * rz + fzp * rz_m) * w) / (1.0 + dts * dss) - d;
            ww = ww + 0.5 * (1.0 + epssm) * r;
        }
        const double r_p = lvl_up<LP>(r, k);
        // (paired 16-B stores, every lane; level L of rho_pp / rtheta_pp keeps its value)
        put2f<LP>(rpp_f, c, rtp_f, c, k, KEEPW(rs - cofrz * (r_p - r), keepv<LP>(S, F_rho_pp, KC, c)),
                 KEEPW(ts - rdzw * (coftz_p * r_p - coftz * r), keepv<LP>(S, F_rtheta_pp, KC, c)));
        // (wold bit 1, option ntu: a stage's last substep before the last stage -- its wwAvg is dead: the
        // stage's recover leaves the average alone and the next stage's first substep sets it)
        if (wold & 2) colk(rwp_f, c) = PADW(r);
        else put2f<LP>(rwp_f, c, ww_f, c, k, PADW(r), PADW(ww));
        return;
    }

    // per-level coefficients of the recurrence
    const double zz_m = lvl_dn<LP>(zz, k), rz_m = lvl_dn<LP>(rz, k), cofwt_m = lvl_dn<LP>(cofwt, k);
    const double tsm = 0.0, rsm = 0.0;  // Q19
    const double rwold = rwp;
    double x;  // new rw_p of this level

    if (EXACT) {
        // literal level-by-level evaluation; lane k-1 hands (rw_p, rho_pp, rtheta_pp) to lane k
        x = rwold;
        double rpp_new = rs - cofrz * (rwp_p - x);
        double rtp_new = ts - rdzw * (coftz_p * rwp_p - coftz * x);
        const int base = (int)(threadIdx.x & 63) & ~(LP - 1);
        for (int kk = 1; kk < L; kk++) {
            double X = __shfl(x, base + kk - 1, 64);
            double R = __shfl(rpp_new, base + kk - 1, 64);
            double T = __shfl(rtp_new, base + kk - 1, 64);
            if (k == kk) {
                double y = rwold;
                y += dts * w - cofwz * ((zz * ts - zz_m * tsm) + resm * (zz * rtp - zz_m * T)) -
                     cofwr * ((rs + rsm) + resm * (rpp + R)) + cofwt * (ts + resm * rtp) + cofwt_m * (tsm + resm * T);
                y -= a_tri * X;
                y *= alpha;
                y += dd - dts * dss * (fzm * zz + fzp * zz_m) * (fzm * rz + fzp * rz_m) * w;
                y /= (1.0 + dts * dss);
                y -= dd;
                x = y;
                rpp_new = rs - cofrz * (rwp_p - x);
                rtp_new = ts - rdzw * (coftz_p * rwp_p - coftz * x);
            }
        }
    } else {
        // x_k = G_k x_{k-1} + H_k with rtheta_pp_new(k-1) = T0 + Tc x_{k-1},
        // rho_pp_new(k-1) = R0 + Rc x_{k-1}; (T0, Tc, R0, Rc) come from lane k-1
        const double T0 = ts - rdzw * (coftz_p * rwp_p), Tc = rdzw * coftz;
        const double R0 = rs - cofrz * rwp_p, Rc = cofrz;
        const double T0m = lvl_dn<LP>(T0, k), Tcm = lvl_dn<LP>(Tc, k);
        const double R0m = lvl_dn<LP>(R0, k), Rcm = lvl_dn<LP>(Rc, k);
        const double x0 = __shfl(rwold, (int)(threadIdx.x & 63) & ~(LP - 1), 64);
        double G = 1.0, H = 0.0;
        if (k >= 1 && k < L) {
            const double P = rwold + dts * w - cofwz * ((zz * ts) + resm * (zz * rtp)) - cofwr * (rs + resm * rpp) +
                             cofwt * (ts + resm * rtp);
            const double cT = cofwz * resm * zz_m + cofwt_m * resm;
            const double cR = cofwr * resm;
            const double F = 1.0 + dts * dss;
            const double Dd = dd;
            const double E = dts * dss * (fzm * zz + fzp * zz_m) * (fzm * rz + fzp * rz_m) * w;
            const double af = alpha / F;
            G = af * (cT * Tcm - cR * Rcm - a_tri);
            H = af * (P + cT * T0m - cR * R0m) + (Dd - E) / F - Dd;
            if (k == 1) {
                H = G * x0 + H;
                G = 0.0;
            }
        }
#pragma unroll
        for (int off = 1; off < LP; off <<= 1) {
            double Gp = __shfl_up(G, off, LP);
            double Hp = __shfl_up(H, off, LP);
            if (k >= off) {
                H = G * Hp + H;
                G = G * Gp;
            }
        }
        x = (k == 0) ? rwold : H;
    }
    if (k < L && k > 0) ww = ww + 0.5 * (1.0 - epssm) * rwold + 0.5 * (1.0 + epssm) * x;
    // (paired 16-B stores, every lane; level L of rho_pp / rtheta_pp keeps its value)
    const double rtp_new = ts - rdzw * (coftz_p * rwp_p - coftz * x);
    if (!nst) {
        put2f<LP>(rpp_f, c, rtp_f, c, k, KEEPW(rs - cofrz * (rwp_p - x), keepv<LP>(S, F_rho_pp, KC, c)),
                 KEEPW(rtp_new, keepv<LP>(S, F_rtheta_pp, KC, c)));
        put2f<LP>(rwp_f, c, ww_f, c, k, PADW((k < L) ? x : rwp), PADW(ww));
    }
    store_div(rtp_new);
}
template <int LP, bool EXACT, bool SELF, bool FIRST, bool MPASV, int MODE, bool TME, int SML>
__global__ __launch_bounds__(256) void k_acoustic(DevState S, double dts, int small_step, double epssm, double resm,
                                                 double coefp, int ncb, int wold, int ddx) {
    acoustic_body<LP, EXACT, SELF, FIRST, MPASV, MODE, TME, SML>(S, dts, small_step, epssm, resm, coefp, ncb,
                                                                this_blk(), wold, ddx);
}
// MODE 2 on a small grid (fewer than kTailCells owned cells, where a launch's fixed cost is
// most of its time): the orphan edges' blocks at the tail of the cell grid, one launch
// instead of two (on large grids the separate launch keeps the cell path's mesh rows in
// scalar loads, profiles/r04/orph_split)
constexpr int kTailCells = 16384;
template <int LP, bool EXACT, bool SELF, bool FIRST, bool TME, int SML>
__global__ __launch_bounds__(256) void k_acoustic_o(DevState S, double dts, int small_step, double epssm, double resm,
                                                   double coefp, int ncb, int wold, int ddx) {
    const int b = (int)blockIdx.x;
    if (b < ncb)
        acoustic_body<LP, EXACT, SELF, FIRST, false, 2, TME, SML>(S, dts, small_step, epssm, resm, coefp, ncb,
                                                                   Blk{b, ncb}, wold, ddx);
    else acoustic_orph_body<LP, TME>(S, coefp, b - ncb);
}
// option "hfuse" (atm_srk3, stages 0 and 1): a stage's last acoustic launch (MODE 2, the
// damping of the previous substep inside) beside the stage's solve_diagnostics vertex /
// cell kernel, which reads u only -- nothing the acoustic step reads or writes
template <int LP, bool EXACT, bool SELF, int EPW>
__global__ __launch_bounds__(256) void k_hf_ac_vc(DevState S, double dts, int small_step, double epssm, double resm,
                                                 double coefp, int ncb, int nb1, int nVB, int wold, int ddx) {
    const int b = (int)blockIdx.x;
    if (b < ncb)
        acoustic_body<LP, EXACT, SELF, false, false, 2, false, false>(S, dts, small_step, epssm, resm, coefp, ncb,
                                                                       Blk{b, ncb}, wold, ddx);
    else if (b < nb1) acoustic_orph_body<LP, false>(S, coefp, b - ncb);
    else solve_vc_body<LP, EPW, false>(S, nVB, 0, Blk{b - nb1, (int)gridDim.x - nb1});
}

// X_smlS for SML = 2 (atm_srk3 fast path, reference semantics; once per step): per cell and
// level k <= L the sum over the cell's edges of set_smlstep's slope-flux terms (k_set_smlstep
// and acoustic_body SML = 1: the same terms, summed instead of subtracted from w one by one)
template <int LP>
__global__ __launch_bounds__(256) void k_sml_flux(DevState S) {
    sml_flux_body<LP>(S, this_blk());
}
template <int LP>
static hipError_t sml_flux_lp(const DevState& S, hipStream_t st) {
    auto run = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (nb) k_sml_flux<LP><<<nb, 256, 0, st>>>(X);
    };
    HALO_RUN_R1(S, st, run, F_u_tend, F_u_tend);  // (u_tend at the edges of owned cells)
    HALO_WROTE(S, X_smlS, X_Dd);
    return hipGetLastError();
}
hipError_t launch_sml_flux(const DevState& S, hipStream_t st) { MPAS_LP_DISPATCH(S.LP, sml_flux_lp, S, st); }

// :1581-1613 restored (Q18, MPAS vertical solver only): ru_p and ruAvg of every owned
// edge, before the cell kernel reads ru_p.  FIRST (small_step 0): ru_p = dts tend_u and
// ruAvg = ru_p need tend_u alone -- the old ru_p / ruAvg columns are not read (their level L,
// stored back as it is, comes by one scalar load each), nor cqu / zxu: 2 of 6 column streams
// DAMP (option mdamp, small_step > 0): the previous substep's atm_divergence_damping_3d (:1742-1762,
// coefficient coefd) applied to the ru_p read here, before this substep's update -- divdamp_body's
// expression on the same values (its rtheta_pp is the one gathered for the pressure gradient; OLD0:
// rtheta_pp_old = 0 after a stage's first substep), so the same bits; the damping launch goes
template <int LP, bool FIRST, bool DAMP = false, bool OLD0 = false>
__global__ __launch_bounds__(256) void k_acoustic_ru(DevState S, double dts, int small_step, double c2, double coefd) {
    static_assert(!DAMP || !FIRST, "the previous substep's damping: small_step > 0");
    ColMap<LP> m(S, KE);
    const int L = S.L, k = m.k, e = m.ent;
    if (e >= S.nEO) return;
    if constexpr (FIRST) {
        const size_t pL = (size_t)e * LP + lpos(LP, L);
        const double rp0 = ldc(fd(S, F_ru_p) + pL), ra0 = ldc(fd(S, F_ruAvg) + pL);
        const double rp = dts * colk(fd(S, F_tend_u), e);
        const double ra = rp;
        colk(fw(S, F_ru_p), e) = KEEPW(rp, rp0);
        colk(fw(S, F_ruAvg), e) = KEEPW(ra, ra0);
        return;
    }
    const int cell1 = fi(S, F_cellsOnEdge)[(size_t)e * 2], cell2 = fi(S, F_cellsOnEdge)[(size_t)e * 2 + 1];
    double rp, ra, tu, cqu, zxu;
    gather2<LP>(fd(S, F_ru_p), e, fd(S, F_ruAvg), e, k, rp, ra);
    const double rp0 = rp, ra0 = ra;  // (level L: stored back as loaded -- the column's lines whole)
    gather2<LP>(fd(S, F_tend_u), e, fd(S, F_cqu), e, k, tu, cqu);
    zxu = colk(fd(S, F_zxu), e);
    if (small_step != 0) {  // (uniform)
        double t1, t2, z1, z2, x1, x2, r1, r2;
        gather2s<LP>(fd(S, F_rtheta_pp), cell1, cell2, k, t1, t2);
        gather2s<LP>(fd(S, F_zz), cell1, cell2, k, z1, z2);
        gather2s<LP>(fd(S, F_exner), cell1, cell2, k, x1, x2);
        gather2s<LP>(fd(S, F_rho_pp), cell1, cell2, k, r1, r2);
        const double invDc = fd(S, F_invDcEdge)[e], spec = fd(S, F_specZoneMaskEdge)[e];
        if constexpr (DAMP) {
            double o1 = 0.0, o2 = 0.0, m1, m2;
            if (!OLD0) gather2s<LP>(fd(S, F_rtheta_pp_old), cell1, cell2, k, o1, o2);
            gather2s<LP>(fd(S, F_theta_m), cell1, cell2, k, m1, m2);
            const int sh1 = fi(S, F_isShared)[cell1], sh2 = fi(S, F_isShared)[cell2];
            const double divCell1 = -(t1 - o1), divCell2 = -(t2 - o2);
            if (k < L && !(sh1 && sh2)) rp = rp + coefd * (divCell2 - divCell1) * (1.0 - spec) / (m1 + m2);
        }
        double pgrad = ((t2 - t1) * invDc) / (0.5 * (z2 + z1));
        pgrad = cqu * 0.5 * c2 * (x1 + x2) * pgrad;
        pgrad = pgrad + 0.5 * zxu * kGravity * (r1 + r2);
        rp = rp + dts * (tu - (1.0 - spec) * pgrad);
        ra = ra + rp;
    } else {
        rp = dts * tu;
        ra = rp;
    }
    // (padding levels: zeros, PADW; level L: the values loaded, which the reference leaves)
    colk(fw(S, F_ru_p), e) = KEEPW(rp, rp0);
    colk(fw(S, F_ruAvg), e) = KEEPW(ra, ra0);
}

template <int LP>
static hipError_t acoustic_lp(const DevState& S, hipStream_t st, double dts, int small_step, int exact, int mode,
                              double coef_prev, int tme, int sml, int wold, int ddx, int mdamp, int rudone) {
    if ((tme && (S.physics || S.halo)) || (sml && S.physics)) return hipErrorInvalidValue;  // (atm_srk3, reference semantics)
    if (mdamp && (!S.physics || small_step == 0)) return hipErrorInvalidValue;
    if (rudone && (S.physics != 2 || small_step != 0)) return hipErrorInvalidValue;
    if (sml && (small_step != 0 || mode == 0)) return hipErrorInvalidValue;
    double epssm = kEpssm;
    double resm = (1.0 - epssm) / (1.0 + epssm);
    if (mode && S.physics) return hipErrorInvalidValue;  // (srk3 never asks: reference semantics only)
    if (ddx && S.physics) return hipErrorInvalidValue;   // (X_Dd: atm_srk3's reference semantics only)
    if (S.physics) {  // Q18: the edges first
        const double rcv = kRgas / (kCp - kRgas), c2 = kCp * rcv;
        // (mdamp, option mdamp: the previous substep's damping here, coefficient coef_prev; 2: that
        // substep was the stage's first, rtheta_pp_old = 0)
        const bool dmp = mdamp != 0, old0 = mdamp == 2;
        auto ru = [&](const DevState& X) {
            const int nb = col_blocks<LP>(X, KE);
            if (!nb) return;
            if (small_step == 0) k_acoustic_ru<LP, true><<<nb, 256, 0, st>>>(X, dts, small_step, c2, 0.0);
            else if (old0) k_acoustic_ru<LP, false, true, true><<<nb, 256, 0, st>>>(X, dts, small_step, c2, coef_prev);
            else if (dmp) k_acoustic_ru<LP, false, true, false><<<nb, 256, 0, st>>>(X, dts, small_step, c2, coef_prev);
            else k_acoustic_ru<LP, false><<<nb, 256, 0, st>>>(X, dts, small_step, c2, 0.0);
        };
        if (small_step == 0 && rudone) {  // (option mru: this stage's dyn_tend stored ru_p / ruAvg)
        } else if (small_step == 0) HALO_RUN(S, st, ru);  // (own columns only: no ghost read)
        else if (dmp) HALO_RUN(S, st, ru, F_rtheta_pp, F_zz, F_exner, F_rho_pp, F_rtheta_pp_old, F_theta_m);
        else HALO_RUN(S, st, ru, F_rtheta_pp, F_zz, F_exner, F_rho_pp);
        HALO_WROTE(S, F_ru_p, F_ruAvg);
    }
    auto run = [&](const DevState& X) {
        const int ncb = col_blocks<LP>(X, KC);
        if (!ncb) return;
        const int nob = (S.n_orph + 256 / LP - 1) / (256 / LP);  // (MODE 2: the edges no cell lists)
        const bool tail = mode == 2 && nob && X.nCO - X.lo[KC] < kTailCells;
        const int grid = ncb;
        const bool first = small_step == 0;
        if (tail) {  // (one launch: the orphan edges' blocks after the cell blocks)
            auto go_t = [&](auto ex, auto sf) {
                constexpr bool E = decltype(ex)::value, SF = decltype(sf)::value;
#define MPAS_ACO(FI, TM, SM) \
    k_acoustic_o<LP, E, SF, FI, TM, SM><<<ncb + nob, 256, 0, st>>>(X, dts, small_step, epssm, resm, coef_prev, ncb, wold, ddx)
                if (first) {
                    if constexpr (!E) {
                        if (sml == 2) {
                            tme ? MPAS_ACO(true, true, 2) : MPAS_ACO(true, false, 2);
                            return;
                        }
                    }
                    if (tme) sml ? MPAS_ACO(true, true, 1) : MPAS_ACO(true, true, 0);
                    else sml ? MPAS_ACO(true, false, 1) : MPAS_ACO(true, false, 0);
                } else {
                    if (tme) MPAS_ACO(false, true, false);
                    else MPAS_ACO(false, false, false);
                }
#undef MPAS_ACO
            };
            auto go_ts = [&](auto ex) {
                if (X.selfc) go_t(ex, std::true_type{});
                else go_t(ex, std::false_type{});
            };
            if (exact) go_ts(std::true_type{});
            else go_ts(std::false_type{});
            return;
        }
        auto go = [&](auto ex, auto sf, auto md) {
            constexpr bool E = decltype(ex)::value, SF = decltype(sf)::value;
            constexpr int M = decltype(md)::value;
#define MPAS_AC(FI, MP, MM, TM, SM) \
    k_acoustic<LP, E, SF, FI, MP, MM, TM, SM><<<grid, 256, 0, st>>>(X, dts, small_step, epssm, resm, coef_prev, ncb, wold, ddx)
            if constexpr (M == 0) {
                if (X.physics) {
                    if (first) MPAS_AC(true, true, 0, false, false);
                    else MPAS_AC(false, true, 0, false, false);
                    return;
                }
                if (tme) first ? MPAS_AC(true, false, 0, true, false) : MPAS_AC(false, false, 0, true, false);
                else first ? MPAS_AC(true, false, 0, false, false) : MPAS_AC(false, false, 0, false, false);
            } else {
                if (first) {
                    if constexpr (!E) {
                        if (sml == 2) {
                            tme ? MPAS_AC(true, false, M, true, 2) : MPAS_AC(true, false, M, false, 2);
                            return;
                        }
                    }
                    if (tme) sml ? MPAS_AC(true, false, M, true, 1) : MPAS_AC(true, false, M, true, 0);
                    else sml ? MPAS_AC(true, false, M, false, 1) : MPAS_AC(true, false, M, false, 0);
                } else {
                    if (tme) MPAS_AC(false, false, M, true, false);
                    else MPAS_AC(false, false, M, false, false);
                }
            }
#undef MPAS_AC
        };
        auto go_m = [&](auto ex, auto sf) {
            if (mode == 1) go(ex, sf, std::integral_constant<int, 1>{});
            else if (mode == 2) go(ex, sf, std::integral_constant<int, 2>{});
            else go(ex, sf, std::integral_constant<int, 0>{});
        };
        auto go_s = [&](auto ex) {
            if (X.selfc) go_m(ex, std::true_type{});
            else go_m(ex, std::false_type{});
        };
        if (exact) go_s(std::true_type{});
        else go_s(std::false_type{});
        if (mode == 2 && nob) {
            if (tme) k_acoustic_orph<LP, true><<<nob, 256, 0, st>>>(X, coef_prev);
            else k_acoustic_orph<LP, false><<<nob, 256, 0, st>>>(X, coef_prev);
        }
    };
    // (ru_p at the edges of owned cells only; MODE 2 also div at their cells -- X_dvB, the
    // previous substep's; SML u_tend at the edges of owned cells)
    if (mode == 2 && sml == 1) HALO_RUN_R1(S, st, run, F_ru_p, F_ru_p, F_theta_m, X_dvB, F_u_tend);
    else if (mode == 2) HALO_RUN_R1(S, st, run, F_ru_p, F_ru_p, F_theta_m, X_dvB);
    else if (sml == 1) HALO_RUN_R1(S, st, run, F_ru_p, F_ru_p, F_theta_m, F_u_tend);
    else HALO_RUN_R1(S, st, run, F_ru_p, F_ru_p, F_theta_m);
    if (mode == 0 || (wold & 1)) HALO_WROTE(S, F_rtheta_pp_old);
    if (!(mode && (wold & 2))) HALO_WROTE(S, F_rho_pp, F_rtheta_pp, F_rw_p, F_wwAvg);  // (wold bit 1: not stored)
    if (sml) HALO_WROTE(S, F_w);
    if (mode) HALO_WROTE(S, X_dvA);
    // MODE 2: the damped ru_p of every edge an owned cell owns (X_eown) -- the owned edges
    // and, the owned cells coming first in the local numbering, the ghost edges of owned
    // cells -- from the fresh ru_p and div there: fresh on the ring-1 ghost edges
    if (mode == 2 && S.halo) S.halo->fresh_ring1({X_rupB});
    return hipGetLastError();
}
hipError_t launch_acoustic(const DevState& S, hipStream_t st, double dts, int small_step, int exact, int mode,
                           double coef_prev, int tme, int sml, int wold, int ddx, int mdamp, int rudone) {
    MPAS_LP_DISPATCH(S.LP, acoustic_lp, S, st, dts, small_step, exact, mode, coef_prev, tme, sml, wold, ddx, mdamp,
                     rudone);
}
template <int LP>
static hipError_t hf_ac_vc_lp(const DevState& S, hipStream_t st, double dts, int small_step, int exact,
                              double coef_prev, int wold, int ddx) {
    if (S.physics || S.halo || small_step == 0 || S.epw != 2) return hipErrorInvalidValue;
    const double epssm = kEpssm, resm = (1.0 - epssm) / (1.0 + epssm);
    const int ncb = col_blocks<LP>(S, KC);
    const int nb1 = ncb + (S.n_orph + 256 / LP - 1) / (256 / LP);
    const int nv = col_blocks_n<LP, 2>(S, KV), nb2 = nv + col_blocks_n<LP, 2>(S, KC);
    if (!ncb || !nb2) return hipErrorInvalidValue;
    const int grid = nb1 + nb2;
    if (exact) {
        if (S.selfc) k_hf_ac_vc<LP, true, true, 2><<<grid, 256, 0, st>>>(S, dts, small_step, epssm, resm, coef_prev, ncb, nb1, nv, wold, ddx);
        else k_hf_ac_vc<LP, true, false, 2><<<grid, 256, 0, st>>>(S, dts, small_step, epssm, resm, coef_prev, ncb, nb1, nv, wold, ddx);
    } else {
        if (S.selfc) k_hf_ac_vc<LP, false, true, 2><<<grid, 256, 0, st>>>(S, dts, small_step, epssm, resm, coef_prev, ncb, nb1, nv, wold, ddx);
        else k_hf_ac_vc<LP, false, false, 2><<<grid, 256, 0, st>>>(S, dts, small_step, epssm, resm, coef_prev, ncb, nb1, nv, wold, ddx);
    }
    return hipGetLastError();
}
hipError_t launch_hf_acoustic_solve_vc(const DevState& S, hipStream_t st, double dts, int small_step, int exact,
                                       double coef_prev, int wold, int ddx) {
    MPAS_LP_DISPATCH(S.LP, hf_ac_vc_lp, S, st, dts, small_step, exact, coef_prev, wold, ddx);
}

}  // namespace mpas
