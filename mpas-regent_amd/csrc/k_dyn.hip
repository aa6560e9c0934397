// k_dyn.hip -- atm_compute_dyn_tend_work (dynamics_tasks.rg:814-1480), the north-star
// kernel, for gfx950.  One wavefront (LP lanes) per cell/edge/vertex column, lane k =
// level k; neighbour columns are contiguous 8*(L+1)-byte gathers; vertical stencils
// (wduz, wdwz, wdtz, k+-1 reads) are lane shuffles.
//
// The reference's ~20 loop nests fold into the global barriers the data flow needs:
//   A  cells    kdiff (rk0, Q11: own level only), h_divergence, tend_rho + dpdz (rk0),
//               wc = w after the zeroing, horizontal advection (Q13) and curvature
//   B  edges    tend_u_euler pressure gradient (rk0), wduz (in-lane), tend_u, q (Q10),
//               ke gradient, curvature (Q12), delsq_u + del2 (rk0), Rayleigh, and, when
//               no del4 follows, tend_u += tend_u_euler + tend_ru_physics; also the
//               per-edge theta reconstruction flux_arr (F) used by E
//   C  rk0      vertices: delsq_vorticity; cells: delsq_divergence, delsq_w + del2 of
//               tend_w_euler, delsq_theta + del2 of tend_theta_euler
//   D  rk0+del4 edges: del4 of tend_u_euler, tend_u finish
//   E  cells    del4 of w/theta (rk0), wdwz (in-lane), w scaling (Q14), buoyancy (rk0),
//               theta advection (F of the cell's edges), perturbation flux (rk>0),
//               wdtz (Q15, in-lane), tend_theta finish
// rk_step > 0 runs A, B, E.
// MD (option physics = 2, the MPAS dynamics; oracle dyn_tend_impl with mpas = 1): the w
// tendency goes to tend_w and is computed from the state w, which dyn_tend no longer
// touches (Q8): B forms each edge's w reconstruction flux_arr (Fw, every edge: Q13) beside
// the theta one (F), E accumulates it over the cell's edges, scales by invAreaCell, adds the
// curvature and the vertical flux (Q14); C mixes the state w; A skips wc; q is summed once
// (Q10), the curvature is -A - B (Q12), the top wduz/wdwz/wdtz are 0, wdtz is MPAS-A's
// 3rd-order flux (Q15), tend_rho keeps the physics term outside the flux divergence.
// Scratch the reference writes to fields (flux_arr,
// ru_edge_w, wduz, q, wdwz, wdtz, u_mix) stays in registers; only their level-L
// slots, which the reference never writes, are read from HBM.
//
// Memory-level parallelism: every loop over a connectivity list first issues the
// loads of the first NF/QF/AF entries unconditionally (padding ids are valid), then
// accumulates in the reference's order; longer lists finish in a generic tail loop.
#include "k_cols.h"
#include "mpas_dev.h"
#include "mpas_halo.h"

#include <type_traits>

namespace mpas {

__device__ __forceinline__ double dmin_(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double dmax_(double a, double b) { return a > b ? a : b; }

__device__ __forceinline__ double flux4(double q_im2, double q_im1, double q_i, double q_ip1, double ua) {
    return ua * (7. * (q_i + q_im1) - (q_ip1 + q_im2)) / 12.0;
}
__device__ __forceinline__ double flux3(double q_im2, double q_im1, double q_i, double q_ip1, double ua, double coef3) {
    return flux4(q_im2, q_im1, q_i, q_ip1, ua) + coef3 * fabs(ua) * ((q_ip1 - q_im2) - 3. * (q_i - q_im1)) / 12.0;
}

struct DynK {
    int rk_step, horiz_mixing, rayleigh, exact_q, tme, cp, d4o, vB;
    double cs_l2, cap, cam_coef, h4, inv_r_earth, r_earth, rayleigh_inv, prandtl_inv;
    double h4d;  // DIN: the h4 of the rk_step 0 call whose del4 of tend_u_euler this call applies
    double rud;  // (option mru, the MPAS dynamics, fast path) the stage's dts: the kernel forming the final
                 // tend_u also stores the first substep's ru_p = dts tend_u and ruAvg = ru_p
    int nhd;     // (option ntu, rk_step 0 with B forming no tend_u) A's h_divergence is dead: not stored
};

// option mru (the MPAS dynamics, atm_srk3 fast path): the stage's first acoustic substep begins with
// ru_p = dts tend_u, ruAvg = ru_p on every edge (k_acoustic_ru FIRST, :1581-1613 restored, Q18) -- formed
// here by the kernel that forms the final tend_u, from the value it stores (the same expressions; level
// L and the padding as k_acoustic_ru stores them), and that launch goes
template <int LP>
__device__ __forceinline__ void ru_first(const DevState& S, double dts, int e, int k, int L, double tu) {
    const size_t pL = (size_t)e * LP + lpos(LP, L);
    const double rp0 = ldc(fd(S, F_ru_p) + pL), ra0 = ldc(fd(S, F_ruAvg) + pL);
    const double rp = dts * tu;
    colk(fw(S, F_ru_p), e) = KEEPW(rp, rp0);
    colk(fw(S, F_ruAvg), e) = KEEPW(rp, ra0);
}


// ------------------------------------------------------------------------ A (cells)
// SETUP (atm_srk3 stage 0 beside the fused setup launch, option hfuse): rho_p_save and qtot
// are being written by that launch -- rho_p_save = rho_p and qtot = 0 at every level A
// stores (k != L) -- so A takes rho_p and 0.0 instead: the same values
template <int LP, bool RK0, bool MD, bool SETUP = false>
__device__ __forceinline__ void dyn_A_body(const DevState& S, const DynK& a, Blk bk) {
    ColMap<LP> m(S, KC, bk);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO) return;
    const size_t p = (size_t)c * LP + lpos(LP, k);
    constexpr bool rk0 = RK0;
    const bool live = k <= L;
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* eocs = fd(S, F_edgesOnCell_sign) + (size_t)c * 10;
    const double* cdv = fd(S, X_ce_dv) + (size_t)c * 10;
    const double *u = fd(S, F_u), *v = fd(S, F_v), *ru = fd(S, F_ru);
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k], rdzw = fd(S, F_rdzw)[k];
    const bool smag = rk0 && a.horiz_mixing == 0;
    // the kept level-L values of the stored columns (keep tails, mpas_dev.h), issued ahead
    const double kl_kd = keepv<LP>(S, F_kdiff, KC, c), kl_hd = keepv<LP>(S, F_h_divergence, KC, c);
    const double kl_tr = keepv<LP>(S, F_tend_rho, KC, c), kl_dp = keepv<LP>(S, F_dpdz, KC, c);

    int e_[NF];
    double ru_[NF], u_[NF], v_[NF], eocs_[NF], cdv_[NF], wfl[2];
    row_ld(fd(S, X_wfl) + (size_t)c * 2, wfl);
    int c1_[NF], c2_[NF];  // unused: the record's edges and count
    const int ne = cell_rec<false>(S, c, e_, c1_, c2_);
    row_ld(eocs, eocs_);
    row_ld(cdv, cdv_);
#pragma unroll
    for (int i = 0; i < NF; i += 2) gather2s<LP>(ru, e_[i], e_[i + 1], k, ru_[i], ru_[i + 1]);
#pragma unroll
    for (int i = 0; i < NF; i++) ru_[i] = ldz(live, ru_[i]);
    if (smag) {
#pragma unroll
        for (int i = 0; i < NF; i += 2) {
            gather2s<LP>(u, e_[i], e_[i + 1], k, u_[i], u_[i + 1]);
            gather2s<LP>(v, e_[i], e_[i + 1], k, v_[i], v_[i + 1]);
        }
#pragma unroll
        for (int i = 0; i < NF; i++) {
            u_[i] = ldz(live, u_[i]);
            v_[i] = ldz(live, v_[i]);
        }
    }
    double rw, rz, urz, urm;
    col_rd2<LP>(fd(S, F_rw), fd(S, F_rho_zz), c, k, L, rw, rz);
    col_rd2<LP>(fd(S, F_uReconstructZonal), fd(S, F_uReconstructMeridional), c, k, L, urz, urm);
    // rk0 loads of the tend_rho/dpdz section, ahead of the stores (aliasing for the compiler)
    double trp = 0.0, qt = 0.0, rb = 0.0, rps = 0.0;
    if (rk0) {
        trp = colk(fd(S, F_tend_rho_physics), c);
        qt = SETUP ? 0.0 : colk(fd(S, F_qtot), c);
        rb = colk(fd(S, F_rho_base), c);
        rps = colk(fd(S, SETUP ? F_rho_p : F_rho_p_save), c);
    }

    // ---- kdiff (:858-917)
    if (rk0 && (a.horiz_mixing == 0 || a.horiz_mixing == 1 || a.cam_coef > 0.0)) {
        double kd;
        if (a.horiz_mixing == 0) {
            const double* defa = fd(S, F_defc_a) + (size_t)c * 10;
            const double* defb = fd(S, F_defc_b) + (size_t)c * 10;
            double d_diag = 0.0, d_off_diag = 0.0, defa_[NF], defb_[NF];
            row_ld(defa, defa_);
            row_ld(defb, defb_);
#pragma unroll
            for (int i = 0; i < NF; i++) {
                d_diag = add_if(i < ne, d_diag, defa_[i] * u_[i] - defb_[i] * v_[i]);
                d_off_diag = add_if(i < ne, d_off_diag, defb_[i] * u_[i] + defa_[i] * v_[i]);
            }
            for (int i = NF; i < ne; i++) {
                int e = eoc[i];
                double ue = col_rd<LP>(u, e, k, L), ve = col_rd<LP>(v, e, k, L);
                d_diag += defa[i] * ue - defb[i] * ve;
                d_off_diag += defb[i] * ue + defa[i] * ve;
            }
            kd = dmin_(a.cs_l2 * sqrt(d_diag * d_diag + d_off_diag * d_off_diag), a.cap);
        } else if (a.horiz_mixing == 1) {
            kd = 0.0;
        } else {
            kd = col_rd<LP>(fd(S, F_kdiff), c, k, L);
        }
        if (a.cam_coef > 0.0 && k >= L - 2 && k <= L) {
            int pw = k - (L - 2);
            kd = dmax_(kd, (pw == 0 ? 1.0 : 2.0) * 2.0833 * kLenDisp * a.cam_coef);
        }
        colk(fw(S, F_kdiff), c) = KEEPW(kd, kl_kd);
    }

    // ---- h_divergence (:924-938)
    double hd = 0.0;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        double edge_sign = eocs_[i] * cdv_[i];
        hd = add_if(i < ne, hd, edge_sign * ru_[i]);
    }
    for (int i = NF; i < ne; i++) {
        double edge_sign = eocs[i] * cdv[i];
        hd += edge_sign * col_rd<LP>(ru, eoc[i], k, L);
    }
    hd *= fd(S, F_invAreaCell)[c];
    // the w scratch wc (below) is formed here at rk_step 0, where C gathers it; at rk_step > 0
    // E, its only reader, forms it from the same operands (wc_body), so A reads ru alone
    constexpr bool WC = !MD && RK0;
    if (!WC) colk(fw(S, F_h_divergence), c) = KEEPW(hd, kl_hd);  // (else paired below)

    // ---- tend_rho, dpdz (:942-951)
    const double rw_p1 = lvl_up<LP>(rw, k);
    if (rk0)  // (paired 16-B store, every lane)
        put2f<LP>(fw(S, F_tend_rho), c, fw(S, F_dpdz), c, k,
                 KEEPW(MD ? -hd - rdzw * (rw_p1 - rw) + trp : -hd - rdzw * (rw_p1 - rw + trp), kl_tr),
                 KEEPW(-kGravity * (rb * (qt) + rps * (1.0 + qt)), kl_dp));

    // ---- w: zeroing (:1170), horizontal advection (:1174-1205, Q13), curvature (:1208-1218)
    // After the zeroing every w(cell, k<L) read by flux_arr is exactly 0.0 (the zero
    // slot is 0 too), so flux_arr = sum_j scalar_weight_j * 0.0 over the advCells of the
    // cell's LAST edge (flux_arr and ru_edge_w are overwritten per edge): +0.0, or NaN
    // where a weight is not finite.  It depends only on the mesh and on
    // copysign(1, ru_edge_w), so k_prepare evaluates it literally for both signs
    // (X_wfl); the sum over the edges is evaluated literally here, so that non-finite
    // values propagate as in the reference.
    double ru_l = 0.0;
#pragma unroll
    for (int i = 0; i < NF; i++)
        if (i == ne - 1) ru_l = ru_[i];
    if (ne > NF) ru_l = col_rd<LP>(ru, eoc[ne - 1], k, L);
    const double ru_lm = lvl_dn<LP>(ru_l, k);
    const double rz_m = lvl_dn<LP>(rz, k), urz_m = lvl_dn<LP>(urz, k), urm_m = lvl_dn<LP>(urm, k);
    if constexpr (!WC) return;  // (MD: the w tendency is formed in E from the state w)
    // (every lane goes on: the scratch wc is stored whole, 0.0 from level L up)
    double w0 = 0.0;
    if (ne > 0 && k > 0) {
        double ru_edge_w = fzm * ru_l + fzp * ru_lm;
        const double flux_arr = copysign(1.0, ru_edge_w) > 0.0 ? wfl[0] : wfl[1];
#pragma unroll
        for (int i = 0; i < NF; i++) w0 = sub_if(i < ne, w0, eocs_[i] * ru_edge_w * flux_arr);
        for (int i = NF; i < ne; i++) w0 -= eocs[i] * ru_edge_w * flux_arr;
    }
    double wc = w0;
    if (k > 0) {
        const double coslat = fd(S, X_cosLatCell)[c];
        double aa = fzm * urz + fzp * urz_m;
        double bb = fzm * urm + fzp * urm_m;
        wc += (rz * fzm + rz_m * fzp) * ((aa * aa) + (bb * bb)) / a.r_earth +
              2.0 * kOmega * coslat * (fzm * urz + fzp * urz_m) * (rz * fzm + rz_m * fzp);
    }
    if (a.nhd) colk(fw(S, X_wc), c) = k < L ? wc : 0.0;  // (option ntu: h_divergence read by no kernel)
    else put2f<LP>(fw(S, F_h_divergence), c, fw(S, X_wc), c, k, KEEPW(hd, kl_hd), k < L ? wc : 0.0);
}
template <int LP, bool RK0, bool MD>
__global__ __launch_bounds__(256) void k_dyn_A(DevState S, DynK a) {
    dyn_A_body<LP, RK0, MD>(S, a, this_blk());
}

// ------------------------------------------------------------------------ B (edges)
// (B's stores leave level L unwritten, as the reference: the keep tails of mpas_dev.h measured
// no gain on this gather-bound kernel and cost its DIN form 5-9 %, profiles/r05/keep_tails)
// DIN (rk_step > 0, option "defer4"): the previous rk_step 0 call left tend_u_euler without
// its del4 part (kernel D, skipped there); this kernel applies D's statements to the
// tend_u_euler it reads -- the same operands in the same order, so the same bits -- and
// stores the result.  D's tend_u of that call is dead in atm_srk3 (this kernel writes tend_u)
// (DIN at LP = 64: capped at 128 VGPRs, the 4 waves per SIMD of the plain rk_step > 0 kernel;
// uncapped the compiler takes 132 and 3 waves: +35 %, profiles/r04.  At LP < 64 the cap made
// it spill ~78 VGPRs.  The MPAS dynamics' B (139-147 VGPRs) under the same cap spills 8-32
// and runs 7-80 % slower: profiles/r04/md_cap_tried)
// NOF (option "bsplit", fast path): the per-edge theta flux H (and the MD w flux) are left to
// k_dyn_Bf, an edge kernel of their own: this one skips the advCells gathers.  Also (option
// "etile", either path) when the tiled E forms each edge's flux itself: no X_F at all
// NTU (atm_srk3, reference semantics, rk_step 0 with defer4 out): the call's tend_u is dead -- the next
// stage's B rewrites it and no task in between reads it (set_smlstep reads u_tend, Q2; the acoustic
// step ru_p, Q18) -- so, as D's tend_u there, it is not formed at all: no wduz, q, ke gradient,
// curvature or Rayleigh term, none of their gathers (u and pv_edge over edgesOnEdge, rw, w, ke,
// h_divergence at the cells, tend_ru_physics).  The kernel keeps what later kernels read:
// tend_u_euler (the pressure gradient and del2, :964-970, :1030-1048), delsq_u, the theta flux,
// setup's copies
template <int LP, bool RK0, bool MD, bool HF, bool DIN = false, bool NOF = false, bool NTU = false>
__global__ __launch_bounds__(256, LP == 64 && DIN ? 4 : 1) void k_dyn_B(DevState S, DynK a) {
    static_assert(!NTU || !MD, "the dead tend_u: reference semantics");
    ColMap<LP> m(S, KE);
    const int L = S.L, k = m.k, e = m.ent;
    if (e >= S.nEO) return;
    const size_t p = (size_t)e * LP + lpos(LP, k);
    constexpr bool rk0 = RK0;
    const bool live = k <= L;
    // the edge's index lists in one record (X_eB): one scalar round trip
    int rec[24];
    row_ld(fi(S, X_eB) + (size_t)e * 24, rec);
    const int cell1 = rec[0], cell2 = rec[1];
    const double invDc = fd(S, F_invDcEdge)[e];
    const double *u_f = fd(S, F_u), *pv_f = fd(S, F_pv_edge), *tm_f = fd(S, F_theta_m);
    const size_t p1 = (size_t)cell1 * LP + lpos(LP, k), p2 = (size_t)cell2 * LP + lpos(LP, k);

    // ---- issue every independent load of the column first (gather2: two columns per load
    // instruction; the raw halves, swapped after the scheduling barrier below)
    double u, ru_e, rw1, rw2, w1, w2, rho_edge, pv;
    const double2 z2 = make_double2(0.0, 0.0);
    const double2 g_uru = gather2_ld<LP>(u_f, e, fd(S, F_ru), e, k);
    const double2 g_rw = NTU ? z2 : gather2s_ld<LP>(fd(S, F_rw), cell1, cell2, k);
    const double2 g_w = NTU ? z2 : gather2s_ld<LP>(fd(S, F_w), cell1, cell2, k);
    const double2 g_rp = NTU ? make_double2(colk(fd(S, F_rho_edge), e), 0.0) : gather2_ld<LP>(fd(S, F_rho_edge), e, pv_f, e, k);
    // No level masks (ldz) in this kernel: lanes k >= L store nothing (k > L: PADW
    // zeros), so a value used in its own lane needs none, and the vertical shuffles
    // (lvl_up/dn) of u and w bring lanes k <= L only levels <= L -- exactly what the
    // masks kept.  (Each ldz is two v_cndmask per double; B was half VALU-bound.)
    // one value: the level-L slot (MD: MPAS-A's wduz(nVertLevels+1) = 0)
    const double wduzL = (MD || NTU) ? 0.0 : fd(S, F_wduz)[(size_t)e * LP + lpos(LP, L)];
    const int neoe = rec[21];
    const int* eoe = fi(S, F_edgesOnEdge) + (size_t)e * 20;
    const double* woe = fd(S, F_weightsOnEdge) + (size_t)e * 20;
    int ee_[QF];
    double ue_[QF], pve_[QF], woe_[QF];
#pragma unroll
    for (int j = 0; j < QF; j++) ee_[j] = rec[2 + j];
    row_ld(woe, woe_);
    const bool kl = k < L;
    double2 g_ue[QF / 2], g_pve[QF / 2];
#pragma unroll
    for (int j = 0; j < QF; j += 2) {
        g_ue[j / 2] = NTU ? z2 : gather2s_ld<LP>(u_f, ee_[j], ee_[j + 1], k);
        g_pve[j / 2] = NTU ? z2 : gather2s_ld<LP>(pv_f, ee_[j], ee_[j + 1], k);
    }
    // theta reconstruction at this edge (:1333-1340), consumed by E
    const int na = rec[22];
    const int* ad = fi(S, F_advCellsForEdge) + (size_t)e * 15;
    const double* ac = fd(S, F_adv_coefs) + (size_t)e * 15;
    const double* ac3 = fd(S, F_adv_coefs_3rd) + (size_t)e * 15;
    int ad_[AF];
    double tv_[AF], ac_[AF], ac3_[AF];
#pragma unroll
    for (int j = 0; j < AF; j++) ad_[j] = rec[12 + j];
    row_ld(ac, ac_);
    row_ld(ac3, ac3_);
    static_assert(AF == 9, "tv_ pairing below");
    double tr_phys;
    double2 g_tv[AF / 2], g_tvl = make_double2(0.0, 0.0);
    const double trp_in = (NOF && !NTU) ? colk(fd(S, F_tend_ru_physics), e) : 0.0;
    if constexpr (!NOF) {
#pragma unroll
        for (int j = 0; j < AF - 1; j += 2) g_tv[j / 2] = gather2s_ld<LP>(tm_f, ad_[j], ad_[j + 1], k);
        g_tvl = NTU ? make_double2(colk(tm_f, ad_[AF - 1]), 0.0) : gather2_ld<LP>(tm_f, ad_[AF - 1], fd(S, F_tend_ru_physics), e, k);
    }

    // MD: the state w at the advCells, for the w reconstruction flux_arr of this edge
    double wv_[AF];
    double2 g_wv[AF / 2];
    if constexpr (MD && !NOF) {
        const double* w_f = fd(S, F_w);
#pragma unroll
        for (int j = 0; j < AF - 1; j += 2) g_wv[j / 2] = gather2s_ld<LP>(w_f, ad_[j], ad_[j + 1], k);
        wv_[AF - 1] = colk(w_f, ad_[AF - 1]);
    }
    // loads of the later sections, also ahead of every store (a store could alias them
    // for the compiler, which would then issue them only after it)
    const double *ke_f = fd(S, F_ke), *hd_f = fd(S, F_h_divergence);
    double ke1, ke2, hd1, hd2;
    const double2 g_ke = NTU ? z2 : gather2s_ld<LP>(ke_f, cell1, cell2, k);
    const double2 g_hd = NTU ? z2 : gather2s_ld<LP>(hd_f, cell1, cell2, k);
    // (the rk0-only loads stay in their section: hoisted they cost more in occupancy,
    // 138 VGPRs, than the second memory round trip)
    // HF (fast path): E's per-edge theta flux H formed here (rk > 0: with the
    // perturbation flux, which needs ru_save at the edge and theta_m_save at its cells)
    double tue_in = 0.0, rus_e = 0.0, ts1 = 0.0, ts2 = 0.0;
    double2 g_tr = make_double2(0.0, 0.0), g_ts = make_double2(0.0, 0.0);
    if constexpr (!RK0) {
        if constexpr (HF && !NOF) {
            g_tr = gather2_ld<LP>(fd(S, F_tend_u_euler), e, fd(S, F_ru_save), e, k);
            g_ts = gather2s_ld<LP>(fd(S, F_theta_m_save), cell1, cell2, k);
        } else {
            tue_in = colk(fd(S, F_tend_u_euler), e);
        }
    }
    double2 g_dd = make_double2(0.0, 0.0), g_dv = make_double2(0.0, 0.0);
    if constexpr (DIN) {
        const int vertex1 = fi(S, F_verticesOnEdge)[(size_t)e * 2], vertex2 = fi(S, F_verticesOnEdge)[(size_t)e * 2 + 1];
        g_dd = gather2s_ld<LP>(fd(S, F_delsq_divergence), cell1, cell2, k);
        g_dv = gather2s_ld<LP>(fd(S, F_delsq_vorticity), vertex1, vertex2, k);
    }
    // NTU: the rk0 section's loads join the first batch (the tend_u loads they replace freed the registers)
    double2 g0[7];
    if constexpr (NTU && RK0) {
        const int vertex1 = fi(S, F_verticesOnEdge)[(size_t)e * 2], vertex2 = fi(S, F_verticesOnEdge)[(size_t)e * 2 + 1];
        g0[0] = gather2_ld<LP>(fd(S, F_cqu), e, fd(S, F_zxu), e, k);
        g0[1] = gather2s_ld<LP>(fd(S, F_pressure_p), cell1, cell2, k);
        g0[2] = gather2s_ld<LP>(fd(S, F_zz), cell1, cell2, k);
        g0[3] = gather2s_ld<LP>(fd(S, F_dpdz), cell1, cell2, k);
        g0[4] = gather2s_ld<LP>(fd(S, F_divergence), cell1, cell2, k);
        g0[5] = gather2s_ld<LP>(fd(S, F_vorticity), vertex1, vertex2, k);
        g0[6] = gather2s_ld<LP>(fd(S, F_kdiff), cell1, cell2, k);
    }
    // every load above in flight before the first swap consumes one (the per-level
    // coefficients after it: cache hits, no registers held across the batch)
    __builtin_amdgcn_sched_barrier(0);
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k], rdzw = fd(S, F_rdzw)[k];
    g2_fin<LP>(g_uru, u, ru_e);
    if constexpr (NTU) {  // (not loaded as pairs: no swaps)
        rw1 = rw2 = w1 = w2 = pv = 0.0;
        rho_edge = g_rp.x;
#pragma unroll
        for (int j = 0; j < QF; j++) ue_[j] = pve_[j] = 0.0;
    } else {
        g2_fin<LP>(g_rw, rw1, rw2);
        g2_fin<LP>(g_w, w1, w2);
        g2_fin<LP>(g_rp, rho_edge, pv);
#pragma unroll
        for (int j = 0; j < QF; j += 2) {
            g2_fin<LP>(g_ue[j / 2], ue_[j], ue_[j + 1]);
            g2_fin<LP>(g_pve[j / 2], pve_[j], pve_[j + 1]);
        }
    }
    if constexpr (NOF) {
        tr_phys = trp_in;
    } else {
#pragma unroll
        for (int j = 0; j < AF - 1; j += 2) g2_fin<LP>(g_tv[j / 2], tv_[j], tv_[j + 1]);
        if constexpr (NTU) {
            tv_[AF - 1] = g_tvl.x;
            tr_phys = 0.0;
        } else {
            g2_fin<LP>(g_tvl, tv_[AF - 1], tr_phys);
        }
    }
    if constexpr (MD && !NOF) {
#pragma unroll
        for (int j = 0; j < AF - 1; j += 2) g2_fin<LP>(g_wv[j / 2], wv_[j], wv_[j + 1]);
    }
    if constexpr (NTU) {
        ke1 = ke2 = hd1 = hd2 = 0.0;
    } else {
        g2_fin<LP>(g_ke, ke1, ke2);
        g2_fin<LP>(g_hd, hd1, hd2);
    }
    if constexpr (!RK0 && HF && !NOF) {
        g2_fin<LP>(g_tr, tue_in, rus_e);
        if (a.cp) rus_e = ru_e;  // (the copy below is setup's: ru_save = ru, read after it)
        g2_fin<LP>(g_ts, ts1, ts2);
    }
    if constexpr (DIN) {  // kernel D of the rk_step 0 call (:1132-1150), deferred here
        double dd1, dd2, dv1, dv2;
        g2_fin<LP>(g_dd, dd1, dd2);
        g2_fin<LP>(g_dv, dv1, dv2);
        const double u_mix_scale = fd(S, F_meshScalingDel4)[e] * a.h4d;
        const double r_dc = u_mix_scale * kDel4uDivFactor * invDc;
        const double r_dv = u_mix_scale * dmin_(fd(S, F_invDvEdge)[e], 4 * invDc);
        const double u_diffusion = rho_edge * ((dd2 - dd1) * r_dc - (dv2 - dv1) * r_dv);
        tue_in -= u_diffusion;
    }

    double tend_u = 0.0, w1p = 0.0, w2p = 0.0, wduz = 0.0, wduz_p = 0.0;
    if constexpr (!NTU) {
        const double u_m = lvl_dn<LP>(u, k), u_m2 = lvl_dn2<LP>(u, k), u_p = lvl_up<LP>(u, k);
        w1p = lvl_up<LP>(w1, k), w2p = lvl_up<LP>(w2, k);
        // ---- wduz (:972-980); level L is never written by the reference: read it
        if (k == 1 || k == L - 1) wduz = 0.5 * (rw1 + rw2) * (fzm * u + fzp * u_m);
        if (k > 1 && k < L - 1) wduz = flux3(u_m2, u_m, u, u_p, 0.5 * (rw1 + rw2), 1.0);
        if (k == L) wduz = wduzL;
        wduz_p = lvl_up<LP>(wduz, k);
    }
    // Every lane goes on (gather2 below needs all of them); level L is not stored, the
    // padding levels get 0.0 (PADW), the scratch F is stored whole.

    double Hv = 0.0, dsq = 0.0;  // HF: the values of the paired stores at the end
    if constexpr (!NOF) {  // flux_arr of this edge
        const double sg = copysign(1.0, ru_e);
        double flux_arr = 0.0;
#pragma unroll
        for (int j = 0; j < AF; j++) {
            double scalar_weight = ac_[j] + sg * ac3_[j];
            flux_arr = add_if(j < na, flux_arr, scalar_weight * tv_[j]);
        }
        for (int j = AF; j < na; j++) {
            double scalar_weight = ac[j] + sg * ac3[j];
            flux_arr += scalar_weight * colk(tm_f, ad[j]);
        }
        if constexpr (HF) {  // H = ru F (+ dvEdge (ru_save - ru) theta_m_save at the edge, rk > 0)
            double h = ru_e * flux_arr;
            if constexpr (!RK0) h += fd(S, F_dvEdge)[e] * ((rus_e - ru_e) * 0.5 * (ts2 + ts1));
            Hv = kl ? h : 0.0;  // (stored with tend_u / delsq_u below: paired stores)
        } else {
            colk(fw(S, X_F), e) = kl ? flux_arr : 0.0;
        }
    }
    if constexpr (MD && !NOF) {  // flux_arr of the w advection at this edge (:1174-1197, every edge)
        const double ru_edge_w = fzm * ru_e + fzp * lvl_dn<LP>(ru_e, k);
        const double sg = copysign(1.0, ru_edge_w);
        double flux_arr = 0.0;
#pragma unroll
        for (int j = 0; j < AF; j++) {
            double scalar_weight = ac_[j] + sg * ac3_[j];
            flux_arr = add_if(j < na, flux_arr, scalar_weight * wv_[j]);
        }
        for (int j = AF; j < na; j++) {
            double scalar_weight = ac[j] + sg * ac3[j];
            flux_arr += scalar_weight * colk(fd(S, F_w), ad[j]);
        }
        // HF: the edge's whole horizontal w flux Hw = ru_edge_w flux_arr (E sums eocs Hw)
        colk(fw(S, X_Fw), e) = (k > 0 && kl) ? (HF ? ru_edge_w * flux_arr : flux_arr) : 0.0;
    }

    // ---- tend_u (:987-1007)
    if constexpr (!NTU) {
    tend_u = -rdzw * (wduz_p - wduz);
    double q = 0.0;
    if (a.exact_q && !MD) {
        for (int j = 0; j < neoe; j++) {  // Q10 literal: each term added nVertLevels times
            double ue = colk(u_f, eoe[j]);
            double pve = colk(pv_f, eoe[j]);
            for (int kk = 0; kk < L; kk++) {
                double workpv = 0.5 * (pv + pve);
                q += woe[j] * ue * workpv;
            }
        }
    } else {
        const double dL = MD ? 1.0 : (double)L;  // Q10 value, nVertLevels * term (MD: once)
#pragma unroll
        for (int j = 0; j < QF; j++) {
            double workpv = 0.5 * (pv + pve_[j]);
            q = add_if(j < neoe, q, (woe_[j] * ue_[j] * workpv) * dL);
        }
        for (int j = QF; j < neoe; j++) {
            double workpv = 0.5 * (pv + colk(pv_f, eoe[j]));
            q += (woe[j] * colk(u_f, eoe[j]) * workpv) * dL;
        }
    }
    tend_u += rho_edge * (q - (ke2 - ke1) * invDc) - u * 0.5 * (hd1 + hd2);
    // (rk_step > 0 only: at rk_step 0 the store would keep the compiler from issuing the rk0
    // section's loads below ahead of it)
    if (!RK0 && a.vB) {  // solve_diagnostics' v (:429-437; Q23: from i = 1) from the same u columns
        double vv = 0.0;
#pragma unroll
        for (int j = 1; j < QF; j++) vv = add_if(j < neoe, vv, woe_[j] * ue_[j]);
        for (int j = QF; j < neoe; j++) vv += woe[j] * colk(u_f, eoe[j]);
        if (k != L) colk(fw(S, F_v), e) = PADW(vv);
    }
    {  // curvature (:1011-1017, Q12 literal)
        // (ldc: mesh tables no step kernel writes -- not held behind the v store above)
        const double cosA = ldc(fd(S, X_cosAngleEdge) + e), cosL = ldc(fd(S, X_cosLatEdge) + e);
        const double cA = (2.0 * kOmega * cosA * cosL * rho_edge * 0.25 * (w1 + w1p + w2 + w2p));
        const double cB = (u * 0.25 * (w1 + w1p + w2 + w2p) * rho_edge * a.inv_r_earth);
        if (MD) tend_u = tend_u - cA - cB;
        else tend_u -= cA - cB;
    }
    }  // (!NTU)

    double tue;
    if (rk0) {
        const double *pp = fd(S, F_pressure_p), *zz = fd(S, F_zz), *dpdz = fd(S, F_dpdz);
        const double *div = fd(S, F_divergence), *vor = fd(S, F_vorticity), *kdiff = fd(S, F_kdiff);
        const int vertex1 = fi(S, F_verticesOnEdge)[(size_t)e * 2], vertex2 = fi(S, F_verticesOnEdge)[(size_t)e * 2 + 1];
        double cqu, zxu, pp1, pp2, zz1, zz2, dz1, dz2, dv1, dv2, vo1, vo2, kf1, kf2;
        if constexpr (NTU && RK0) {  // (loaded with the first batch)
            g2_fin<LP>(g0[0], cqu, zxu);
            g2_fin<LP>(g0[1], pp1, pp2);
            g2_fin<LP>(g0[2], zz1, zz2);
            g2_fin<LP>(g0[3], dz1, dz2);
            g2_fin<LP>(g0[4], dv1, dv2);
            g2_fin<LP>(g0[5], vo1, vo2);
            g2_fin<LP>(g0[6], kf1, kf2);
        } else {
            gather2<LP>(fd(S, F_cqu), e, fd(S, F_zxu), e, k, cqu, zxu);
            gather2s<LP>(pp, cell1, cell2, k, pp1, pp2);
            gather2s<LP>(zz, cell1, cell2, k, zz1, zz2);
            gather2s<LP>(dpdz, cell1, cell2, k, dz1, dz2);
            gather2s<LP>(div, cell1, cell2, k, dv1, dv2);
            gather2s<LP>(vor, vertex1, vertex2, k, vo1, vo2);
            gather2s<LP>(kdiff, cell1, cell2, k, kf1, kf2);
        }
        // ---- pressure gradient (:964-970)
        tue = -cqu * ((pp2 - pp1) * invDc / (0.5 * (zz2 + zz1)) - 0.5 * zxu * (dz1 + dz2));
        // ---- del2 (:1030-1048)
        const double r_dc = invDc;
        const double r_dv = dmin_(fd(S, F_invDvEdge)[e], 4 * r_dc);
        double u_diffusion = (dv2 - dv1) * r_dc - (vo2 - vo1) * r_dv;
        double delsq_u = 0.0;
        delsq_u += u_diffusion;
        if (HF) dsq = PADW(delsq_u);
        else if (k != L) colk(fw(S, F_delsq_u), e) = PADW(delsq_u);
        double kdiffu = 0.5 * (kf1 + kf2);
        tue += rho_edge * kdiffu * u_diffusion * fd(S, F_meshScalingDel2)[e];
    } else {
        tue = tue_in;
    }
    // ---- Rayleigh damping (:1152-1159)
    if (!NTU && a.rayleigh && k > L - kRayleighLevels + 1)
        tend_u -= rho_edge * u * (((double)k - (double)(L - kRayleighLevels)) * a.rayleigh_inv);
    if (a.tme) {  // X_tme for the stage's acoustic substeps: theta_m(cell2) + theta_m(cell1)
        double t2pt1;
        if (!NOF && na >= 2 && ad_[0] == cell1 && ad_[1] == cell2) {  // (the adv list starts with the two cells)
            t2pt1 = tv_[1] + tv_[0];
        } else {
            double t1, t2;
            gather2s<LP>(tm_f, cell1, cell2, k, t1, t2);
            t2pt1 = t2 + t1;
        }
        if (k != L) colk(fw(S, X_tme), e) = PADW(t2pt1);
    }
    // a.cp (atm_srk3 stage 0, option "fusecopy"): atm_rk_integration_setup's edge copies
    // (:758-761, every level but L) from the u and ru columns this kernel has loaded; no
    // task between setup and here reads ru_save or u_2 (dyn_tend reads ru_save at
    // rk_step > 0 only, after this kernel), and u / ru are not written in between
    if (a.cp) put2<LP>(fw(S, F_ru_save), e, fw(S, F_u_2), e, k, PADW(ru_e), PADW(u), k != L, k != L);
    if constexpr (HF) {  // every lane stores (paired 16-B stores); level L keeps its value
        double* Fo = fw(S, X_F);
        double* tuo = fw(S, F_tend_u);
        double* tueo = fw(S, F_tend_u_euler);
        if (rk0 && a.h4 > 0.0) {  // D finishes tend_u after the del4 part of tend_u_euler
            if (a.d4o) {  // (defer4: D runs in the next call's B; this tend_u is dead)
                if constexpr (NOF) put2<LP>(tueo, e, fw(S, F_delsq_u), e, k, PADW(tue), dsq, k != L, k != L);
                else put2<LP>(Fo, e, tueo, e, k, Hv, PADW(tue), true, k != L);
                if (!NOF && k != L) colk(fw(S, F_delsq_u), e) = dsq;
            } else {
                if constexpr (NOF) {
                    if (k != L) colk(fw(S, F_delsq_u), e) = dsq;
                } else {
                    put2<LP>(Fo, e, fw(S, F_delsq_u), e, k, Hv, dsq, true, k != L);
                }
                put2<LP>(tueo, e, tuo, e, k, PADW(tue), PADW(tend_u), k != L, k != L);
            }
        } else {
            if constexpr (NTU) {  // (the dead tend_u is not stored; the flux alone, whole)
                if constexpr (!NOF) colk(Fo, e) = Hv;
            } else {
                tend_u += tue + tr_phys;  // :1161-1163 (rk > 0: tue is the tend_u_euler read)
                if constexpr (NOF) {
                    if (k != L) colk(tuo, e) = PADW(tend_u);
                } else {
                    put2<LP>(Fo, e, tuo, e, k, Hv, PADW(tend_u), true, k != L);
                }
                if constexpr (MD) {  // (option mru; rp at level L and above is not the stored tend_u's: KEEPW)
                    if (a.rud != 0.0) ru_first<LP>(S, a.rud, e, k, L, PADW(tend_u));
                }
            }
            if (rk0) put2<LP>(tueo, e, fw(S, F_delsq_u), e, k, PADW(tue), dsq, k != L, k != L);
            if (DIN && k != L) colk(tueo, e) = PADW(tue);
        }
        return;
    }
    if (k == L) return;
    if (rk0 && a.h4 > 0.0) {  // D finishes tend_u after the del4 part of tend_u_euler
        colk(fw(S, F_tend_u_euler), e) = PADW(tue);
        if (!NTU && !a.d4o) colk(fw(S, F_tend_u), e) = PADW(tend_u);
    } else {
        if (rk0 || DIN) colk(fw(S, F_tend_u_euler), e) = PADW(tue);
        tend_u += tue + tr_phys;  // :1161-1163
        if (!NTU) colk(fw(S, F_tend_u), e) = PADW(tend_u);
    }
}

// option "bsplit" (fast path): B's per-edge theta flux H = ru F (+ dvEdge (ru_save - ru)
// theta_m_save at the edge, rk > 0) for E, and under the MPAS dynamics the w flux Hw, as an edge
// kernel of their own beside k_dyn_B<NOF>: the advCells gathers leave B's registers (the same
// expressions on the same values: the same bits)
template <int LP, bool RK0, bool MD>
__global__ __launch_bounds__(256) void k_dyn_Bf(DevState S, DynK a) {
    ColMap<LP> m(S, KE);
    const int L = S.L, k = m.k, e = m.ent;
    if (e >= S.nEO) return;
    int rec[24];
    row_ld(fi(S, X_eB) + (size_t)e * 24, rec);
    const int cell1 = rec[0], cell2 = rec[1], na = rec[22];
    const double* tm_f = fd(S, F_theta_m);
    const int* ad = fi(S, F_advCellsForEdge) + (size_t)e * 15;
    const double* ac = fd(S, F_adv_coefs) + (size_t)e * 15;
    const double* ac3 = fd(S, F_adv_coefs_3rd) + (size_t)e * 15;
    int ad_[AF];
    double tv_[AF], ac_[AF], ac3_[AF], wv_[AF];
#pragma unroll
    for (int j = 0; j < AF; j++) ad_[j] = rec[12 + j];
    row_ld(ac, ac_);
    row_ld(ac3, ac3_);
    const bool kl = k < L;
    double2 g_tv[AF / 2], g_wv[AF / 2];
#pragma unroll
    for (int j = 0; j < AF - 1; j += 2) g_tv[j / 2] = gather2s_ld<LP>(tm_f, ad_[j], ad_[j + 1], k);
    const double2 g_tvl = gather2_ld<LP>(tm_f, ad_[AF - 1], fd(S, F_ru), e, k);
    if constexpr (MD) {
#pragma unroll
        for (int j = 0; j < AF - 1; j += 2) g_wv[j / 2] = gather2s_ld<LP>(fd(S, F_w), ad_[j], ad_[j + 1], k);
    }
    double2 g_ts = make_double2(0.0, 0.0);
    double rus_e = 0.0;
    if constexpr (!RK0) {
        g_ts = gather2s_ld<LP>(fd(S, F_theta_m_save), cell1, cell2, k);
        rus_e = colk(fd(S, F_ru_save), e);
    }
    const double wvl = MD ? colk(fd(S, F_w), ad_[AF - 1]) : 0.0;
    __builtin_amdgcn_sched_barrier(0);
    double ru_e;
#pragma unroll
    for (int j = 0; j < AF - 1; j += 2) g2_fin<LP>(g_tv[j / 2], tv_[j], tv_[j + 1]);
    g2_fin<LP>(g_tvl, tv_[AF - 1], ru_e);
    if constexpr (MD) {
#pragma unroll
        for (int j = 0; j < AF - 1; j += 2) g2_fin<LP>(g_wv[j / 2], wv_[j], wv_[j + 1]);
        wv_[AF - 1] = wvl;
    }
    double ts1 = 0.0, ts2 = 0.0;
    if constexpr (!RK0) {
        g2_fin<LP>(g_ts, ts1, ts2);
        if (a.cp) rus_e = ru_e;  // (k_dyn_B's rule: the copy is setup's, ru_save = ru)
    }
    {  // k_dyn_B's flux_arr and H, the same expressions
        const double sg = copysign(1.0, ru_e);
        double flux_arr = 0.0;
#pragma unroll
        for (int j = 0; j < AF; j++) {
            double scalar_weight = ac_[j] + sg * ac3_[j];
            flux_arr = add_if(j < na, flux_arr, scalar_weight * tv_[j]);
        }
        for (int j = AF; j < na; j++) {
            double scalar_weight = ac[j] + sg * ac3[j];
            flux_arr += scalar_weight * colk(tm_f, ad[j]);
        }
        double h = ru_e * flux_arr;
        if constexpr (!RK0) h += fd(S, F_dvEdge)[e] * ((rus_e - ru_e) * 0.5 * (ts2 + ts1));
        colk(fw(S, X_F), e) = kl ? h : 0.0;
    }
    if constexpr (MD) {  // k_dyn_B's w flux, the same expressions
        const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
        const double ru_edge_w = fzm * ru_e + fzp * lvl_dn<LP>(ru_e, k);
        const double sg = copysign(1.0, ru_edge_w);
        double flux_arr = 0.0;
#pragma unroll
        for (int j = 0; j < AF; j++) {
            double scalar_weight = ac_[j] + sg * ac3_[j];
            flux_arr = add_if(j < na, flux_arr, scalar_weight * wv_[j]);
        }
        for (int j = AF; j < na; j++) {
            double scalar_weight = ac[j] + sg * ac3[j];
            flux_arr += scalar_weight * colk(fd(S, F_w), ad[j]);
        }
        colk(fw(S, X_Fw), e) = (k > 0 && kl) ? ru_edge_w * flux_arr : 0.0;
    }
}

// ------------------------------------------------------------------------ C (rk0)
// VE vertices per vertex wave of C (at LP = 64): a vertex is 3 gathers and one store, so a
// one-vertex wave is latency-bound; the VE vertices issue their gathers together
// (option "cve", default 4; profiles/r03/c_vertex_epw: C 482 -> 398 us at x1.163842, the
// step -0.7 %; 8 vertices: C 410 us, the step and x1.2562 no better than 4)
// (C's stores leave level L unwritten: the keep tails cost it 4 %, profiles/r05/keep_tails)
// PART (a launch's blocks): 1 the vertex blocks, 2 the cell blocks -- two launches, each
// with its mesh rows as scalar loads (one grid of both interleaved made the compiler load
// ~24 of them per wave with vector loads: the other path's stores could clobber them)
// bi: the block's index among its part's blocks (after the XCD remap)
template <int LP, bool SELF, int VE, int PART>
__device__ __forceinline__ void dyn_C_body(const DevState& S, const DynK& a, int bi) {
    const int L = S.L;
    const double* dsu = fd(S, F_delsq_u);
    const int kk = (int)(threadIdx.x % LP);
    if constexpr (PART == 1) {  // VE vertices: delsq_vorticity (:1052-1060)
        const int v0 = col_of<LP>(bi) * VE + S.lo[KV], k = kk;
        if (v0 >= S.nVO) return;  // (k >= L exits after the gathers: gather2 needs every lane)
        int ev[VE][3];
        double d[VE][3], sg_[VE][3], dc_[VE][3], iat[VE];
#pragma unroll
        for (int j = 0; j < VE; j++) {
            const int v = min(v0 + j, S.nVO - 1);
            row_ld(fi(S, F_edgesOnVertex) + (size_t)v * 3, ev[j]);
            row_ld(fd(S, F_edgesOnVertex_sign) + (size_t)v * 3, sg_[j]);
            row_ld(fd(S, X_ve_dc) + (size_t)v * 3, dc_[j]);  // dcEdge(edgesOnVertex)
            iat[j] = fd(S, F_invAreaTriangle)[v];
        }
#pragma unroll
        for (int j = 0; j < VE; j++) gather2s<LP>(dsu, ev[j][0], ev[j][1], k, d[j][0], d[j][1]);
#pragma unroll
        for (int j = 0; j + 1 < VE; j += 2) gather2s<LP>(dsu, ev[j][2], ev[j + 1][2], k, d[j][2], d[j + 1][2]);
        if (VE % 2) d[VE - 1][2] = colk(dsu, ev[VE - 1][2]);
        if (k >= L) return;
#pragma unroll
        for (int j = 0; j < VE; j++) {
            if (v0 + j >= S.nVO) break;  // (wave-uniform)
            double dsv = 0.0;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                double edge_sign = iat[j] * dc_[j][i] * sg_[j][i];
                dsv += edge_sign * d[j][i];
            }
            colk(fw(S, F_delsq_vorticity), v0 + j) = dsv;
        }
        return;
    }
    const int c = col_of<LP>(bi) + S.lo[KC];
    const int k = kk;
    if (c >= S.nCO) return;
    const size_t p = (size_t)c * LP + lpos(LP, k);
    const bool live = k <= L, kl = k < L;
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* eocs = fd(S, F_edgesOnCell_sign) + (size_t)c * 10;
    const int *cc1 = fi(S, X_ce_c1) + (size_t)c * 10, *cc2 = fi(S, X_ce_c2) + (size_t)c * 10;
    const double *cdv = fd(S, X_ce_dv) + (size_t)c * 10, *cidc = fd(S, X_ce_idc) + (size_t)c * 10;
    const double* cmsd2 = fd(S, X_ce_msd2) + (size_t)c * 10;
    // the w the mixing acts on: dyn_tend's partial w tendency (the reference, Q8), the state
    // w under the MPAS dynamics
    const double *rho_edge = fd(S, F_rho_edge), *wc = fd(S, S.physics == 2 ? F_w : X_wc), *kdiff = fd(S, F_kdiff),
                 *tm = fd(S, F_theta_m);
    const double r_areaCell = fd(S, F_invAreaCell)[c];
    const bool del4 = a.h4 > 0.0;

    const int *coth = fi(S, X_ce_oth) + (size_t)c * 10, *cs1 = fi(S, X_ce_s1) + (size_t)c * 10;
    int e_[NF], c1_[NF], c2_[NF], o_[NF], s1_[NF];
    double re_[NF], kd1_[NF], kd2_[NF], wc1_[NF], wc2_[NF], t1_[NF], t2_[NF], ds_[NF];
    double eocs_[NF], cdv_[NF], cidc_[NF], cmsd2_[NF];
    const int ne = SELF ? cell_rec<true>(S, c, e_, o_, s1_) : cell_rec<false>(S, c, e_, c1_, c2_);
    row_ld(eocs, eocs_);
    row_ld(cdv, cdv_);
    row_ld(cidc, cidc_);
    row_ld(cmsd2, cmsd2_);
    const double kd_c = SELF ? colk(kdiff, c) : 0.0, wc_c = SELF ? colk(wc, c) : 0.0, tm_c = SELF ? colk(tm, c) : 0.0;
#pragma unroll
    for (int i = 0; i < NF; i += 2) {
        gather2s<LP>(rho_edge, e_[i], e_[i + 1], k, re_[i], re_[i + 1]);
        cell_pair2<LP, SELF>(kdiff, c1_, c2_, o_, s1_, kd_c, i, k, kd1_[i], kd2_[i], kd1_[i + 1], kd2_[i + 1]);
        cell_pair2<LP, SELF>(wc, c1_, c2_, o_, s1_, wc_c, i, k, wc1_[i], wc2_[i], wc1_[i + 1], wc2_[i + 1]);
        cell_pair2<LP, SELF>(tm, c1_, c2_, o_, s1_, tm_c, i, k, t1_[i], t2_[i], t1_[i + 1], t2_[i + 1]);
        gather2s<LP>(dsu, e_[i], e_[i + 1], k, ds_[i], ds_[i + 1]);
    }
#pragma unroll
    for (int i = 0; i < NF; i++) {
        re_[i] = ldz(live, re_[i]);
        kd1_[i] = ldz(live, kd1_[i]);
        kd2_[i] = ldz(live, kd2_[i]);
        wc1_[i] = ldz(kl, wc1_[i]);
        wc2_[i] = ldz(kl, wc2_[i]);
        t1_[i] = ldz(kl, t1_[i]);
        t2_[i] = ldz(kl, t2_[i]);
        ds_[i] = ldz((kl && del4), ds_[i]);
    }
    double re_m_[NF], kd1m_[NF], kd2m_[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        re_m_[i] = lvl_dn<LP>(re_[i], k);
        kd1m_[i] = lvl_dn<LP>(kd1_[i], k);
        kd2m_[i] = lvl_dn<LP>(kd2_[i], k);
    }
    double dsd = 0.0, delsq_w = 0.0, twe = 0.0, delsq_theta = 0.0, tte = 0.0;
    // the terms of edge slot i, accumulated where `on` holds (selects: no branches)
    auto edge_terms = [&](bool on, double eocs_i, double dv, double idc, double msd2, double re_k, double re_m,
                          double kd1, double kd2, double kd1m, double kd2m, double wc1, double wc2, double tm1,
                          double tm2, double dsue) {
        if (del4) {  // delsq_divergence (:1062-1070)
            double edge_sign = r_areaCell * dv * eocs_i;
            dsd = add_if(on, dsd, edge_sign * dsue);
        }
        {  // delsq_w, tend_w_euler del2 (:1231-1254)
            double edge_sign = 0.5 * r_areaCell * eocs_i * dv * idc;
            double w_turb_flux = edge_sign * (re_k + re_m) * (wc2 - wc1);
            delsq_w = add_if(on && k > 0, delsq_w, w_turb_flux);
            w_turb_flux *= msd2 * 0.25 * (kd1 + kd2 + kd1m + kd2m);
            twe = add_if(on && k > 0, twe, w_turb_flux);
        }
        {  // delsq_theta, tend_theta_euler del2 (:1365-1382)
            double edge_sign = r_areaCell * eocs_i * dv * idc;
            double pr_scale = a.prandtl_inv * msd2;
            double theta_turb_flux = edge_sign * (tm2 - tm1) * re_k;
            delsq_theta = add_if(on, delsq_theta, theta_turb_flux);
            theta_turb_flux *= 0.5 * (kd1 + kd2) * pr_scale;
            tte = add_if(on, tte, theta_turb_flux);
        }
    };
#pragma unroll
    for (int i = 0; i < NF; i++)
        edge_terms(i < ne && kl, eocs_[i], cdv_[i], cidc_[i], cmsd2_[i], re_[i], re_m_[i], kd1_[i], kd2_[i],
                   kd1m_[i], kd2m_[i], wc1_[i], wc2_[i], t1_[i], t2_[i], ds_[i]);
    for (int i = NF; i < ne; i++) {  // generic tail (shuffles: whole column takes it)
        const int e = eoc[i], c1 = cc1[i], c2 = cc2[i];
        double re_k = col_rd<LP>(rho_edge, e, k, L), kd1 = col_rd<LP>(kdiff, c1, k, L), kd2 = col_rd<LP>(kdiff, c2, k, L);
        double re_m = lvl_dn<LP>(re_k, k), kd1m = lvl_dn<LP>(kd1, k), kd2m = lvl_dn<LP>(kd2, k);
        edge_terms(kl, eocs[i], cdv[i], cidc[i], cmsd2[i], re_k, re_m, kd1, kd2, kd1m, kd2m, ldz(kl, colk(wc, c1)),
                   ldz(kl, colk(wc, c2)), ldz(kl, colk(tm, c1)), ldz(kl, colk(tm, c2)), ldz(kl && del4, colk(dsu, e)));
    }
    // (padding levels: zeros, PADW; level L keeps its value; paired 16-B stores, every lane)
    if (del4 && k != L) colk(fw(S, F_delsq_divergence), c) = PADW(dsd);
    put2<LP>(fw(S, F_delsq_w), c, fw(S, F_tend_w_euler), c, k, PADW(delsq_w), PADW(twe), k != L, k != L);
    put2<LP>(fw(S, F_delsq_theta), c, fw(S, F_tend_theta_euler), c, k, PADW(delsq_theta), PADW(tte), k != L, k != L);
}
template <int LP, bool SELF, int VE, int PART>
__global__ __launch_bounds__(256) void k_dyn_C(DevState S, DynK a) {
    dyn_C_body<LP, SELF, VE, PART>(S, a, xcd_block(S.xcd));
}
// both parts in one grid, the vertex and the cell blocks interleaved in proportion
// (vc_block, option vcmix) so that the delsq_u columns both gather are fetched into L2 once
template <int LP, bool SELF, int VE>
__global__ __launch_bounds__(256) void k_dyn_C12(DevState S, DynK a, int nv) {
    int bi;
    if (vc_block(S, xcd_block(S.xcd), nv, bi)) dyn_C_body<LP, SELF, VE, 1>(S, a, bi);
    else dyn_C_body<LP, SELF, VE, 2>(S, a, bi);
}

// ------------------------------------------------------------------------ D (rk0, del4)
template <int LP>
__device__ __forceinline__ void dyn_D_body(const DevState& S, const DynK& a, Blk bk) {
    ColMap<LP> m(S, KE, bk);
    const int L = S.L, k = m.k, e = m.ent;
    if (e >= S.nEO) return;  // (k >= L after the gathers: gather2 needs every lane)
    const int cell1 = fi(S, F_cellsOnEdge)[(size_t)e * 2], cell2 = fi(S, F_cellsOnEdge)[(size_t)e * 2 + 1];
    const int vertex1 = fi(S, F_verticesOnEdge)[(size_t)e * 2], vertex2 = fi(S, F_verticesOnEdge)[(size_t)e * 2 + 1];
    const double invDc = fd(S, F_invDcEdge)[e];
    const double kl_tue = keepv<LP>(S, F_tend_u_euler, KE, e), kl_tu = keepv<LP>(S, F_tend_u, KE, e);
    double u_mix_scale = fd(S, F_meshScalingDel4)[e] * a.h4;
    double r_dc = u_mix_scale * kDel4uDivFactor * invDc;
    double r_dv = u_mix_scale * dmin_(fd(S, F_invDvEdge)[e], 4 * invDc);
    const double *dd = fd(S, F_delsq_divergence), *dvv = fd(S, F_delsq_vorticity);
    double re, tue, dd1, dd2, dv1, dv2, tend_u, trp;
    gather2<LP>(fd(S, F_rho_edge), e, fd(S, F_tend_u_euler), e, k, re, tue);
    gather2s<LP>(dd, cell1, cell2, k, dd1, dd2);
    gather2s<LP>(dvv, vertex1, vertex2, k, dv1, dv2);
    gather2<LP>(fd(S, F_tend_u), e, fd(S, F_tend_ru_physics), e, k, tend_u, trp);
    double u_diffusion = re * ((dd2 - dd1) * r_dc - (dv2 - dv1) * r_dv);
    tue -= u_diffusion;
    tend_u += tue + trp;
    // (padding levels: zeros, PADW; level L keeps its value; one paired 16-B store, every lane)
    put2f<LP>(fw(S, F_tend_u_euler), e, fw(S, F_tend_u), e, k, KEEPW(tue, kl_tue), KEEPW(tend_u, kl_tu));
    if (a.rud != 0.0) ru_first<LP>(S, a.rud, e, k, L, KEEPW(tend_u, kl_tu));  // (option mru)
}

// ------------------------------------------------------------------------ E (cells)
template <int LP>
__global__ __launch_bounds__(256) void k_dyn_D(DevState S, DynK a) {
    dyn_D_body<LP>(S, a, this_blk());
}

// TILE (option "etile", k_dyn_Et below): the cell is one of a tile whose theta_m closure sits
// in LDS (tl.lds, level order, one LP-double column per closure cell; tl.row the cell's
// TrTiles slot row): the flux of each edge over its advCells (B's flux_arr, and under HF B's H)
// is formed here from LDS with B's expressions in B's order, instead of gathered from X_F
struct EtTile {
    const double* lds;    // the closure's theta_m columns, then the zero column
    const double* ldsw;   // (exact) per tile edge, per advCell j: B's weights ac + ac3, ac - ac3 (0, 0 past nAdv);
                          // (HF) per tile edge its flux H, one column (k_dyn_Et's edge phase)
    const unsigned* rec;  // the cell's ETT_REC-byte record (TrTiles::erow)
};
// ETM (TILE): 0 each edge's flux formed per cell (the cell's gathers of ru, ru_save and the
// theta_m_save pairs issued with its own columns: one memory round trip), 1 the same with the flux
// sum formed before the own columns are loaded (fewer registers, two round trips), 2 (HF) the
// tile's edge phase formed every edge's H (k_dyn_Et et_edges)
// NTH (atm_srk3, reference semantics, a stage before the step's last): the call's theta tendency
// outputs (tend_theta, tend_rtheta_adv, rthdynten) are dead -- the last stage rewrites them and no task
// in between reads them (the acoustic step reads theta_m as its tend_rt, Q8) -- so the theta
// advection, wdtz and those stores go, with B's per-edge flux (X_F) that only they read; w, and at
// rk_step 0 tend_w_euler / tend_theta_euler (read by the later stages), are formed as always
// SMLF (option msml, the MPAS dynamics): the stage's atm_set_smlstep_pert_variables_work applied to the
// tend_w formed here (k_set_smlstep's MD form: the same loads and the same order of operations, from the
// value it would read back), so its launch and the tend_w round trip go
template <int LP, bool RK0, bool SELF, bool MD, bool HF, bool TILE = false, int ETM = 0, bool NTH = false,
          bool SMLF = false>
__device__ __forceinline__ void dyn_E_cell(const DevState& S, const DynK& a, int c, int k, EtTile tl = {}) {
    static_assert(!NTH || (!MD && !TILE), "the dead theta tendency: reference semantics, untiled");
    static_assert(!TILE || (LP == 64 && !MD), "the tiled E: LP = 64, reference semantics");
    const int L = S.L;
    const size_t p = (size_t)c * LP + lpos(LP, k);
    constexpr bool rk0 = RK0;
    const bool kl = k < L;
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* eocs = fd(S, F_edgesOnCell_sign) + (size_t)c * 10;
    const int *cc1 = fi(S, X_ce_c1) + (size_t)c * 10, *cc2 = fi(S, X_ce_c2) + (size_t)c * 10;
    const double *cdv = fd(S, X_ce_dv) + (size_t)c * 10, *cidc = fd(S, X_ce_idc) + (size_t)c * 10;
    const double* cmsd4 = fd(S, X_ce_msd4) + (size_t)c * 10;
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k], rdzw = fd(S, F_rdzw)[k], rdzu = fd(S, F_rdzu)[k];
    const double invA = fd(S, F_invAreaCell)[c];
    const bool del4 = rk0 && a.h4 > 0.0;
    // the kept level-L values of the stored columns (keep tails, mpas_dev.h), issued ahead
    const double kl_tra = keepv<LP>(S, F_tend_rtheta_adv, KC, c), kl_w = keepv<LP>(S, F_w, KC, c);
    const double kl_rth = keepv<LP>(S, F_rthdynten, KC, c), kl_tt = keepv<LP>(S, F_tend_theta, KC, c);
    const double kl_twe = keepv<LP>(S, F_tend_w_euler, KC, c), kl_tte = keepv<LP>(S, F_tend_theta_euler, KC, c);
    const double *ru = fd(S, F_ru), *Ff = fd(S, X_F), *rus = fd(S, F_ru_save), *tms_f = fd(S, F_theta_m_save);
    const double *dw = fd(S, F_delsq_w), *dth = fd(S, F_delsq_theta), *tm = fd(S, F_theta_m);

    // ---- issue the independent loads
    const int *coth = fi(S, X_ce_oth) + (size_t)c * 10, *cs1 = fi(S, X_ce_s1) + (size_t)c * 10;
    int e_[NF], c1_[NF], c2_[NF], o_[NF], s1_[NF];
    double ru_[NF], F_[NF], rus_[NF], ts1_[NF], ts2_[NF], dw1_[NF], dw2_[NF], dt1_[NF], dt2_[NF];
    double eocs_[NF], cdv_[NF], cidc_[NF], cmsd4_[NF];
    const int ne = SELF ? cell_rec<true>(S, c, e_, o_, s1_) : cell_rec<false>(S, c, e_, c1_, c2_);
    row_ld(eocs, eocs_);
    row_ld(cdv, cdv_);
    if (rk0) {
        row_ld(cidc, cidc_);
        row_ld(cmsd4, cmsd4_);
    }
    // TILE: E's theta advection sum over the cell's edges (:1328-1360), into tth -- each edge's flux
    // over its advCells from the tile's LDS columns with B's expressions in B's order (B's flux_arr;
    // under HF B's H), then summed in E's order.  Its gathers first, then the cell's own columns
    // below, then the sum (before the w section): one memory round trip for both
    // (lanes k >= L: unmasked values, their sums are never used -- tend_theta takes tth where k < L)
    double tth = 0.0;
    double tru[NF], trus[NF], tt1[NF], tt2[NF];
    constexpr bool EPH = HF && ETM == 2;  // (the edge phase formed every edge's H)
    if constexpr (TILE && !EPH) {
        const double ts_own = SELF ? colk(tms_f, c) : 0.0;
#pragma unroll
        for (int i = 0; i < NF; i += 2) {
            gather2s<LP>(ru, e_[i], e_[i + 1], k, tru[i], tru[i + 1]);
            if (!rk0) {
                gather2s<LP>(rus, e_[i], e_[i + 1], k, trus[i], trus[i + 1]);
                cell_pair2<LP, SELF>(tms_f, c1_, c2_, o_, s1_, ts_own, i, k, tt1[i], tt2[i], tt1[i + 1], tt2[i + 1]);
            }
        }
    }
    auto tile_flux = [&]() {
        // per edge: B's scalar weights (ac + sign ac3: the tile's LDS pair, picked per lane by the sign
        // of ru) times the advCells' columns from LDS, in B's order; the slots past nAdvCellsForEdge
        // add 0 * 0 (the zero column), which leaves the sum as B's masked add does (it is never -0)
        unsigned rw_[ETT_REC / 4];
        row_ld(tl.rec, rw_);
        auto byte_at = [&](int b) { return (int)((rw_[b >> 2] >> ((b & 3) * 8)) & 0xffu); };
#pragma unroll
        for (int i = 0; i < NF; i++) {
            const bool pos = copysign(1.0, tru[i]) > 0.0;
            const double* wr = tl.ldsw + byte_at(i * ETT_EB) * (2 * AF) + (pos ? 0 : 1);
            double flux_arr = 0.0;
#pragma unroll
            for (int j = 0; j < AF; j++) flux_arr = flux_arr + wr[2 * j] * tl.lds[byte_at(i * ETT_EB + 1 + j) * LP + k];
            if constexpr (HF) {  // B's H: ru F (+ dvEdge (ru_save - ru) theta_m_save at the edge, rk > 0)
                double h = tru[i] * flux_arr;
                if constexpr (!RK0) {
                    const double rus_e = a.cp ? tru[i] : trus[i];
                    h += cdv_[i] * ((rus_e - tru[i]) * 0.5 * (tt2[i] + tt1[i]));
                }
                tth = sub_if(i < ne, tth, eocs_[i] * (kl ? h : 0.0));
            } else {
                tth = sub_if(i < ne, tth, eocs_[i] * tru[i] * (kl ? flux_arr : 0.0));
            }
            // one edge at a time (the asm ties tth to this point): the scheduler would otherwise hoist
            // all 54 LDS reads of the cell and spill
            asm volatile("" : "+v"(tth));
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (!HF && !RK0) {  // :1347-1360
#pragma unroll
            for (int i = 0; i < NF; i++) {
                double flux = eocs_[i] * cdv_[i] * (trus[i] - tru[i]) * 0.5 * (tt2[i] + tt1[i]);
                tth = sub_if(i < ne, tth, flux);
            }
        }
    };
    if constexpr (TILE && !EPH && ETM == 1) tile_flux();
    // own columns (gather2: two columns per load instruction; the theta-section loads
    // too, ahead of the w stores that could alias them for the compiler)
    double wc, rw, pp, dpdz, rws, tms, tmv, twe, tte, rho_zz, rt_diab, trp, cqw = 0.0, dw_c = 0.0, dt_c = 0.0;
    // wc: the reference's partial w tendency (A at rk_step 0; WCE: formed below); MD: the state w
    constexpr bool WCE = !MD && !RK0;
    double urz = 0.0, urm = 0.0, Fw_[NF], ru_l = 0.0, wfl[2];
    if constexpr (WCE) {
        col_rd2<LP>(fd(S, F_uReconstructZonal), fd(S, F_uReconstructMeridional), c, k, L, urz, urm);
        rw = colk(fd(S, F_rw), c);
        int el = 0;  // the cell's last edge (Q13: ru_edge_w of the last edge)
#pragma unroll
        for (int i = 0; i < NF; i++) el = (i == ne - 1) ? e_[i] : el;
        if (ne > NF) el = eoc[ne - 1];
        ru_l = ne > 0 ? col_rd<LP>(ru, el, k, L) : 0.0;
        row_ld(fd(S, X_wfl) + (size_t)c * 2, wfl);
        wc = 0.0;
    } else {
        gather2<LP>(fd(S, MD ? F_w : X_wc), c, fd(S, F_rw), c, k, wc, rw);
    }
    if constexpr (MD) {
        gather2<LP>(fd(S, F_uReconstructZonal), c, fd(S, F_uReconstructMeridional), c, k, urz, urm);
#pragma unroll
        for (int i = 0; i < NF; i += 2) gather2s<LP>(fd(S, X_Fw), e_[i], e_[i + 1], k, Fw_[i], Fw_[i + 1]);
    }
    if (rk0) gather2<LP>(fd(S, F_pressure_p), c, fd(S, F_dpdz), c, k, pp, dpdz);
    else pp = dpdz = 0.0;
    if constexpr (NTH) rws = tms = 0.0;  // (wdtz's, dead)
    else gather2<LP>(fd(S, F_rw_save), c, tms_f, c, k, rws, tms);
    gather2<LP>(tm, c, fd(S, F_tend_w_euler), c, k, tmv, twe);
    gather2<LP>(fd(S, F_tend_theta_euler), c, fd(S, F_rho_zz), c, k, tte, rho_zz);
    if constexpr (NTH) rt_diab = trp = 0.0;
    else gather2<LP>(fd(S, F_rt_diabatic_tend), c, fd(S, F_tend_rtheta_physics), c, k, rt_diab, trp);
    if (rk0) {
        if (SELF) gather2<LP>(fd(S, F_cqw), c, dw, c, k, cqw, dw_c);
        else cqw = colk(fd(S, F_cqw), c);
        if (SELF) dt_c = colk(dth, c);
    }
    const double ts_c = tms;  // (SELF, rk > 0: theta_m_save at the cell itself)
    // HF: F holds B's per-edge flux H (ru F + the rk > 0 perturbation flux): ru, ru_save
    // and the theta_m_save pairs are not gathered here
    // (TILE: the theta advection sum tth was formed above; no ru, ru_save, theta_m_save or X_F here)
    constexpr bool GRU = !HF && !TILE && !NTH;
#pragma unroll
    for (int i = 0; i < NF; i += 2) {
        if (GRU) gather2s<LP>(ru, e_[i], e_[i + 1], k, ru_[i], ru_[i + 1]);
        if (!TILE && !NTH) gather2s<LP>(Ff, e_[i], e_[i + 1], k, F_[i], F_[i + 1]);
    }
#pragma unroll
    for (int i = 0; i < NF; i++) {
        ru_[i] = GRU ? ldz(kl, ru_[i]) : 0.0;
        F_[i] = (TILE || NTH) ? 0.0 : ldz(kl, F_[i]);
        rus_[i] = ts1_[i] = ts2_[i] = dw1_[i] = dw2_[i] = dt1_[i] = dt2_[i] = 0.0;
    }
    if (!rk0 && GRU) {
#pragma unroll
        for (int i = 0; i < NF; i += 2) {
            gather2s<LP>(rus, e_[i], e_[i + 1], k, rus_[i], rus_[i + 1]);
            cell_pair2<LP, SELF>(tms_f, c1_, c2_, o_, s1_, ts_c, i, k, ts1_[i], ts2_[i], ts1_[i + 1], ts2_[i + 1]);
        }
#pragma unroll
        for (int i = 0; i < NF; i++) {
            rus_[i] = ldz(kl, rus_[i]);
            ts1_[i] = ldz(kl, ts1_[i]);
            ts2_[i] = ldz(kl, ts2_[i]);
        }
    }
    if (rk0) {  // (compile-time: a runtime `if (del4)` here would put each slot's loads in a branch)
#pragma unroll
        for (int i = 0; i < NF; i++) {
            cell_pair_ff<LP, SELF>(dw, dth, c1_, c2_, o_, s1_, dw_c, dt_c, i, k, dw1_[i], dw2_[i], dt1_[i], dt2_[i]);
            dw1_[i] = ldz(kl && del4, dw1_[i]);
            dw2_[i] = ldz(kl && del4, dw2_[i]);
            dt1_[i] = ldz(kl && del4, dt1_[i]);
            dt2_[i] = ldz(kl && del4, dt2_[i]);
        }
    }
    if constexpr (TILE && EPH) {  // B's per-edge H, from the edge phase's LDS column of each edge
        unsigned rw_[ETT_REC / 4];
        row_ld(tl.rec, rw_);
#pragma unroll
        for (int i = 0; i < NF; i++) {
            const int te = (int)((rw_[(i * ETT_EB) >> 2] >> (((i * ETT_EB) & 3) * 8)) & 0xffu);
            tth = sub_if(i < ne, tth, eocs_[i] * tl.ldsw[te * LP + k]);
        }
    } else if constexpr (TILE) {
        if constexpr (ETM == 0) tile_flux();
    }
    if constexpr (WCE) {  // dyn_A's w section (:1170-1218, Q13), the same operands in the same order
        const double ru_lm = lvl_dn<LP>(ru_l, k);
        const double rz = ldz(k <= L, rho_zz);
        const double rz_m = lvl_dn<LP>(rz, k), urz_m = lvl_dn<LP>(urz, k), urm_m = lvl_dn<LP>(urm, k);
        double w0 = 0.0;
        if (ne > 0 && k > 0) {
            double ru_edge_w = fzm * ru_l + fzp * ru_lm;
            const double flux_arr = copysign(1.0, ru_edge_w) > 0.0 ? wfl[0] : wfl[1];
#pragma unroll
            for (int i = 0; i < NF; i++) w0 = sub_if(i < ne, w0, eocs_[i] * ru_edge_w * flux_arr);
            for (int i = NF; i < ne; i++) w0 -= eocs[i] * ru_edge_w * flux_arr;
        }
        wc = w0;
        if (k > 0) {
            const double coslat = fd(S, X_cosLatCell)[c];
            double aa = fzm * urz + fzp * urz_m;
            double bb = fzm * urm + fzp * urm_m;
            wc += (rz * fzm + rz_m * fzp) * ((aa * aa) + (bb * bb)) / a.r_earth +
                  2.0 * kOmega * coslat * (fzm * urz + fzp * urz_m) * (rz * fzm + rz_m * fzp);
        }
    }
    wc = ldz(kl, wc);
    rw = ldz(k <= L, rw);
    pp = ldz(k <= L, pp);
    dpdz = ldz(k <= L, dpdz);
    rws = ldz(k <= L, rws);
    tms = ldz(k <= L, tms);
    tmv = ldz(k <= L, tmv);
    twe = ldz(kl, twe);
    tte = ldz(kl, tte);
    // level-L slots (MD: MPAS-A's top fluxes are 0)
    const double wdwzL = MD ? 0.0 : fd(S, F_wdwz)[(size_t)c * LP + lpos(LP, L)];
    const double wdtzL = (MD || NTH) ? 0.0 : fd(S, F_wdtz)[(size_t)c * LP + lpos(LP, L)];

    // ================= W =================
    if (del4 && kl) {  // :1258-1272
        double r_areaCell = a.h4 * invA;
#pragma unroll
        for (int i = 0; i < NF; i++) {
            double edge_sign = cmsd4_[i] * r_areaCell * cdv_[i] * eocs_[i] * cidc_[i];
            twe = sub_if(i < ne && k > 0, twe, edge_sign * (dw2_[i] - dw1_[i]));
        }
        for (int i = NF; i < ne; i++) {
            double edge_sign = cmsd4[i] * r_areaCell * cdv[i] * eocs[i] * cidc[i];
            if (k > 0) twe -= edge_sign * (colk(dw, cc2[i]) - colk(dw, cc1[i]));
        }
    }
    const double wc_m = lvl_dn<LP>(wc, k), wc_m2 = lvl_dn2<LP>(wc, k), wc_p = lvl_up<LP>(wc, k);
    const double rw_m = lvl_dn<LP>(rw, k);
    double wdwz = 0.0;  // :1277-1287
    if (k == 1 || k == L - 1) wdwz = 0.25 * (rw + rw_m) * (wc + wc_m);
    if (k > 1 && k < L - 1) wdwz = flux3(wc_m2, wc_m, wc, wc_p, 0.5 * (rw + rw_m), 1.0);
    if (k == L) wdwz = wdwzL;
    const double wdwz_p = lvl_up<LP>(wdwz, k);
    const double pp_m = lvl_dn<LP>(pp, k), dpdz_m = lvl_dn<LP>(dpdz, k);
    double w = wc;
    if constexpr (MD) {  // the horizontal w flux over every edge, then the area scaling
        double hw = 0.0;
        if constexpr (HF) {  // B's per-edge Hw (fast path: reassociated)
#pragma unroll
            for (int i = 0; i < NF; i++) hw = sub_if(i < ne && k > 0 && kl, hw, eocs_[i] * Fw_[i]);
            for (int i = NF; i < ne; i++) hw = sub_if(k > 0 && kl, hw, eocs[i] * colk(fd(S, X_Fw), eoc[i]));
        } else {
#pragma unroll
            for (int i = 0; i < NF; i++) {
                const double ru_edge_w = fzm * ru_[i] + fzp * lvl_dn<LP>(ru_[i], k);
                hw = sub_if(i < ne && k > 0 && kl, hw, eocs_[i] * ru_edge_w * Fw_[i]);
            }
            for (int i = NF; i < ne; i++) {
                const double ru_k = ldz(kl, colk(ru, eoc[i])), ru_edge_w = fzm * ru_k + fzp * lvl_dn<LP>(ru_k, k);
                hw = sub_if(k > 0 && kl, hw, eocs[i] * ru_edge_w * colk(fd(S, X_Fw), eoc[i]));
            }
        }
        const double rz_m = lvl_dn<LP>(rho_zz, k), urz_m = lvl_dn<LP>(urz, k), urm_m = lvl_dn<LP>(urm, k);
        const double coslat = fd(S, X_cosLatCell)[c];
        const double aa = fzm * urz + fzp * urz_m, bb = fzm * urm + fzp * urm_m;
        const double curv = (rho_zz * fzm + rz_m * fzp) * ((aa * aa) + (bb * bb)) / a.r_earth +
                            2.0 * kOmega * coslat * (fzm * urz + fzp * urz_m) * (rho_zz * fzm + rz_m * fzp);
        w = 0.0;
        if (k > 0 && kl) {
            w = hw * invA + curv - rdzu * (wdwz_p - wdwz);
            if (rk0) twe -= cqw * (rdzu * (pp - pp_m) - (fzm * dpdz + fzp * dpdz_m));
            w += twe;
        }
        if constexpr (SMLF) {  // :1503-1528 with the MPAS forms (k_set_smlstep<MD>), on the tend_w just formed
            static_assert(MD, "set_smlstep in E: the MPAS dynamics");
            const double w_in = ldz(k <= L, PADW(w));  // (the value k_set_smlstep would read back)
            const double* ut_f = fd(S, F_tend_u);
            const double *zb = fd(S, F_zb_cell), *zb3 = fd(S, F_zb3_cell);
            const double zzv = col_rd<LP>(fd(S, F_zz), c, k, L), zz_m = lvl_dn<LP>(zzv, k);
            double ut_[NF], utm_[NF], zb_[NF], zb3_[NF];
#pragma unroll
            for (int i = 0; i < NF; i += 2) gather2s<LP>(ut_f, e_[i], e_[i + 1], k, ut_[i], ut_[i + 1]);
#pragma unroll
            for (int i = 0; i < NF; i++) {
                ut_[i] = ldz(k <= L, ut_[i]);
                gather2<LP>(zb, c * 10 + i, zb3, c * 10 + i, k, zb_[i], zb3_[i]);
            }
#pragma unroll
            for (int i = 0; i < NF; i++) utm_[i] = lvl_dn<LP>(ut_[i], k);
            double ws = w_in;
#pragma unroll
            for (int i = 0; i < NF; i++) {
                double flux = eocs_[i] * (fzm * ut_[i] + fzp * utm_[i]);
                const double t = (zb_[i] + copysign(1.0, ut_[i]) * zb3_[i]) * flux;
                ws = sub_if(i < ne, ws, t);
            }
            for (int i = NF; i < ne; i++) {
                int iEdge = eoc[i];
                double ut = col_rd<LP>(ut_f, iEdge, k, L);
                double ut_m = lvl_dn<LP>(ut, k);
                double flux = eocs[i] * (fzm * ut + fzp * ut_m);
                size_t q = ((size_t)c * 10 + i) * LP + lpos(LP, k);
                ws -= (zb[q] + copysign(1.0, ut) * zb3[q]) * flux;
            }
            ws *= (fzm * zzv + fzp * zz_m);
            const bool in_zone = fi(S, F_bdyMaskCell)[c] <= kRelaxZone;
            colk(fw(S, F_tend_w), c) = in_zone ? ((k >= 1 && k < L) ? ws : PADW(w_in)) : PADW(w);
        } else {
            colk(fw(S, F_tend_w), c) = PADW(w);
        }
        if (rk0) colk(fw(S, F_tend_w_euler), c) = KEEPW(twe, kl_twe);
    } else {
        if (k > 0 && kl) {  // :1289-1302 (Q14 literal), :1318-1322
            w *= invA - rdzu * (wdwz_p - wdwz);
            if (rk0) twe -= cqw * (rdzu * (pp - pp_m) - (fzm * dpdz + fzp * dpdz_m));
            w += twe;
        }
        if (!HF && k != L) {  // (padding levels: zeros, PADW; HF: paired stores at the end)
            colk(fw(S, F_w), c) = PADW(w);
            if (rk0) colk(fw(S, F_tend_w_euler), c) = PADW(twe);
        }
    }

    // ================= theta =================
    if constexpr (NTH) {  // the live outputs only: w, and at rk_step 0 the euler tendencies (del4 of theta)
        if (rk0 && kl && del4) {  // :1384-1400
            double r_areaCell = a.h4 * a.prandtl_inv * invA;
#pragma unroll
            for (int i = 0; i < NF; i++) {
                double edge_sign = cmsd4_[i] * r_areaCell * cdv_[i] * eocs_[i] * cidc_[i];
                tte = sub_if(i < ne, tte, edge_sign * (dt2_[i] - dt1_[i]));
            }
            for (int i = NF; i < ne; i++) {
                double edge_sign = cmsd4[i] * r_areaCell * cdv[i] * eocs[i] * cidc[i];
                tte -= edge_sign * (colk(dth, cc2[i]) - colk(dth, cc1[i]));
            }
        }
        if constexpr (HF) {
            colk(fw(S, F_w), c) = KEEPW(w, kl_w);
            if (rk0)
                put2f<LP>(fw(S, F_tend_w_euler), c, fw(S, F_tend_theta_euler), c, k, KEEPW(twe, kl_twe),
                         KEEPW(tte, kl_tte));
        } else if (rk0 && k != L) {  // (w and tend_w_euler stored above)
            colk(fw(S, F_tend_theta_euler), c) = PADW(tte);
        }
        return;
    }
    double tend_theta = 0.0;  // :1328-1344
    if (TILE) {  // (formed above)
        if (kl) tend_theta = tth;
    } else if (kl && HF) {  // the same sums over B's per-edge H (fast path: reassociated)
#pragma unroll
        for (int i = 0; i < NF; i++) tend_theta = sub_if(i < ne, tend_theta, eocs_[i] * F_[i]);
        if constexpr (!TILE)
            for (int i = NF; i < ne; i++) tend_theta -= eocs[i] * colk(Ff, eoc[i]);
    } else if (kl) {
#pragma unroll
        for (int i = 0; i < NF; i++) tend_theta = sub_if(i < ne, tend_theta, eocs_[i] * ru_[i] * F_[i]);
        if constexpr (!TILE)
            for (int i = NF; i < ne; i++) tend_theta -= eocs[i] * colk(ru, eoc[i]) * colk(Ff, eoc[i]);
        if (!rk0) {  // :1347-1360
#pragma unroll
            for (int i = 0; i < NF; i++) {
                double flux = eocs_[i] * cdv_[i] * (rus_[i] - ru_[i]) * 0.5 * (ts2_[i] + ts1_[i]);
                tend_theta = sub_if(i < ne, tend_theta, flux);
            }
            for (int i = NF; i < ne; i++) {
                const int e = eoc[i];
                double flux = eocs[i] * cdv[i] * (colk(rus, e) - colk(ru, e)) * 0.5 *
                              (colk(tms_f, cc2[i]) + colk(tms_f, cc1[i]));
                tend_theta -= flux;
            }
        }
    }
    if (kl) {
        if (del4) {  // :1384-1400
            double r_areaCell = a.h4 * a.prandtl_inv * invA;
#pragma unroll
            for (int i = 0; i < NF; i++) {
                double edge_sign = cmsd4_[i] * r_areaCell * cdv_[i] * eocs_[i] * cidc_[i];
                tte = sub_if(i < ne, tte, edge_sign * (dt2_[i] - dt1_[i]));
            }
            for (int i = NF; i < ne; i++) {
                double edge_sign = cmsd4[i] * r_areaCell * cdv[i] * eocs[i] * cidc[i];
                tte -= edge_sign * (colk(dth, cc2[i]) - colk(dth, cc1[i]));
            }
        }
    }
    // wdtz (:1406-1420, Q15 literal order); level L read from the never-written field
    const double tms_m = lvl_dn<LP>(tms, k), tm_m = lvl_dn<LP>(tmv, k);
    double wdtz = 0.0;
    if constexpr (MD) {  // MPAS-A: 3rd-order flux of theta_m by rw + the rtheta_pp redefinition term
        const double tm_m2 = lvl_dn2<LP>(tmv, k), tm_p = lvl_up<LP>(tmv, k);
        if (k == 1) wdtz = rw * (fzm * tmv + fzp * tm_m) + (rws - rw) * (fzm * tms + fzp * tms_m);
        if (k > 1 && k < L - 1) wdtz = flux3(tm_m2, tm_m, tmv, tm_p, rw, 0.25) + (rws - rw) * (fzm * tms + fzp * tms_m);
        if (k == L - 1) wdtz = rws * (fzm * tmv + fzp * tm_m);
    } else {
        if (k > 0 && k < L - 1) wdtz = ((rws - rw) * (fzm * tms + fzp * tms_m));
        if (k == 1) wdtz += rw * (fzm * tmv + fzp * tm_m);
        if (k == L - 1) wdtz = rws * (fzm * tms + fzp * tms_m);
    }
    if (k == L) wdtz = wdtzL;
    const double wdtz_p = lvl_up<LP>(wdtz, k);
    if constexpr (HF) {  // every lane stores (paired 16-B stores); level L keeps its value
        // :1422-1427, :1477-1479 (MD: the MPAS-A form, Q14; its w stores are made above)
        if (MD) tend_theta = tend_theta * invA - rdzw * (wdtz_p - wdtz);
        else tend_theta *= invA - rdzw * (wdtz_p - wdtz);
        const double rth = tend_theta / rho_zz;
        // (level L: the kept values, keep tails in mpas_dev.h -- every line written whole)
        if (MD) colk(fw(S, F_tend_rtheta_adv), c) = KEEPW(tend_theta, kl_tra);
        if (!MD)
            put2f<LP>(fw(S, F_w), c, fw(S, F_tend_rtheta_adv), c, k, KEEPW(w, kl_w),
                     KEEPW(tend_theta, kl_tra));
        tend_theta += rho_zz * rt_diab;
        tend_theta += tte + trp;
        put2f<LP>(fw(S, F_rthdynten), c, fw(S, F_tend_theta), c, k, KEEPW(rth, kl_rth), KEEPW(tend_theta, kl_tt));
        if (rk0 && MD) colk(fw(S, F_tend_theta_euler), c) = KEEPW(tte, kl_tte);
        if (rk0 && !MD)
            put2f<LP>(fw(S, F_tend_w_euler), c, fw(S, F_tend_theta_euler), c, k,
                     KEEPW(twe, kl_twe), KEEPW(tte, kl_tte));
        return;
    }
    if (k == L) return;  // (padding levels: zeros, PADW)
    // :1422-1427, :1477-1479
    if (MD) tend_theta = tend_theta * invA - rdzw * (wdtz_p - wdtz);
    else tend_theta *= invA - rdzw * (wdtz_p - wdtz);
    colk(fw(S, F_tend_rtheta_adv), c) = PADW(tend_theta);
    colk(fw(S, F_rthdynten), c) = PADW(tend_theta / rho_zz);
    tend_theta += rho_zz * rt_diab;
    tend_theta += tte + trp;
    colk(fw(S, F_tend_theta), c) = PADW(tend_theta);
    if (rk0) colk(fw(S, F_tend_theta_euler), c) = PADW(tte);
}

template <int LP, bool RK0, bool SELF, bool MD, bool HF, bool NTH = false, bool SMLF = false>
__device__ __forceinline__ void dyn_E_body(const DevState& S, const DynK& a, Blk bk) {
    ColMap<LP> m(S, KC, bk);
    if (m.ent >= S.nCO) return;
    dyn_E_cell<LP, RK0, SELF, MD, HF, false, 0, NTH, SMLF>(S, a, m.ent, m.k);
}

// option "etile" (reference semantics, LP = 64): E over the tiles of TrTiles (mpas_dev.h; the
// cells of a tile compact, its closure every cell the tile's cells read theta_m at).  The block
// stages the closure's theta_m columns in LDS once -- two columns per 16-B lane load, level
// order --, then its waves run E for the tile's cells, one cell per wave at a time, each edge's
// advCells flux formed from LDS (dyn_E_cell TILE): no per-edge scratch X_F, and the ~27 theta_m
// column gathers per cell of B's flux become the tile's closure, ~4 columns per cell
struct EtK {
    const int *tptr, *tcell, *cptr, *ccell, *teptr, *tedge;
    const unsigned *erow, *terec;
    int maxclo;
};

// the fast path's edge phase: every edge of the tile gets B's H (k_dyn_B HF: ru F, + dvEdge (ru_save -
// ru) theta_m_save at rk_step > 0) -- B's expressions in B's order on the same values, the advCells'
// theta_m from the tile's LDS columns -- into its LDS column (level order; 0 from level L up, as X_F).
// Two edges per wave at a time (their loads together)
template <bool RK0, int NT>
__device__ __forceinline__ void et_edges(const DevState& S, const DynK& a, const EtK& T, int eb, int nte,
                                         const double* lds, double* ldsH, int w, int k) {
    constexpr int LP = 64, NW = NT / LP, U = 2;
    const int L = S.L;
    const bool kl = k < L;
    const double *ru_f = fd(S, F_ru), *rus_f = fd(S, F_ru_save), *tms_f = fd(S, F_theta_m_save);
    for (int q0 = w; q0 < nte; q0 += U * NW) {
        int e[U];
        double ru_e[U], rus_e[U], ts1[U], ts2[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int q = q0 + u * NW < nte ? q0 + u * NW : q0;
            e[u] = ldc(T.tedge + eb + q);
            if constexpr (RK0) {
                ru_e[u] = colk(ru_f, e[u]);
                rus_e[u] = ts1[u] = ts2[u] = 0.0;
            } else {
                const int c1 = ldc(fi(S, F_cellsOnEdge) + (size_t)e[u] * 2), c2 = ldc(fi(S, F_cellsOnEdge) + (size_t)e[u] * 2 + 1);
                gather2<LP>(ru_f, e[u], rus_f, e[u], k, ru_e[u], rus_e[u]);
                gather2s<LP>(tms_f, c1, c2, k, ts1[u], ts2[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int q = q0 + u * NW;
            if (q >= nte) break;  // (wave-uniform)
            unsigned r3[ETT_ER / 4];
            row_ld(T.terec + (size_t)(eb + q) * (ETT_ER / 4), r3);
            auto slot = [&](int j) { return (int)((r3[j >> 2] >> ((j & 3) * 8)) & 0xffu); };
            const double *acr = fd(S, F_adv_coefs) + (size_t)e[u] * 15, *ac3r = fd(S, F_adv_coefs_3rd) + (size_t)e[u] * 15;
            const int na = ldc(fi(S, F_nAdvCellsForEdge) + e[u]);
            const double sg = copysign(1.0, ru_e[u]);
            double flux_arr = 0.0;
            if (na == AF) {  // (the usual list; past nAdv the zero column would add 0 * w)
#pragma unroll
                for (int j = 0; j < AF; j++)
                    flux_arr = flux_arr + (ldc(acr + j) + sg * ldc(ac3r + j)) * lds[slot(j) * LP + k];
            } else {
#pragma unroll
                for (int j = 0; j < AF; j++)
                    flux_arr = add_if(j < na, flux_arr, (ldc(acr + j) + sg * ldc(ac3r + j)) * lds[slot(j) * LP + k]);
            }
            double h = ru_e[u] * flux_arr;
            if constexpr (!RK0) {
                const double rs = a.cp ? ru_e[u] : rus_e[u];  // (k_dyn_B's rule: the copy is setup's, ru_save = ru)
                h += ldc(fd(S, F_dvEdge) + e[u]) * ((rs - ru_e[u]) * 0.5 * (ts2[u] + ts1[u]));
            }
            ldsH[q * LP + k] = kl ? h : 0.0;
        }
    }
}

template <bool RK0, bool SELF, bool HF, int ETM, int NT>
__global__ __launch_bounds__(NT, ETM == 2 && !RK0 ? 5 : 4) void k_dyn_Et(DevState S, DynK a, EtK T) {
    constexpr int LP = 64, NW = NT / LP, U = 4;
    constexpr bool EPH = HF && ETM == 2;
    extern __shared__ double lds[];
    double* ldsw = lds + (size_t)(T.maxclo + 1) * LP;
    const int tile = xcd_block(S.xcd);
    const int k = (int)(threadIdx.x % LP), w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / LP));
    const int cb = ldc(T.cptr + tile), n = ldc(T.cptr + tile + 1) - cb;
    const double* tm = fd(S, F_theta_m);
    // the closure's theta_m columns, level order (two columns per 16-B lane load), and the zero column
    for (int i0 = 2 * w; i0 < n; i0 += 2 * NW * U) {
        double2 g[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + 2 * NW * u;
            const int ca = ldc(T.ccell + cb + (i < n ? i : 0)), cc = ldc(T.ccell + cb + (i + 1 < n ? i + 1 : 0));
            g[u] = gather2s_ld<LP>(tm, ca, cc, k);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + 2 * NW * u;
            double x, y;
            g2_fin<LP>(g[u], x, y);
            if (i < n) lds[i * LP + k] = x;
            if (i + 1 < n) lds[(i + 1) * LP + k] = y;
        }
    }
    if (w == NW - 1) lds[n * LP + k] = 0.0;
    const int eb = ldc(T.teptr + tile), nte = ldc(T.teptr + tile + 1) - eb;
    if constexpr (EPH) {
        __syncthreads();
        et_edges<RK0, NT>(S, a, T, eb, nte, lds, ldsw, w, k);
    } else {  // B's scalar weights of the tile's edges (ac + s ac3 for s = +1, -1: exact in s, B's values)
        const double *acf = fd(S, F_adv_coefs), *ac3f = fd(S, F_adv_coefs_3rd);
        for (int t = (int)threadIdx.x; t < nte * AF; t += NT) {
            const int q = t / AF, j = t - q * AF;
            const int e = T.tedge[eb + q];
            const bool on = j < fi(S, F_nAdvCellsForEdge)[e];
            const double ac = acf[(size_t)e * 15 + j], ac3 = ac3f[(size_t)e * 15 + j];
            *(double2*)(ldsw + 2 * t) = on ? make_double2(ac + 1.0 * ac3, ac + -1.0 * ac3) : make_double2(0.0, 0.0);
        }
    }
    __syncthreads();
    const int tb = ldc(T.tptr + tile), nt = ldc(T.tptr + tile + 1) - tb;
    for (int q = w; q < nt; q += NW) {
        const int c = ldc(T.tcell + tb + q);
        dyn_E_cell<LP, RK0, SELF, false, HF, true, ETM>(S, a, c, k, EtTile{lds, ldsw, T.erow + (size_t)(tb + q) * (ETT_REC / 4)});
    }
}

// (rk_step > 0, reference semantics, LP = 64: 4 waves per SIMD, as before E formed wc itself;
// at LP < 64 that cap spilled 10-22 VGPRs)
template <int LP, bool RK0, bool SELF, bool MD, bool HF, bool NTH = false, bool SMLF = false>
__global__ __launch_bounds__(256, LP == 64 && !RK0 && !MD ? 4 : 1) void k_dyn_E(DevState S, DynK a) {
    dyn_E_body<LP, RK0, SELF, MD, HF, NTH, SMLF>(S, a, this_blk());
}
// D and E of rk_step 0 in one grid (option "hfuse": neither reads what the other writes)
template <int LP, bool SELF, bool MD, bool HF>
__global__ __launch_bounds__(256) void k_dyn_DE(DevState S, DynK a, int nb1) {
    const int b = (int)blockIdx.x;
    if (b < nb1) dyn_D_body<LP>(S, a, Blk{b, nb1});
    else dyn_E_body<LP, true, SELF, MD, HF>(S, a, Blk{b - nb1, (int)gridDim.x - nb1});
}

static DynK make_dynk(const DevState& S, const DynTendArgs& in) {
    DynK a;
    a.rk_step = in.rk_step;
    a.horiz_mixing = in.horiz_mixing;
    a.rayleigh = in.rayleigh_damp_u;
    a.exact_q = in.exact_q;
    a.tme = in.tme && !S.halo;
    a.cp = in.cp;  // (decomposed: owned edges, like the setup copy; ru_save / u_2 then stale on ghosts)
    const double invDt = 1.0 / in.dt;
    const double c_s = kSmagCoef;
    a.cs_l2 = (c_s * kLenDisp) * (c_s * kLenDisp);
    a.cap = (0.01 * (kLenDisp * kLenDisp)) * invDt;
    a.cam_coef = in.cam_coef;
    a.h4 = (in.rk_step == 0 && in.horiz_mixing == 0) ? kVisc4_2dsmag * (kLenDisp * kLenDisp * kLenDisp) : 0.0;
    a.r_earth = kSphereRadius;
    a.inv_r_earth = 1.0 / a.r_earth;
    a.rayleigh_inv = 1.0 / ((double)kRayleighLevels * (kRayleighDays * kSecondsPerDay));
    a.prandtl_inv = 1.0 / kPrandtl;
    a.d4o = (in.defer_out && in.rk_step == 0 && a.h4 > 0.0) ? 1 : 0;
    a.vB = (in.store_v && S.eoe_same && S.physics != 2) ? 1 : 0;
    a.h4d = (in.defer_in && in.rk_step != 0 && in.horiz_mixing == 0) ? kVisc4_2dsmag * (kLenDisp * kLenDisp * kLenDisp) : 0.0;
    a.rud = (S.physics == 2 && !in.exact_q) ? in.rud : 0.0;  // (option mru: the fast path's HF kernels, and D)
    // (option ntu at rk_step 0 where B forms no tend_u -- dyn_lp_md's `ntu`: h_divergence, which only tend_u
    // reads, is dead; the last stage's A rewrites it)
    a.nhd = (S.physics == 0 && in.ntu && in.rk_step == 0 && !(a.h4 > 0.0 && !a.d4o)) ? 1 : 0;
    return a;
}

template <int LP, bool MD>
static hipError_t dyn_lp_md(const DevState& S, hipStream_t st, const DynTendArgs& in) {
    const DynK a = make_dynk(S, in);
    const bool rk0 = a.rk_step == 0, del4 = rk0 && a.h4 > 0.0;
    // HF: the fast path's theta flux per edge formed in B (E sums eocs H; reassociated, so
    // exact mode keeps the reference's per-cell order)
    const bool hf = !a.exact_q;
    // kernel launches over the entities of a DevState range (HALO_RUN: interior /
    // boundary halves around a halo exchange, or all owned entities)
    auto kA = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (!nb) return;
        if (rk0) k_dyn_A<LP, true, MD><<<nb, 256, 0, st>>>(X, a);
        else k_dyn_A<LP, false, MD><<<nb, 256, 0, st>>>(X, a);
    };
    const bool din = !MD && a.h4d > 0.0;  // (defer4: this rk_step > 0 call applies rk_step 0's D)
    // option etile (reference semantics, LP = 64): E over cell tiles forms the fluxes; B none
    const bool et = !MD && LP == 64 && S.ett != nullptr;
    // option ntu (atm_srk3, reference semantics, a stage before the step's last): the call's tend_u
    // is dead -- B forms none (k_dyn_B NTU; never where D runs in this call and reads it) -- and so
    // are its theta tendencies -- E forms none (k_dyn_E NTH) and B no flux for them (NOF)
    const bool ntu = !MD && in.ntu && !(rk0 && del4 && !a.d4o);
    const bool nth = !MD && in.nth;
    auto kB = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KE);
        if (!nb) return;
        if (et) {
            if (hf) {
                if (rk0) k_dyn_B<LP, true, MD, true, false, true><<<nb, 256, 0, st>>>(X, a);
                else if (din) k_dyn_B<LP, false, MD, true, !MD, true><<<nb, 256, 0, st>>>(X, a);
                else k_dyn_B<LP, false, MD, true, false, true><<<nb, 256, 0, st>>>(X, a);
            } else {
                if (rk0) k_dyn_B<LP, true, MD, false, false, true><<<nb, 256, 0, st>>>(X, a);
                else if (din) k_dyn_B<LP, false, MD, false, !MD, true><<<nb, 256, 0, st>>>(X, a);
                else k_dyn_B<LP, false, MD, false, false, true><<<nb, 256, 0, st>>>(X, a);
            }
        } else if (!MD && (nth || ntu)) {
            if constexpr (!MD) {
                using T_ = std::true_type;
                using F_ = std::false_type;
                auto go = [&](auto R, auto H, auto Di, auto Nf, auto Nt) {
                    k_dyn_B<LP, decltype(R)::value, false, decltype(H)::value, decltype(Di)::value, decltype(Nf)::value,
                            decltype(Nt)::value><<<nb, 256, 0, st>>>(X, a);
                };
                auto go4 = [&](auto R, auto H, auto Di) {
                    if (nth && ntu) go(R, H, Di, T_{}, T_{});
                    else if (nth) go(R, H, Di, T_{}, F_{});
                    else go(R, H, Di, F_{}, T_{});
                };
                auto go3 = [&](auto R, auto Di) {
                    if (hf) go4(R, T_{}, Di);
                    else go4(R, F_{}, Di);
                };
                if (rk0) go3(T_{}, F_{});
                else if (din) go3(F_{}, T_{});
                else if (!(nth && ntu) || a.vB || a.tme || a.cp) go3(F_{}, F_{});
                // (else: nothing of this rk_step > 0 edge kernel is live -- no launch; setup's copies, fusecopy,
                // would be: a reference-driver stage 0 at rk_step > 0 keeps the launch for them)
            }
        } else if (hf && (X.bsplit == 1 || (X.bsplit == 2 && MD))) {  // (option bsplit: the fluxes in k_dyn_Bf first)
            if (rk0) k_dyn_Bf<LP, true, MD><<<nb, 256, 0, st>>>(X, a);
            else k_dyn_Bf<LP, false, MD><<<nb, 256, 0, st>>>(X, a);
            if (rk0) k_dyn_B<LP, true, MD, true, false, true><<<nb, 256, 0, st>>>(X, a);
            else if (din) k_dyn_B<LP, false, MD, true, !MD, true><<<nb, 256, 0, st>>>(X, a);
            else k_dyn_B<LP, false, MD, true, false, true><<<nb, 256, 0, st>>>(X, a);
        } else if (hf) {
            if (rk0 && ntu) k_dyn_B<LP, true, false, true, false, false, !MD><<<nb, 256, 0, st>>>(X, a);
            else if (rk0) k_dyn_B<LP, true, MD, true><<<nb, 256, 0, st>>>(X, a);
            else if (din) k_dyn_B<LP, false, MD, true, !MD><<<nb, 256, 0, st>>>(X, a);
            else k_dyn_B<LP, false, MD, true><<<nb, 256, 0, st>>>(X, a);
        } else {
            if (rk0 && ntu) k_dyn_B<LP, true, false, false, false, false, !MD><<<nb, 256, 0, st>>>(X, a);
            else if (rk0) k_dyn_B<LP, true, MD, false><<<nb, 256, 0, st>>>(X, a);
            else if (din) k_dyn_B<LP, false, MD, false, !MD><<<nb, 256, 0, st>>>(X, a);
            else k_dyn_B<LP, false, MD, false><<<nb, 256, 0, st>>>(X, a);
        }
    };
    auto kC = [&](const DevState& X) {  // the vertex blocks (del4), then the cell blocks
        auto go = [&](auto ve) {
            constexpr int VE = LP == 64 ? decltype(ve)::value : 1;
            const int nv = del4 ? col_blocks_n<LP, VE>(X, KV) : 0, nc = col_blocks<LP>(X, KC);
            if (nv && nc) {
                if (X.selfc) k_dyn_C12<LP, true, VE><<<nv + nc, 256, 0, st>>>(X, a, nv);
                else k_dyn_C12<LP, false, VE><<<nv + nc, 256, 0, st>>>(X, a, nv);
                return;
            }
            if (nv && X.selfc) k_dyn_C<LP, true, VE, 1><<<nv, 256, 0, st>>>(X, a);
            else if (nv) k_dyn_C<LP, false, VE, 1><<<nv, 256, 0, st>>>(X, a);
            if (nc && X.selfc) k_dyn_C<LP, true, VE, 2><<<nc, 256, 0, st>>>(X, a);
            else if (nc) k_dyn_C<LP, false, VE, 2><<<nc, 256, 0, st>>>(X, a);
        };
        const int ve = X.cve ? X.cve : 4;  // (option "cve")
        if (ve == 8) go(std::integral_constant<int, 8>{});
        else if (ve == 4) go(std::integral_constant<int, 4>{});
        else go(std::integral_constant<int, 1>{});
    };
    auto kD = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KE);
        if (nb) k_dyn_D<LP><<<nb, 256, 0, st>>>(X, a);
    };
    auto kE = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (!nb) return;
        if constexpr (LP == 64 && !MD) {
            if (et) {  // (tiles only undecomposed: X is the whole owned range)
                const TrTiles& TT = *X.ett;
                const EtK T{TT.tptr, TT.tcell, TT.cptr, TT.ccell, TT.teptr, TT.tedge, TT.erow, TT.terec, TT.maxclo};
                // (the closure and its zero column; then per tile edge its H column, or in exact mode B's weights)
                const int etm = hf ? X.etm : 0, nt = hf ? X.etnt : 512;
                const size_t shm = ((size_t)(TT.maxclo + 1) * LP + (size_t)TT.maxte * (hf && etm == 2 ? LP : 2 * AF)) * sizeof(double);
                auto go = [&](auto hfc, auto rkc, auto mc, auto ntc) {
                    constexpr bool H = decltype(hfc)::value, R = decltype(rkc)::value;
                    constexpr int M = decltype(mc)::value, N = decltype(ntc)::value;
                    if (X.selfc) k_dyn_Et<R, true, H, M, N><<<TT.ntiles, N, shm, st>>>(X, a, T);
                    else k_dyn_Et<R, false, H, M, N><<<TT.ntiles, N, shm, st>>>(X, a, T);
                };
                using I0 = std::integral_constant<int, 0>;
                using I1 = std::integral_constant<int, 1>;
                using I2 = std::integral_constant<int, 2>;
                using N256 = std::integral_constant<int, 256>;
                using N512 = std::integral_constant<int, 512>;
                auto goh = [&](auto rkc) {
                    if (etm == 2 && nt == 256) go(std::true_type{}, rkc, I2{}, N256{});
                    else if (etm == 2) go(std::true_type{}, rkc, I2{}, N512{});
                    else if (etm == 1 && nt == 256) go(std::true_type{}, rkc, I1{}, N256{});
                    else if (etm == 1) go(std::true_type{}, rkc, I1{}, N512{});
                    else if (nt == 256) go(std::true_type{}, rkc, I0{}, N256{});
                    else go(std::true_type{}, rkc, I0{}, N512{});
                };
                if (hf && rk0) goh(std::true_type{});
                else if (hf) goh(std::false_type{});
                else if (rk0) go(std::false_type{}, std::true_type{}, I0{}, N512{});
                else go(std::false_type{}, std::false_type{}, I0{}, N512{});
                return;
            }
        }
        if constexpr (!MD) {
            if (nth) {  // (k_dyn_E NTH: the theta tendencies dead in this call)
                auto go = [&](auto hfc) {
                    constexpr bool H = decltype(hfc)::value;
                    if (rk0) {
                        if (X.selfc) k_dyn_E<LP, true, true, false, H, true><<<nb, 256, 0, st>>>(X, a);
                        else k_dyn_E<LP, true, false, false, H, true><<<nb, 256, 0, st>>>(X, a);
                    } else {
                        if (X.selfc) k_dyn_E<LP, false, true, false, H, true><<<nb, 256, 0, st>>>(X, a);
                        else k_dyn_E<LP, false, false, false, H, true><<<nb, 256, 0, st>>>(X, a);
                    }
                };
                if (hf) go(std::true_type{});
                else go(std::false_type{});
                return;
            }
        }
        auto go = [&](auto hfc) {
            constexpr bool H = decltype(hfc)::value;
            if constexpr (MD) {
                if (in.smlE) {  // (option msml: the stage's set_smlstep in E)
                    if (rk0 && X.selfc) k_dyn_E<LP, true, true, MD, H, false, true><<<nb, 256, 0, st>>>(X, a);
                    else if (rk0) k_dyn_E<LP, true, false, MD, H, false, true><<<nb, 256, 0, st>>>(X, a);
                    else if (X.selfc) k_dyn_E<LP, false, true, MD, H, false, true><<<nb, 256, 0, st>>>(X, a);
                    else k_dyn_E<LP, false, false, MD, H, false, true><<<nb, 256, 0, st>>>(X, a);
                    return;
                }
            }
            if (rk0) {
                if (X.selfc) k_dyn_E<LP, true, true, MD, H><<<nb, 256, 0, st>>>(X, a);
                else k_dyn_E<LP, true, false, MD, H><<<nb, 256, 0, st>>>(X, a);
            } else {
                if (X.selfc) k_dyn_E<LP, false, true, MD, H><<<nb, 256, 0, st>>>(X, a);
                else k_dyn_E<LP, false, false, MD, H><<<nb, 256, 0, st>>>(X, a);
            }
        };
        if (hf) go(std::true_type{});
        else go(std::false_type{});
    };
    // halo: fields each kernel gathers through an index array / fields it writes
    // (u and v only for the Smagorinsky deformation of rk_step 0: a gather declared but not
    // made would cost an exchange whenever v is stale)
    if (in.skipA) {  // (A ran in the previous combined launch, atm_srk3 hfuse; no halo)
    } else if (ntu && !rk0) {  // (A's one output at rk_step > 0, h_divergence, feeds only the dead tend_u)
    } else if (rk0 && a.horiz_mixing == 0) {
        HALO_RUN(S, st, kA, F_ru, F_u, F_v);
    } else {
        HALO_RUN(S, st, kA, F_ru);
    }
    HALO_WROTE(S, F_kdiff, F_tend_rho, F_dpdz);
    if (!a.nhd) HALO_WROTE(S, F_h_divergence);
    if (!MD && rk0) HALO_WROTE(S, X_wc);
    if (rk0) {
        if (ntu && nth)  // (the pressure gradient and del2 alone)
            HALO_RUN_R1(S, st, kB, F_vorticity, F_pressure_p, F_zz, F_dpdz, F_divergence, F_kdiff, F_vorticity);
        else
            HALO_RUN_R1(S, st, kB, F_vorticity, F_rw, F_w, F_ke, F_h_divergence, F_pv_edge, F_u, F_theta_m, F_pressure_p,
                        F_zz, F_dpdz, F_divergence, F_kdiff, F_vorticity);  // (vorticity at vertices of owned edges)
        HALO_WROTE(S, X_F, F_tend_u, F_tend_u_euler, F_delsq_u);
        if (MD) HALO_WROTE(S, X_Fw);
        if (MD) HALO_RUN(S, st, kC, F_delsq_u, F_rho_edge, F_kdiff, F_w, F_theta_m);
        else HALO_RUN(S, st, kC, F_delsq_u, F_rho_edge, F_kdiff, X_wc, F_theta_m);
        HALO_WROTE(S, F_delsq_vorticity, F_delsq_divergence, F_delsq_w, F_tend_w_euler, F_delsq_theta,
                   F_tend_theta_euler);
        const bool runD = del4 && !a.d4o;  // (defer4: D runs in the next call's B)
        if (runD && in.hfuse && !S.halo && !et && !nth && !in.smlE) {  // D beside E, one grid
            const int nb1 = col_blocks<LP>(S, KE), nb = nb1 + col_blocks<LP>(S, KC);
            auto go = [&](auto hfc) {
                constexpr bool H = decltype(hfc)::value;
                if (S.selfc) k_dyn_DE<LP, true, MD, H><<<nb, 256, 0, st>>>(S, a, nb1);
                else k_dyn_DE<LP, false, MD, H><<<nb, 256, 0, st>>>(S, a, nb1);
            };
            if (nb) {
                if (hf) go(std::true_type{});
                else go(std::false_type{});
            }
        } else {
            if (runD) {
                HALO_RUN(S, st, kD, F_delsq_divergence, F_delsq_vorticity);
                HALO_WROTE(S, F_tend_u_euler, F_tend_u);
            }
            if (in.smlE && hf) HALO_RUN(S, st, kE, X_F, X_Fw, F_delsq_w, F_delsq_theta, F_tend_u);  // (msml)
            else if (in.smlE) HALO_RUN(S, st, kE, F_ru, X_F, X_Fw, F_delsq_w, F_delsq_theta, F_tend_u);
            else if (nth) HALO_RUN(S, st, kE, F_delsq_w, F_delsq_theta);
            else if (et) HALO_RUN(S, st, kE, F_ru, F_theta_m, F_delsq_w, F_delsq_theta);
            else if (hf) HALO_RUN(S, st, kE, X_F, X_Fw, F_delsq_w, F_delsq_theta);  // (X_Fw: MD only written)
            else HALO_RUN(S, st, kE, F_ru, X_F, X_Fw, F_delsq_w, F_delsq_theta);
        }
    } else {
        if (ntu && nth)  // (the deferred del4 of tend_u_euler alone, or nothing)
            HALO_RUN(S, st, kB, F_delsq_divergence, F_delsq_vorticity);
        else if (din && hf)
            HALO_RUN(S, st, kB, F_rw, F_w, F_ke, F_h_divergence, F_pv_edge, F_u, F_theta_m, F_theta_m_save,
                     F_delsq_divergence, F_delsq_vorticity);
        else if (din)
            HALO_RUN(S, st, kB, F_rw, F_w, F_ke, F_h_divergence, F_pv_edge, F_u, F_theta_m, F_delsq_divergence,
                     F_delsq_vorticity);
        else if (hf) HALO_RUN(S, st, kB, F_rw, F_w, F_ke, F_h_divergence, F_pv_edge, F_u, F_theta_m, F_theta_m_save);
        else HALO_RUN(S, st, kB, F_rw, F_w, F_ke, F_h_divergence, F_pv_edge, F_u, F_theta_m);
        HALO_WROTE(S, X_F, F_tend_u);
        if (din) HALO_WROTE(S, F_tend_u_euler);
        if (a.vB) HALO_WROTE(S, F_v);
        if (MD) HALO_WROTE(S, X_Fw);
        if (in.smlE && hf) HALO_RUN(S, st, kE, F_ru, X_F, X_Fw, F_tend_u);  // (msml: tend_u at the cells' edges)
        else if (in.smlE) HALO_RUN(S, st, kE, F_ru, X_F, X_Fw, F_ru_save, F_theta_m_save, F_tend_u);
        else if (nth) HALO_RUN(S, st, kE, F_ru);
        else if (et) HALO_RUN(S, st, kE, F_ru, F_ru_save, F_theta_m, F_theta_m_save);
        else if (hf) HALO_RUN(S, st, kE, F_ru, X_F, X_Fw);  // (ru: wc at the cell's last edge, reference semantics)
        else HALO_RUN(S, st, kE, F_ru, X_F, X_Fw, F_ru_save, F_theta_m_save);
    }
    HALO_WROTE(S, F_tend_w_euler, F_tend_rtheta_adv, F_rthdynten, F_tend_theta, F_tend_theta_euler);
    HALO_WROTE(S, MD ? F_tend_w : F_w);
    if (a.cp) HALO_WROTE(S, F_ru_save, F_u_2);
    if (a.rud != 0.0) HALO_WROTE(S, F_ru_p, F_ruAvg);  // (option mru)
    return hipGetLastError();
}
template <int LP>
static hipError_t dyn_lp(const DevState& S, hipStream_t st, const DynTendArgs& in) {
    return S.physics == 2 ? dyn_lp_md<LP, true>(S, st, in) : dyn_lp_md<LP, false>(S, st, in);
}
hipError_t launch_dyn_tend(const DevState& S, hipStream_t st, const DynTendArgs& in) {
    MPAS_LP_DISPATCH(S.LP, dyn_lp, S, st, in);
}

// option "hfuse" (atm_srk3, reference semantics, undecomposed): the next stage's dyn_tend A
// (cells: h_divergence and the w scratch from ru, rw, rho_zz, uReconstruct*; at rk_step 0
// also kdiff, tend_rho, dpdz from u, v, qtot, rho_p_save) beside the stage's solve_diagnostics
// edge kernel (h_edge, ke_edge, pv_edge from h, u, pv_vertex) -- and, after stage 0, beside
// stage 1's vert_imp too: none of them reads what another writes
template <int LP, int EPW, bool RK0, bool VI>
__global__ __launch_bounds__(256) void k_hf_e_A(DevState S, DynK a, int nb1, int nb2, double dtseps, double rcv,
                                               double c2) {
    const int b = (int)blockIdx.x;
    if (b < nb1) {
        solve_e_body<LP, false, false, EPW>(S, Blk{b, nb1});
    } else if (VI && b < nb1 + nb2) {
        vert_imp_body<LP, false>(S, dtseps, rcv, c2, Blk{b - nb1, nb2});
    } else {
        const int o = nb1 + (VI ? nb2 : 0);
        dyn_A_body<LP, RK0, false>(S, a, Blk{b - o, (int)gridDim.x - o});
    }
}
template <int LP>
static hipError_t hf_e_A_lp(const DevState& S, hipStream_t st, const DynTendArgs& next, int vi, double dts_vi) {
    if (S.halo || S.physics || S.epw != 2) return hipErrorInvalidValue;
    const DynK a = make_dynk(S, next);
    const bool rk0 = a.rk_step == 0;
    const double dtseps = .5 * dts_vi * (1.0 + kEpssm), rcv = kRgas / (kCp - kRgas), c2 = kCp * rcv;
    const int nb1 = col_blocks_n<LP, 2>(S, KE), nb2 = vi ? col_blocks<LP>(S, KC) : 0, nb3 = col_blocks<LP>(S, KC);
    if (!nb1 || !nb3) return hipErrorInvalidValue;
    const int grid = nb1 + nb2 + nb3;
    if (vi) {
        if (rk0) k_hf_e_A<LP, 2, true, true><<<grid, 256, 0, st>>>(S, a, nb1, nb2, dtseps, rcv, c2);
        else k_hf_e_A<LP, 2, false, true><<<grid, 256, 0, st>>>(S, a, nb1, nb2, dtseps, rcv, c2);
    } else {
        if (rk0) k_hf_e_A<LP, 2, true, false><<<grid, 256, 0, st>>>(S, a, nb1, 0, dtseps, rcv, c2);
        else k_hf_e_A<LP, 2, false, false><<<grid, 256, 0, st>>>(S, a, nb1, 0, dtseps, rcv, c2);
    }
    return hipGetLastError();
}
hipError_t launch_hf_solve_e_dyn_A(const DevState& S, hipStream_t st, const DynTendArgs& next, int vi, double dts_vi) {
    MPAS_LP_DISPATCH(S.LP, hf_e_A_lp, S, st, next, vi, dts_vi);
}

// option "hfuse" (atm_srk3 stage 0, with fusesetup): dyn_tend A beside the setup + moist +
// vert_imp launch (k_setup_vi's body, k_misc.hip); A reads nothing that launch writes but
// rho_p_save and qtot, whose values it takes at their source (SETUP above)
// (+ option smlsum: set_smlstep's flux sum of the step, X_smlS, in the last ncb blocks -- it
// reads u_tend / zb_cell / zb3_cell and writes a scratch column neither other body touches)
template <int LP, bool RK0, bool FLUX>
__global__ __launch_bounds__(256) void k_hf_setup_A(DevState S, DynK a, int ncb, int nb1, double dtseps, double rcv,
                                                   double c2) {
    const int b = (int)blockIdx.x;
    const int nA = FLUX ? ((int)gridDim.x - nb1) / 2 : (int)gridDim.x - nb1;
    if (b < nb1) setup_vi_body<LP>(S, ncb, dtseps, rcv, c2, Blk{b, nb1});
    else if (!FLUX || b < nb1 + nA) dyn_A_body<LP, RK0, false, true>(S, a, Blk{b - nb1, nA});
    else sml_flux_body<LP, true>(S, Blk{b - nb1 - nA, nA});
}
template <int LP>
static hipError_t hf_setup_A_lp(const DevState& S, hipStream_t st, const DynTendArgs& stage0, double dts, int edges,
                                int flux) {
    if (S.halo || S.physics) return hipErrorInvalidValue;
    const DynK a = make_dynk(S, stage0);
    const double dtseps = .5 * dts * (1.0 + kEpssm), rcv = kRgas / (kCp - kRgas), c2 = kCp * rcv;
    const int ncb = col_blocks<LP>(S, KC), nb1 = ncb + (edges ? col_blocks<LP>(S, KE) : 0);
    if (!ncb) return hipErrorInvalidValue;
    const int nb = nb1 + ncb * (flux ? 2 : 1);
    if (a.rk_step == 0 && flux) k_hf_setup_A<LP, true, true><<<nb, 256, 0, st>>>(S, a, ncb, nb1, dtseps, rcv, c2);
    else if (a.rk_step == 0) k_hf_setup_A<LP, true, false><<<nb, 256, 0, st>>>(S, a, ncb, nb1, dtseps, rcv, c2);
    else if (flux) k_hf_setup_A<LP, false, true><<<nb, 256, 0, st>>>(S, a, ncb, nb1, dtseps, rcv, c2);
    else k_hf_setup_A<LP, false, false><<<nb, 256, 0, st>>>(S, a, ncb, nb1, dtseps, rcv, c2);
    if (flux) HALO_WROTE(S, X_smlS, X_Dd);
    return hipGetLastError();
}
hipError_t launch_hf_setup_dyn_A(const DevState& S, hipStream_t st, const DynTendArgs& stage0, double dts, int edges,
                                 int flux) {
    MPAS_LP_DISPATCH(S.LP, hf_setup_A_lp, S, st, stage0, dts, edges, flux);
}

}  // namespace mpas
