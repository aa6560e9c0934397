// k_cols.h -- kernel bodies shared by two translation units: each __global__ kernel of
// the step that can share a launch with an independent neighbour (k_solve.hip's combined
// launches, option "hfuse") is a thin wrapper around its body here, which takes the
// block index range it runs on (Blk, mpas_dev.h).  Bodies only; launchers stay with
// their tasks (k_misc.hip, k_solve.hip).
#pragma once
#include "mpas_dev.h"

namespace mpas {

// grid of a grid-stride streaming launch over n threads (at most 8192 blocks)
static inline int stream_grid_(size_t n) {
    size_t g = (n + 255) / 256;
    return (int)(g < 8192 ? (g ? g : 1) : 8192);
}

// ---------------------------------------------------------------- streaming copies
// LP = 64 streaming form: one 16-B position pair per thread (positions 2j, 2j+1 of a
// column = levels j and j+32, mpas_dev.h lpos), every copy of the task in ONE launch
// (blockIdx.y = copy).  The never-written level-L slot sits in pair lpos(L) >> 1 of each
// column: that pair stores only its other element.
struct Pair64 {
    int pair, el;  // pair index within the column holding level L, and L's element in it
    __host__ __device__ Pair64(int L) : pair(lpos(64, L) >> 1), el(lpos(64, L) & 1) {}
};
__device__ __forceinline__ void st64(double* d, size_t i, double2 v, Pair64 q) {
    if ((int)(i & 31) != q.pair) *(double2*)(d + 2 * i) = v;
    else d[2 * i + (1 - q.el)] = q.el ? v.x : v.y;
}
// st64 with the level-L element written too, with kl (its kept value: keep tails, mpas_dev.h):
// every line of the column whole
__device__ __forceinline__ void st64k(double* d, size_t i, double2 v, Pair64 q, double kl) {
    if ((int)(i & 31) == q.pair) {
        if (q.el) v.y = kl;
        else v.x = kl;
    }
    *(double2*)(d + 2 * i) = v;
}

// ---------------------------------------------------------------- vert_imp
// one column of atm_compute_vert_imp_coefs from its loaded inputs (k_vert_imp, and the
// stage-0 fusion with the setup copies and the moist coefficients, k_setup_vi)
template <int LP, bool MPASV>
__device__ __forceinline__ void vi_column(const DevState& S, int c, int k, double zz, double exner, double tm, double cqw,
                                          double qtot, double rb, double rtb, double rtp, double exb, double gamma_old,
                                          double coftz_old, double dtseps, double rcv, double c2, bool live = true,
                                          bool nbc = false) {
    // (nbc, atm_srk3 option ntu: stage 0's vert_imp -- b_tri and c_tri are dead there: stage 1's vert_imp
    // rewrites both and no task reads them in between, nor does that vert_imp; not stored)
    const int L = S.L;
    const double *fzm_a = fd(S, F_fzm), *fzp_a = fd(S, F_fzp), *rdzu_a = fd(S, F_rdzu), *rdzw_a = fd(S, F_rdzw);
    const double fzm = fzm_a[k], fzp = fzp_a[k], rdzu = rdzu_a[k], rdzw = rdzw_a[k];
    const double rdzw_m = k > 0 ? rdzw_a[k - 1] : 0.0;
    const double zz_m = lvl_dn<LP>(zz, k), exner_m = lvl_dn<LP>(exner, k), tm_m = lvl_dn<LP>(tm, k);

    // :550-564
    double cofwr = 0.0, cofwz = 0.0, coftz = coftz_old, cofwt = 0.0;
    if (k < L) {
        if (k > 0) cofwr = .5 * dtseps * kGravity * (fzm * zz + fzp * zz_m);
        coftz = 0.0;
        if (k > 0) {
            cofwz = dtseps * c2 * (fzm * zz + fzp * zz_m) * rdzu * cqw * (fzm * exner + fzp * exner_m);
            coftz = dtseps * (fzm * tm + fzp * tm_m);
        }
        double qtotal = qtot;
        cofwt = .5 * dtseps * rcv * zz * kGravity * rb / (1.0 + qtotal) * exner / ((rtb + rtp) * exb);
    }
    const double coftz_m = lvl_dn<LP>(coftz, k), coftz_p = lvl_up<LP>(coftz, k);
    const double cofwt_m = lvl_dn<LP>(cofwt, k);
    const double gamma_dn = lvl_dn<LP>(gamma_old, k);  // shuffle outside any branch
    const double gamma_m = (k == 1) ? 0.0 : gamma_dn;  // Q17: gamma(0) was just zeroed
    const double cofrz = dtseps * rdzw, cofrz_m = dtseps * rdzw_m;      // :537-539

    // :566-578 (every lane; used at 0 < k < L)
    const double a = -1.0 * cofwz * coftz_m * rdzw_m * zz_m + cofwr * cofrz_m - cofwt_m * coftz_m * rdzw_m;
    const double b = MPASV ? 1.0 + cofwz * (coftz * rdzw * zz + coftz * rdzw_m * zz_m) -
                                 coftz * (cofwt * rdzw - cofwt_m * rdzw_m) + cofwr * ((cofrz - cofrz_m))
                           : 1.0 + cofwz * (coftz * rdzw * zz + coftz * rdzw_m * zz_m) -
                                 coftz * (cofwt * rdzw - cofwt * rdzw_m) + cofwr * ((cofrz - cofrz_m));  // Q16 literal
    const double cc = -1.0 * cofwz * coftz_p * rdzw * zz - cofwr * cofrz + cofwt * coftz_p * rdzw;
    double alpha, gamma;
    if constexpr (MPASV) {
        // level by level: a nonlinear recurrence (a prefix scan of its Moebius maps measured
        // 2-4e-9 off the oracle over a step on the blowing-up random states, beyond RTOL_STEP).
        // The block's columns run it side by side, one lane per column, on their a / b / c
        // staged in LDS -- the level-by-level expressions, so the same values -- instead of
        // every lane of a column's wavefront stepping through all L - 1 levels.  Every wave of
        // the block reaches both barriers (callers clamp a dead column and pass live = false)
        constexpr int CPB = 256 / LP;
        __shared__ double s_a[CPB][LP], s_b[CPB][LP], s_c[CPB][LP];
        const int j = (int)(threadIdx.x / LP);
        s_a[j][k] = a;
        s_b[j][k] = b;
        s_c[j][k] = cc;
        __syncthreads();
        if ((int)threadIdx.x < CPB) {
            const int jj = (int)threadIdx.x;
            double gp = 0.0;
            for (int kk = 1; kk < L; kk++) {
                const double al = 1.0 / (s_b[jj][kk] - s_a[jj][kk] * gp);
                gp = s_c[jj][kk] * al;
                s_a[jj][kk] = al;  // (alpha)
                s_c[jj][kk] = gp;  // (gamma)
            }
        }
        __syncthreads();
        const bool in = k >= 1 && k < L;
        alpha = in ? s_a[j][k] : 0.0;
        gamma = in ? s_c[j][k] : 0.0;
    } else {
        alpha = 1.0 / (b - a * gamma_m);  // :580-585
        gamma = cc * alpha;               // :587-591
    }

    // written: every level but L (padding levels: zeros, full 64-B sectors; see PADW); the
    // tridiagonal coefficients not at level 0 either, gamma_tri 0.0 there.  Paired 16-B
    // stores (put2: every lane takes part)
    // (the slots the reference leaves -- level L, and level 0 of the tridiagonal coefficients --
    // written with their kept values: keep tails, mpas_dev.h; every line of a column whole)
    auto kL = [&](int f) { return keepv<LP>(S, f, KC, c); };
    auto k0 = [&](int f) { return keepv<LP>(S, f, KC, c, true); };
    put2<LP>(fw(S, F_coftz), c, fw(S, F_cofwt), c, k, KEEPW(coftz, kL(F_coftz)), KEEPW(cofwt, kL(F_cofwt)), live, live);
    put2<LP>(fw(S, F_cofwr), c, fw(S, F_cofwz), c, k, KEEPW0(cofwr, k0(F_cofwr), kL(F_cofwr)),
             KEEPW0(cofwz, k0(F_cofwz), kL(F_cofwz)), live, live);
    if (nbc) {
        if (live) {
            colk(fw(S, F_a_tri), c) = KEEPW0(a, k0(F_a_tri), kL(F_a_tri));
            colk(fw(S, F_alpha_tri), c) = KEEPW0(alpha, k0(F_alpha_tri), kL(F_alpha_tri));
        }
    } else {
        put2<LP>(fw(S, F_a_tri), c, fw(S, F_b_tri), c, k, KEEPW0(a, k0(F_a_tri), kL(F_a_tri)),
                 KEEPW0(b, k0(F_b_tri), kL(F_b_tri)), live, live);
        put2<LP>(fw(S, F_c_tri), c, fw(S, F_alpha_tri), c, k, KEEPW0(cc, k0(F_c_tri), kL(F_c_tri)),
                 KEEPW0(alpha, k0(F_alpha_tri), kL(F_alpha_tri)), live, live);
    }
    if (live) colk(fw(S, F_gamma_tri), c) = k == 0 ? 0.0 : KEEPW(gamma, kL(F_gamma_tri));
    if (live && c == 0 && k < L) fw(S, F_cofrz)[k] = cofrz;
}

template <int LP, bool MPASV>
__device__ __forceinline__ void vert_imp_body(const DevState& S, double dtseps, double rcv, double c2, Blk bk) {
    ColMap<LP> m(S, KC, bk);
    const int k = m.k;
    const bool live = m.ent < S.nCO;
    if (!MPASV && !live) return;  // (MPASV: vi_column's barriers need every wave; a dead column
    const int c = live ? m.ent : S.nCO - 1;  // loads the last one and stores nothing)
    // (gather2: two own columns per 16-B load instruction)
    double zz, exner, tm, cqw, qtot, rb, rtb, rtp, exb, gamma_old;
    gather2<LP>(fd(S, F_zz), c, fd(S, F_exner), c, k, zz, exner);
    gather2<LP>(fd(S, F_theta_m), c, fd(S, F_cqw), c, k, tm, cqw);
    gather2<LP>(fd(S, F_qtot), c, fd(S, F_rho_base), c, k, qtot, rb);
    gather2<LP>(fd(S, F_rtheta_base), c, fd(S, F_rtheta_p), c, k, rtb, rtp);
    gather2<LP>(fd(S, F_exner_base), c, fd(S, F_gamma_tri), c, k, exb, gamma_old);
    const double coftz_old = colk(fd(S, F_coftz), c);  // level L keeps its (never written) value
    vi_column<LP, MPASV>(S, c, k, zz, exner, tm, cqw, qtot, rb, rtb, rtp, exb, gamma_old, coftz_old, dtseps, rcv, c2,
                         live);
}


// ---------------------------------------------------------------- divergence damping
// OLD0: rtheta_pp_old is known to be 0.0 (srk3, right after the first acoustic substep
// of a stage, which sets it so on every cell, :1615-1618): its columns are not read, and
// -(r - 0.0) is the same value as the literal expression gives
// DIVB (option fusedamp, the step's last damping): the cells' div = -(rtheta_pp -
// rtheta_pp_old) comes from the acoustic step's X_dvB (the same subtraction, made there)
template <int LP, int EPW, bool OLD0, bool DIVB = false, bool TME = false>
__device__ __forceinline__ void divdamp_body(const DevState& S, double coef_divdamp, Blk bk) {
    ColMapN<LP, EPW> m(S, KE, bk);
    const int L = S.L, k = m.k;
    const int *coe = fi(S, F_cellsOnEdge), *sh = fi(S, F_isShared);
    const double *rtp = fd(S, F_rtheta_pp), *rtpo = fd(S, F_rtheta_pp_old), *tm = fd(S, F_theta_m);
    const double* spz = fd(S, F_specZoneMaskEdge);
    double* rup = fw(S, F_ru_p);
    // every load of the EPW edges first (the isShared test only decides the store)
    int c1[EPW], c2[EPW], sh1[EPW], sh2[EPW];
    double r1[EPW], ro1[EPW], r2[EPW], ro2[EPW], t1[EPW], t2[EPW], ru[EPW], spec[EPW];
#pragma unroll
    for (int i = 0; i < EPW; i++) {
        const int e = min(m.base + i, S.nEO - 1);
        c1[i] = coe[(size_t)e * 2];
        c2[i] = coe[(size_t)e * 2 + 1];
        spec[i] = spz[e];
        ru[i] = colk(rup, e);
    }
#pragma unroll
    for (int i = 0; i < EPW; i++) {
        sh1[i] = sh[c1[i]];
        sh2[i] = sh[c2[i]];
        if (DIVB) {
            gather2s<LP>(fd(S, X_dvB), c1[i], c2[i], k, r1[i], r2[i]);
            ro1[i] = ro2[i] = 0.0;
        } else {
            gather2s<LP>(rtp, c1[i], c2[i], k, r1[i], r2[i]);
            if (OLD0) ro1[i] = ro2[i] = 0.0;
            else gather2s<LP>(rtpo, c1[i], c2[i], k, ro1[i], ro2[i]);
        }
        if (TME) {  // theta_m(cell2) + theta_m(cell1) from X_tme (atm_srk3, option tmedge)
            t1[i] = colk(fd(S, X_tme), min(m.base + i, S.nEO - 1));
            t2[i] = 0.0;
        } else {
            gather2s<LP>(tm, c1[i], c2[i], k, t1[i], t2[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < EPW; i++) {
        const int e = m.base + i;
        if (e >= S.nEO || (sh1[i] && sh2[i])) continue;
        double divCell1 = DIVB ? r1[i] : -(r1[i] - ro1[i]);
        double divCell2 = DIVB ? r2[i] : -(r2[i] - ro2[i]);
        // (levels >= L: the value loaded, zeros on the padding -- the column's lines written whole)
        colk(rup, e) = k < L ? ru[i] + coef_divdamp * (divCell2 - divCell1) * (1.0 - spec[i]) / (TME ? t1[i] : t1[i] + t2[i])
                             : PADW(ru[i]);
    }
}

// ---------------------------------------------------------------- substep finish
// cells: the cell part (else the edges); blocks b of nb cover its pairs (grid stride)
// (CELLS a template argument: every keep tail is addressed with a constant entity kind -- a runtime
// kind select in keep_tail was miscompiled once, mpas_dev.h k_keep_refresh)
template <bool CELLS>
// (norz, atm_srk3 in the reference semantics: the copy rho_zz = rho_zz_old_split is the identity -- this
// step's setup made rho_zz_old_split from rho_zz, with the same levels and keep tails, and nothing writes
// either in between -- so it is not made)
__device__ __forceinline__ void finish64_part(const DevState& S, int substep, int split, double inv_split, Pair64 q,
                                              int b, int nb, int norz = 0) {
    constexpr bool cells = CELLS;
    constexpr int kind = CELLS ? KC : KE;
    const size_t n = (size_t)(cells ? S.nCO : S.nEO) * 32;
    double *avg = fw(S, cells ? F_wwAvg : F_ruAvg), *avgS = fw(S, cells ? F_wwAvg_split : F_ruAvg_split);
    const bool restore = substep < split, last = substep == split, same = substep == 1 && inv_split == 1.0;
    for (size_t i = (size_t)b * 256 + threadIdx.x; i < n; i += (size_t)nb * 256) {
        // (level L: the kept value of the destination -- its keep tail, or for the averages the
        // value just loaded -- so every line of a column is written whole)
        const int col = (int)(i >> 5);
        auto cp = [&](int from, int to) {
            st64k(fw(S, to), i, ((const double2*)fd(S, from))[i], q, keepv<64>(S, to, kind, col));
        };
        if (restore) {
            if (cells) {
                cp(F_rw, F_rw_save);
                cp(F_rtheta_p, F_rtheta_p_save);
                cp(F_rho_p, F_rho_p_save);
                cp(F_w_2, F_w);
                cp(F_theta_m_2, F_theta_m);
                cp(F_rho_zz_2, F_rho_zz);
            } else {
                cp(F_ru, F_ru_save);
                cp(F_u_2, F_u);
            }
        }
        const double2 a = ((const double2*)avg)[i];
        double2 sv = a;
        if (substep != 1) {
            const double2 b = ((const double2*)avgS)[i];
            sv = make_double2(a.x + b.x, a.y + b.y);
        }
        st64k(avgS, i, sv, q, keepv<64>(S, cells ? F_wwAvg_split : F_ruAvg_split, kind, col));
        if (last && !same) st64k(avg, i, make_double2(sv.x * inv_split, sv.y * inv_split), q, q.el ? a.y : a.x);
        if (cells && last && S.physics != 2 && !norz) cp(F_rho_zz_old_split, F_rho_zz);
    }
}
__device__ __forceinline__ void finish64_body(const DevState& S, int substep, int split, double inv_split, Pair64 q,
                                              bool cells, int b, int nb, int norz = 0) {
    if (cells) finish64_part<true>(S, substep, split, inv_split, q, b, nb, norz);
    else finish64_part<false>(S, substep, split, inv_split, q, b, nb, norz);
}


// ---------------------------------------------------------------- solve_diagnostics
// MD: the MPAS dynamics (physics = 2, ora_mpas_solve_diagnostics): divergence += s * u (Q9),
// h = rho_zz and rho_edge = h_edge (Q2: MPAS-A passes diag%rho_edge as h_edge), v over
// every edgesOnEdge entry (Q23)
// LIVE (atm_srk3 option ntu: a call before the last stage's, the next stage at rk_step > 0): only what
// the next stage's dyn_tend reads is stored -- ke, and pv_vertex for pv_edge (MD: rho_edge too).
// vorticity, divergence, h_edge and ke_edge have no reader before the last stage's solve_diagnostics
// rewrites them (dyn_tend reads divergence and vorticity at rk_step 0 only; nothing reads h_edge or
// ke_edge)
template <int LP, int EPW, bool MD, bool LIVE = false>
__device__ __forceinline__ void solve_vc_body(const DevState& S, int nVB, int hollingsworth_part, Blk bk) {
    const int L = S.L;
    const double* u = fd(S, F_u);
    const double *dcEdge = fd(S, F_dcEdge), *dvEdge = fd(S, F_dvEdge);
    ColMapN<LP, EPW> m(S, KV, bk);
    const int k = m.k;
    int bi;
    if (vc_block(S, m.blk, nVB, bi, bk.n)) {  // EPW vertices: vorticity, pv_vertex (:381-396)
        m.base = col_of<LP>(bi) * EPW + S.lo[KV];
        int ev[EPW][3];
        double sg_[EPW][3], dc_[EPW][3], u_[EPW][3], iat[EPW], fv[EPW];
#pragma unroll
        for (int j = 0; j < EPW; j++) {
            const int v = min(m.base + j, S.nVO - 1);
            row_ld(fi(S, F_edgesOnVertex) + (size_t)v * 3, ev[j]);
            row_ld(fd(S, F_edgesOnVertexSign) + (size_t)v * 3, sg_[j]);
            row_ld(fd(S, X_ve_dc) + (size_t)v * 3, dc_[j]);  // dcEdge(edgesOnVertex)
            iat[j] = ldc(fd(S, F_invAreaTriangle) + v);
            fv[j] = ldc(fd(S, F_fVertex) + v);
        }
#pragma unroll
        for (int j = 0; j < EPW; j++) gather2s<LP>(u, ev[j][0], ev[j][1], k, u_[j][0], u_[j][1]);
#pragma unroll
        for (int j = 0; j + 1 < EPW; j += 2) gather2s<LP>(u, ev[j][2], ev[j + 1][2], k, u_[j][2], u_[j + 1][2]);
        if (EPW % 2) u_[EPW - 1][2] = colk(u, ev[EPW - 1][2]);
#pragma unroll
        for (int j = 0; j < EPW; j++) {
            const int v = m.base + j;
            if (v >= S.nVO) break;  // (wave-uniform; padding levels: zeros, PADW)
            double vort = 0.0;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                double s = sg_[j][i] * dc_[j][i];
                vort += s * u_[j][i];
            }
            vort *= iat[j];
            // (one paired 16-B store, every lane; level L keeps its value)
            // (level L left unwritten, as the reference: the keep tails cost this kernel 12 %)
            if constexpr (LIVE) {
                if (k != L) colk(fw(S, F_pv_vertex), v) = PADW(fv[j] + vort);
            } else {
                put2<LP>(fw(S, F_vorticity), v, fw(S, F_pv_vertex), v, k, PADW(vort), PADW(fv[j] + vort), k != L, k != L);
            }
            if (k == L) continue;
            if (hollingsworth_part) {
                double r = 0.25 * iat[j];
                double kes[3];
                for (int i = 0; i < 3; i++) {
                    int iEdge = ev[j][i];
                    double efac = dcEdge[iEdge] * dvEdge[iEdge];
                    double uu = u_[j][i];
                    kes[i] = (iEdge < S.nEdges) ? efac * (uu * uu) : 0.0;
                }
                colk(fw(S, F_ke_vertex), v) = PADW((kes[0] + kes[1] + kes[2]) * r);
            }
        }
        return;
    }
    // EPW cells: divergence (Q9 "s + u") and ke (:369-379, :357-367)
    const int c0 = col_of<LP>(bi) * EPW + S.lo[KC];
    int ne[EPW], e_[EPW][NF];
    double u_[EPW][NF], sgn_[EPW][NF], dv_[EPW][NF], dc_[EPW][NF], invA[EPW];
#pragma unroll
    for (int j = 0; j < EPW; j++) {
        const int c = min(c0 + j, S.nCO - 1);
        ne[j] = ldc(fi(S, F_nEdgesOnCell) + c);
        invA[j] = ldc(fd(S, F_invAreaCell) + c);
        row_ld(fi(S, F_edgesOnCell) + (size_t)c * 10, e_[j]);
        row_ld(fd(S, F_edgesOnCellSign) + (size_t)c * 10, sgn_[j]);
        row_ld(fd(S, X_ce_dv) + (size_t)c * 10, dv_[j]);  // dvEdge(edgesOnCell)
        row_ld(fd(S, X_ce_dc) + (size_t)c * 10, dc_[j]);  // dcEdge(edgesOnCell)
    }
#pragma unroll
    for (int j = 0; j < EPW; j++)
#pragma unroll
        for (int i = 0; i < NF; i += 2) gather2s<LP>(u, e_[j][i], e_[j][i + 1], k, u_[j][i], u_[j][i + 1]);
#pragma unroll
    for (int j = 0; j < EPW; j++) {
        const int c = c0 + j;
        if (c >= S.nCO) break;  // (wave-uniform; padding levels: zeros, PADW)
        double div = 0.0, ke = 0.0;
#pragma unroll
        for (int i = 0; i < NF; i++) {
            const double uu = u_[j][i];
            double s = sgn_[j][i] * dv_[j][i];
            div = add_if(i < ne[j], div, MD ? s * uu : s + uu);
            // ke_edge(iEdge,k) exactly as the edge loop (:352) writes it; the zero slot
            // row of ke_edge is never written, and its recomputation is 0*0*0 as well
            double efac = dc_[j][i] * dv_[j][i];
            double kee = (e_[j][i] < S.nEdges) ? efac * (uu * uu) : 0.0;
            ke = add_if(i < ne[j], ke, 0.25 * kee);
        }
        const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
        const double* sgn = fd(S, F_edgesOnCellSign) + (size_t)c * 10;
        for (int i = NF; i < ne[j]; i++) {
            int iEdge = eoc[i];
            double uu = colk(u, iEdge);
            double s = sgn[i] * dvEdge[iEdge];
            div += MD ? s * uu : s + uu;
            double efac = dcEdge[iEdge] * dvEdge[iEdge];
            double kee = (iEdge < S.nEdges) ? efac * (uu * uu) : 0.0;
            ke += 0.25 * kee;
        }
        div *= invA[j];
        ke *= invA[j];
        // (one paired 16-B store, every lane; level L keeps its value)
        if constexpr (LIVE) {
            if (k != L) colk(fw(S, F_ke), c) = PADW(ke);
        } else {
            put2<LP>(fw(S, F_divergence), c, fw(S, F_ke), c, k, PADW(div), PADW(ke), k != L, k != L);
        }
    }
}

// EPW consecutive edges per column slot (option "epw"): the loads of all of them are issued
// before the first store; the paired 16-B stores write h_edge with ke_edge and pv_edge with
// v (or alone) -- every lane takes part (put2), level L keeps its value
// LIVE (see solve_vc_body): pv_edge alone (MD: and rho_edge)
template <int LP, bool RECON_V, bool MD, int EPW, bool LIVE = false>
__device__ __forceinline__ void solve_e_body(const DevState& S, Blk bk) {
    static_assert(!LIVE || !RECON_V, "the dead diagnostics: no v");
    ColMapN<LP, EPW> m(S, KE, bk);
    const int L = S.L, k = m.k;
    const double *h = fd(S, MD ? F_rho_zz : F_h), *u = fd(S, F_u), *pvv = fd(S, F_pv_vertex);
    double h1[EPW], h2[EPW], uu[EPW], pv1[EPW], pv2[EPW], vv[EPW];
    int ee[EPW];
#pragma unroll
    for (int j = 0; j < EPW; j++) {
        const int e = min(m.base + j, S.nEO - 1);
        ee[j] = e;
        const int* coe = fi(S, F_cellsOnEdge) + (size_t)e * 2;
        const int* voe = fi(S, F_verticesOnEdge) + (size_t)e * 2;
        if constexpr (LIVE && !MD) h1[j] = h2[j] = 0.0;
        else gather2s<LP>(h, coe[0], coe[1], k, h1[j], h2[j]);
        gather2s<LP>(pvv, voe[0], voe[1], k, pv1[j], pv2[j]);
    }
#pragma unroll
    for (int j = 0; j < EPW; j++) {
        const int e = ee[j];
        vv[j] = 0.0;
        if (RECON_V) {
            const int* eoe = fi(S, F_edgesOnEdge_ECP) + (size_t)e * 20;
            const double* wts = fd(S, F_weightsOnEdge) + (size_t)e * 20;
            const int neoe = fi(S, F_nEdgesOnEdge)[e];
            int ee_[QF];
            double ue[QF], wts_[QF];
            row_ld(eoe, ee_);
            row_ld(wts, wts_);
            static_assert(QF == 10, "pairs below");
            if (MD) {
#pragma unroll
                for (int i = 0; i < QF; i += 2) gather2s<LP>(u, ee_[i], ee_[i + 1], k, ue[i], ue[i + 1]);
                uu[j] = colk(u, e);
            } else {
#pragma unroll
                for (int i = 1; i < QF - 1; i += 2) gather2s<LP>(u, ee_[i], ee_[i + 1], k, ue[i], ue[i + 1]);
                gather2s<LP>(u, ee_[QF - 1], e, k, ue[QF - 1], uu[j]);
            }
            double v = 0;  // Q23: the sum starts at i = 1
#pragma unroll
            for (int i = MD ? 0 : 1; i < QF; i++) v = add_if(i < neoe, v, wts_[i] * ue[i]);
            for (int i = QF; i < neoe; i++) v += wts[i] * colk(u, eoe[i]);
            vv[j] = v;
        } else {
            uu[j] = LIVE ? 0.0 : colk(u, e);
        }
    }
#pragma unroll
    for (int j = 0; j < EPW; j++) {
        const int e = m.base + j;
        if (e >= S.nEO) break;  // (wave-uniform)
        const double efac = fd(S, F_dcEdge)[e] * fd(S, F_dvEdge)[e];
        // (padding levels k > L: zeros; level L: the kept values, keep tails in mpas_dev.h)
        auto kL = [&](int f) { return keepv<LP>(S, f, KE, e); };
        if constexpr (LIVE) {
            if (MD) colk(fw(S, F_rho_edge), e) = KEEPW(0.5 * (h1[j] + h2[j]), kL(F_rho_edge));
            colk(fw(S, F_pv_edge), e) = KEEPW(0.5 * (pv1[j] + pv2[j]), kL(F_pv_edge));
            continue;
        }
        put2f<LP>(fw(S, F_h_edge), e, fw(S, F_ke_edge), e, k, KEEPW(0.5 * (h1[j] + h2[j]), kL(F_h_edge)),
                 KEEPW(efac * (uu[j] * uu[j]), kL(F_ke_edge)));
        if (MD) colk(fw(S, F_rho_edge), e) = KEEPW(0.5 * (h1[j] + h2[j]), kL(F_rho_edge));
        if (RECON_V)
            put2f<LP>(fw(S, F_v), e, fw(S, F_pv_edge), e, k, KEEPW(vv[j], kL(F_v)),
                     KEEPW(0.5 * (pv1[j] + pv2[j]), kL(F_pv_edge)));
        else colk(fw(S, F_pv_edge), e) = KEEPW(0.5 * (pv1[j] + pv2[j]), kL(F_pv_edge));
    }
}


// ---------------------------------------------------------------- set_smlstep's flux sum
// X_smlS (atm_srk3 fast path, reference semantics; once per step: k_sml_flux, or a body of
// stage 0's combined hfuse launch): per cell and level k <= L the sum over the cell's edges of
// set_smlstep's slope-flux terms, in the order every fast-path set_smlstep adds them; and X_Dd
// = rw_save - rw for the stages' acoustic launches (the same difference they formed)
// SETUP: beside the stage-0 setup launch that is writing rw_save = rw (every level but L): rw
// stands in for rw_save (the same values where the acoustic step reads the difference)
template <int LP, bool SETUP = false>
__device__ __forceinline__ void sml_flux_body(const DevState& S, Blk bk) {
    ColMap<LP> m(S, KC, bk);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO) return;
    int e_[NF], c1_[NF], c2_[NF];
    const int ne = cell_rec<false>(S, c, e_, c1_, c2_);
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* sgnc = fd(S, F_edgesOnCell_sign) + (size_t)c * 10;
    const double *ut_f = fd(S, F_u_tend), *zb = fd(S, F_zb_cell), *zb3 = fd(S, F_zb3_cell);
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    double ut_[NF], utm_[NF], zb_[NF], zb3_[NF], sgs_[NF];
    row_ld(sgnc, sgs_);
#pragma unroll
    for (int i = 0; i < NF; i += 2) gather2s<LP>(ut_f, e_[i], e_[i + 1], k, ut_[i], ut_[i + 1]);
#pragma unroll
    for (int i = 0; i < NF; i++) {
        ut_[i] = ldz(k <= L, ut_[i]);
        gather2<LP>(zb, c * 10 + i, zb3, c * 10 + i, k, zb_[i], zb3_[i]);
    }
#pragma unroll
    for (int i = 0; i < NF; i++) utm_[i] = lvl_dn<LP>(ut_[i], k);
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        double flux = sgs_[i] * (fzm * ut_[i] + fzp * utm_[i]);
        sum = add_if(i < ne, sum, (zb_[i] + copysign(1.0, ut_[i]) * zb3_[i]) * flux);
    }
    for (int i = NF; i < ne; i++) {
        int iEdge = eoc[i];
        double ut = col_rd<LP>(ut_f, iEdge, k, L);
        double ut_m = lvl_dn<LP>(ut, k);
        double flux = sgnc[i] * (fzm * ut + fzp * ut_m);
        size_t q = ((size_t)c * 10 + i) * LP + lpos(LP, k);
        sum += (zb[q] + copysign(1.0, ut) * zb3[q]) * flux;
    }
    colk(fw(S, X_smlS), c) = k <= L ? sum : 0.0;
    double rws, rw;
    if constexpr (SETUP) rws = rw = col_rd<LP>(fd(S, F_rw), c, k, L);
    else col_rd2<LP>(fd(S, F_rw_save), fd(S, F_rw), c, k, L, rws, rw);
    // (level L: 0.0 in both forms -- the SETUP form's rw stands in for rw_save, which differs there;
    // the acoustic step reads the interfaces 1..L-1 only: ADVICE r05)
    colk(fw(S, X_Dd), c) = k < L ? rws - rw : 0.0;
}

// ---------------------------------------------------------------- setup + moist + vert_imp
// Stage 0 of atm_srk3 in one launch (option "fusesetup", reference semantics; k_setup_vi,
// k_misc.hip, and its combined launch with dyn_tend A, k_dyn.hip): blocks [0, ncb) one cell
// column each, the rest (if any) the edge copies ru_save = ru, u_2 = u
// MPASV (physics >= 1): vert_imp's MPAS form (vi_column); MD (physics = 2): also setup's
// theta_m_save = theta_m and moist's edge loop cqu = 1 / (1 + qtotal) (k_moist_edges), by the
// edge blocks, from the qtot this launch zeroes everywhere
template <int LP, bool MPASV = false, bool MD = false>
__device__ __forceinline__ void setup_vi_body(const DevState& S, int ncb, double dtseps, double rcv, double c2, Blk bk,
                                              int copies = 1) {
    const int L = S.L, k = (int)(threadIdx.x % LP);
    int blk = bk.b;
    if (blk >= ncb) {  // :767-771 ru_save = ru, u_2 = u (every level but L)
        const int e = col_of<LP>(xcd_block_n(S.xcd, blk - ncb, bk.n - ncb)) + S.lo[KE];
        if (e >= S.nEO) return;
        if (copies & 1) {
            double ru, u;
            gather2<LP>(fd(S, F_ru), e, fd(S, F_u), e, k, ru, u);
            put2f<LP>(fw(S, F_ru_save), e, fw(S, F_u_2), e, k, KEEPW(ru, keepv<LP>(S, F_ru_save, KE, e)),
                     KEEPW(u, keepv<LP>(S, F_u_2, KE, e)));
        }
        if constexpr (MD) {  // :491-501 (Q25 fixed): qtot(cell1) = qtot(cell2) = 0 just written
            const double q1 = 0.0, q2 = 0.0, qtotal = 0.5 * (q1 + q2);
            colk(fw(S, F_cqu), e) = KEEPW(1.0 / (1.0 + qtotal), keepv<LP>(S, F_cqu, KE, e));
        }
        return;
    }
    const int c0 = col_of<LP>(xcd_block_n(S.xcd, blk, ncb)) + S.lo[KC];
    const bool live = c0 < S.nCO;
    if (!MPASV && !live) return;  // (MPASV: as vert_imp_body)
    const int c = live ? c0 : S.nCO - 1;
    double rw, rtp, rp, w, tm, rz, zz, exner, rb, rtb, exb, gamma_old;
    gather2<LP>(fd(S, F_rw), c, fd(S, F_rtheta_p), c, k, rw, rtp);
    gather2<LP>(fd(S, F_rho_p), c, fd(S, F_w), c, k, rp, w);
    gather2<LP>(fd(S, F_theta_m), c, fd(S, F_rho_zz), c, k, tm, rz);
    gather2<LP>(fd(S, F_zz), c, fd(S, F_exner), c, k, zz, exner);
    gather2<LP>(fd(S, F_rho_base), c, fd(S, F_rtheta_base), c, k, rb, rtb);
    gather2<LP>(fd(S, F_exner_base), c, fd(S, F_gamma_tri), c, k, exb, gamma_old);
    const double coftz_old = colk(fd(S, F_coftz), c);
    // :773-777 the save copies (every level but L; padding levels carry zeros either way)
    // (level L: the kept values, keep tails in mpas_dev.h -- every line of a column whole)
    auto kL = [&](int f) { return keepv<LP>(S, f, KC, c); };
    put2<LP>(fw(S, F_rw_save), c, fw(S, F_rtheta_p_save), c, k, KEEPW(rw, kL(F_rw_save)),
             KEEPW(rtp, kL(F_rtheta_p_save)), live, live);
    put2<LP>(fw(S, F_rho_p_save), c, fw(S, F_w_2), c, k, KEEPW(rp, kL(F_rho_p_save)), KEEPW(w, kL(F_w_2)), live, live);
    put2<LP>(fw(S, F_theta_m_2), c, fw(S, F_rho_zz_2), c, k, KEEPW(tm, kL(F_theta_m_2)), KEEPW(rz, kL(F_rho_zz_2)),
             live, live);
    if constexpr (MD)
        put2<LP>(fw(S, F_rho_zz_old_split), c, fw(S, F_theta_m_save), c, k, KEEPW(rz, kL(F_rho_zz_old_split)),
                 KEEPW(tm, kL(F_theta_m_save)), live, live);
    else if (live) colk(fw(S, F_rho_zz_old_split), c) = KEEPW(rz, kL(F_rho_zz_old_split));
    // :473-489 (k_moist's expressions): qtot = 0; cqw(k > 0) from the two zeroed qtot
    const double q_k = 0.0, q_km1 = 0.0, qtotal = 0.5 * (q_k + q_km1);
    const double cqw = k > L ? 0.0 : 1.0 / (1.0 + qtotal), qtot = 0.0;
    put2<LP>(fw(S, F_qtot), c, fw(S, F_cqw), c, k, KEEPW(qtot, kL(F_qtot)),
             KEEPW0(cqw, keepv<LP>(S, F_cqw, KC, c, true), kL(F_cqw)), live, live);
    // (cqw is used at 0 < k < L only, qtot at k < L: the values just written)
    vi_column<LP, MPASV>(S, c, k, zz, exner, tm, cqw, qtot, rb, rtb, rtp, exb, gamma_old, coftz_old, dtseps, rcv, c2,
                         live, (copies & 2) != 0);  // (copies bit 1: b_tri / c_tri dead, atm_srk3 option ntu)
}
}  // namespace mpas
