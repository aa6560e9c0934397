// k_misc.hip -- column-local and streaming tasks of the RK3 step (gfx950):
//   atm_rk_integration_setup        dynamics_tasks.rg:747-778
//   atm_compute_moist_coefficients  dynamics_tasks.rg:460-502
//   atm_compute_vert_imp_coefs      dynamics_tasks.rg:513-592
//   atm_set_smlstep_pert_variables  dynamics_tasks.rg:1503-1528
//   atm_divergence_damping_3d       dynamics_tasks.rg:1726-1763
//   atm_rk_dynamics_substep_finish  dynamics_tasks.rg:1951-2007
//   synthetic-state fill (mpas_synth.h, identical to the oracle's generator)
// All are HBM-streaming (fp64, no MFMA).  Expressions are written in the Regent
// operand order and the library is built with -ffp-contract=off, so results are
// bit-identical to the oracle's.
#include "mpas_dev.h"
#include "mpas_halo.h"
#include "k_cols.h"
#include "mpas_synth.h"

namespace mpas {

// ---------------------------------------------------------------- setup
__global__ __launch_bounds__(256) void k_setup_cells(DevState S) {
    const size_t n = (size_t)S.nCO * S.LP;
    const double *rw = fd(S, F_rw), *rtp = fd(S, F_rtheta_p), *rp = fd(S, F_rho_p), *w = fd(S, F_w);
    const double *tm = fd(S, F_theta_m), *rz = fd(S, F_rho_zz);
    double *rws = fw(S, F_rw_save), *rtps = fw(S, F_rtheta_p_save), *rps = fw(S, F_rho_p_save);
    double *w2 = fw(S, F_w_2), *tm2 = fw(S, F_theta_m_2), *rz2 = fw(S, F_rho_zz_2), *rzo = fw(S, F_rho_zz_old_split);
    double* tms = fw(S, F_theta_m_save);
    const bool md = S.physics == 2;  // the MPAS dynamics: theta_m_save = theta_m (never written, Q2)
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (plev(S.LP, (int)(i & (size_t)(S.LP - 1))) == S.L) continue;  // (padding copied: zeros, full 64-B sectors)
        rws[i] = rw[i];
        rtps[i] = rtp[i];
        rps[i] = rp[i];
        w2[i] = w[i];
        tm2[i] = tm[i];
        if (md) tms[i] = tm[i];
        double r = rz[i];
        rz2[i] = r;
        rzo[i] = r;
    }
}
__global__ __launch_bounds__(256) void k_setup_edges(DevState S) {
    const size_t n = (size_t)S.nEO * S.LP;
    const double *ru = fd(S, F_ru), *u = fd(S, F_u);
    double *rus = fw(S, F_ru_save), *u2 = fw(S, F_u_2);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (plev(S.LP, (int)(i & (size_t)(S.LP - 1))) == S.L) continue;  // (padding copied: zeros, full 64-B sectors)
        rus[i] = ru[i];
        u2[i] = u[i];
    }
}
static int stream_grid(size_t n) {
    size_t g = (n + 255) / 256;
    return (int)(g < 8192 ? (g ? g : 1) : 8192);
}

struct CopyList {
    const double* src[8];
    double* dst[8];
    double* dst2[8];  // optional second destination of the same source (nullptr: none)
    size_t npair[8];
};
__global__ __launch_bounds__(256) void k_copy64(CopyList cl, Pair64 q) {
    const int j = blockIdx.y;
    const double2* s = (const double2*)cl.src[j];
    double *d = cl.dst[j], *d2 = cl.dst2[j];
    const size_t n = cl.npair[j];
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const double2 v = s[i];
        st64(d, i, v, q);
        if (d2) st64(d2, i, v, q);
    }
}
static void copy64(const DevState& S, hipStream_t st, const CopyList& cl, int ncopy) {
    size_t nmax = 0;
    for (int j = 0; j < ncopy; j++) nmax = cl.npair[j] > nmax ? cl.npair[j] : nmax;
    const int gx = (int)((stream_grid(nmax) + 3) / 4);
    if (nmax) k_copy64<<<dim3(gx, ncopy), 256, 0, st>>>(cl, Pair64(S.L));
}

hipError_t launch_rk_integration_setup(const DevState& S, hipStream_t st) {
    if (S.LP == 64) {
        CopyList cl{};
        int n = 0;
        const size_t ne = (size_t)S.nEO * 32, nc = (size_t)S.nCO * 32;
        auto add = [&](int from, int to, int to2, size_t np) {
            cl.src[n] = (const double*)S.f[from];
            cl.dst[n] = (double*)S.f[to];
            cl.dst2[n] = to2 >= 0 ? (double*)S.f[to2] : nullptr;
            cl.npair[n++] = np;
        };
        add(F_ru, F_ru_save, -1, ne);
        add(F_u, F_u_2, -1, ne);
        add(F_rw, F_rw_save, -1, nc);
        add(F_rtheta_p, F_rtheta_p_save, -1, nc);
        add(F_rho_p, F_rho_p_save, -1, nc);
        add(F_w, F_w_2, -1, nc);
        add(F_theta_m, F_theta_m_2, S.physics == 2 ? F_theta_m_save : -1, nc);
        add(F_rho_zz, F_rho_zz_2, F_rho_zz_old_split, nc);
        copy64(S, st, cl, n);
    } else {
        k_setup_edges<<<stream_grid((size_t)S.nEO * S.LP), 256, 0, st>>>(S);
        k_setup_cells<<<stream_grid((size_t)S.nCO * S.LP), 256, 0, st>>>(S);
    }
    HALO_WROTE(S, F_ru_save, F_u_2, F_rw_save, F_rtheta_p_save, F_rho_p_save, F_w_2, F_theta_m_2, F_rho_zz_2,
               F_rho_zz_old_split);
    if (S.physics == 2) HALO_WROTE(S, F_theta_m_save);
    return hipGetLastError();
}

// ---------------------------------------------------------------- moist
__global__ __launch_bounds__(256) void k_moist(DevState S) {
    const size_t n = (size_t)S.nCO * S.LP;
    double *qtot = fw(S, F_qtot), *cqw = fw(S, F_cqw);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        int k = plev(S.LP, (int)(i & (size_t)(S.LP - 1)));
        if (k == S.L) continue;  // (padding levels k > L get zeros: full 64-B sectors)
        qtot[i] = 0.0;  // :473-482
        if (k > S.L) {
            cqw[i] = 0.0;
        } else if (k > 0) {  // :484-489, qtot(k) and qtot(k-1) were both just zeroed
            double q_k = 0.0, q_km1 = 0.0;
            double qtotal = 0.5 * (q_k + q_km1);
            cqw[i] = 1.0 / (1.0 + qtotal);
        }
    }
}
// the MPAS dynamics (physics = 2): the edge loop of :491-501 the reference comments out
// (Q25), cqu = 1 / (1 + qtotal), qtotal = 0.5 (qtot(cell1) + qtot(cell2)) of the qtot the
// cell loop has just zeroed everywhere (the zero slot is 0 too)
__global__ __launch_bounds__(256) void k_moist_edges(DevState S) {
    const size_t n = (size_t)S.nEO * S.LP;
    double* cqu = fw(S, F_cqu);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const int k = plev(S.LP, (int)(i & (size_t)(S.LP - 1)));
        if (k == S.L) continue;
        const double q1 = 0.0, q2 = 0.0, qtotal = 0.5 * (q1 + q2);
        cqu[i] = k > S.L ? 0.0 : 1.0 / (1.0 + qtotal);
    }
}
hipError_t launch_moist_coefficients(const DevState& S, hipStream_t st) {
    k_moist<<<stream_grid((size_t)S.nCO * S.LP), 256, 0, st>>>(S);
    HALO_WROTE(S, F_qtot, F_cqw);
    if (S.physics == 2) {
        k_moist_edges<<<stream_grid((size_t)S.nEO * S.LP), 256, 0, st>>>(S);
        HALO_WROTE(S, F_cqu);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- vert_imp
// MPASV: the MPAS vertical solver (option "physics" = 1, oracle ora_mpas_vert_imp_coefs):
// b_tri with cofwt(k-1) (Q16) and the LU recurrence alpha(k) = 1 / (b(k) - a(k) gamma(k-1)),
// gamma(k) = c(k) alpha(k) from gamma(0) = 0 within the call (Q17), level by level
// (a nonlinear recurrence: lane k waits for lane k-1's gamma, broadcast by a shuffle)
// Stage 0 of atm_srk3 in one launch (option "fusesetup", reference semantics): the copies
// of atm_rk_integration_setup (:747-778), atm_compute_moist_coefficients (:460-502) and
// the first atm_compute_vert_imp_coefs (:513-592) -- all column-local, run in this order
// by one wavefront per cell column: vert_imp takes theta_m and rtheta_p from the copy's
// loads and qtot / cqw as moist has just set them, so those four columns are read once.
// Edge blocks (ncb..) copy ru and u (none with option "fusecopy": dyn_tend's edge kernel
// makes those copies).  The same values as the three launches.
// MPAS vertical solver / dynamics (physics 1 / 2): the same fusion with vert_imp's MPAS form,
// and under the MPAS dynamics setup's theta_m_save and moist's cqu (edge blocks) too
template <int LP, bool MPASV = false, bool MD = false>
__global__ __launch_bounds__(256) void k_setup_vi(DevState S, int ncb, double dtseps, double rcv, double c2, int copies) {
    setup_vi_body<LP, MPASV, MD>(S, ncb, dtseps, rcv, c2, this_blk(), copies);
}
template <int LP>
static hipError_t setup_vi_lp(const DevState& S, hipStream_t st, double dts, bool edges, int nbc) {
    double dtseps = .5 * dts * (1.0 + kEpssm);
    double rcv = kRgas / (kCp - kRgas);
    double c2 = kCp * rcv;
    const bool md = S.physics == 2;
    const int ncb = col_blocks<LP>(S, KC), neb = (edges || md) ? col_blocks<LP>(S, KE) : 0;
    const int cp = (edges ? 1 : 0) | (nbc ? 2 : 0);
    if (ncb + neb) {
        if (md) k_setup_vi<LP, true, true><<<ncb + neb, 256, 0, st>>>(S, ncb, dtseps, rcv, c2, cp);
        else if (S.physics) k_setup_vi<LP, true, false><<<ncb + neb, 256, 0, st>>>(S, ncb, dtseps, rcv, c2, cp);
        else k_setup_vi<LP><<<ncb + neb, 256, 0, st>>>(S, ncb, dtseps, rcv, c2, cp);
    }
    if (md) HALO_WROTE(S, F_theta_m_save, F_cqu);
    if (edges) HALO_WROTE(S, F_ru_save, F_u_2);
    HALO_WROTE(S, F_rw_save, F_rtheta_p_save, F_rho_p_save, F_w_2, F_theta_m_2, F_rho_zz_2, F_rho_zz_old_split, F_qtot,
               F_cqw);
    HALO_WROTE(S, F_coftz, F_cofwt, F_gamma_tri, F_cofwr, F_cofwz, F_a_tri, F_alpha_tri);
    if (!nbc) HALO_WROTE(S, F_b_tri, F_c_tri);
    return hipGetLastError();
}
hipError_t launch_setup_moist_vert_imp(const DevState& S, hipStream_t st, double dts, bool edges, int nbc) {
    MPAS_LP_DISPATCH(S.LP, setup_vi_lp, S, st, dts, edges, nbc);
}

template <int LP, bool MPASV>
__global__ __launch_bounds__(256) void k_vert_imp(DevState S, double dtseps, double rcv, double c2) {
    vert_imp_body<LP, MPASV>(S, dtseps, rcv, c2, this_blk());
}
template <int LP>
static hipError_t vert_imp_lp(const DevState& S, hipStream_t st, double dts) {
    double dtseps = .5 * dts * (1.0 + kEpssm);
    double rcv = kRgas / (kCp - kRgas);
    double c2 = kCp * rcv;
    const int grid = col_blocks<LP>(S, KC);
    if (grid && S.physics) k_vert_imp<LP, true><<<grid, 256, 0, st>>>(S, dtseps, rcv, c2);
    else if (grid) k_vert_imp<LP, false><<<grid, 256, 0, st>>>(S, dtseps, rcv, c2);
    HALO_WROTE(S, F_coftz, F_cofwt, F_gamma_tri, F_cofwr, F_cofwz, F_a_tri, F_b_tri, F_c_tri, F_alpha_tri);
    return hipGetLastError();
}
hipError_t launch_vert_imp_coefs(const DevState& S, hipStream_t st, double dts) {
    MPAS_LP_DISPATCH(S.LP, vert_imp_lp, S, st, dts);
}

// ---------------------------------------------------------------- set_smlstep
// MD: the MPAS dynamics (physics = 2, ora_mpas_set_smlstep): u_tend is dyn_tend's tend_u
// and w_tend its tend_w (Q2/Q8), levels 1..L-1 of every cell within the relaxation zone
// SUM (reference semantics, fast path): the slope-flux terms summed first, then subtracted from
// w (k_sml_flux's order: the same bits as atm_srk3's fused set_smlstep); else one by one (:1512-1521)
template <int LP, bool MD, bool SUM>
__global__ __launch_bounds__(256) void k_set_smlstep(DevState S) {
    ColMap<LP> m(S, KC);
    const int L = S.L, k = m.k, c = m.ent;
    if (c >= S.nCO) return;
    const size_t p = (size_t)c * LP + lpos(LP, k);
    const int ne = fi(S, F_nEdgesOnCell)[c];
    const int* eoc = fi(S, F_edgesOnCell) + (size_t)c * 10;
    const double* sgn = fd(S, F_edgesOnCell_sign) + (size_t)c * 10;
    const double* ut_f = fd(S, MD ? F_tend_u : F_u_tend);
    const int wf = MD ? F_tend_w : F_w;
    const double* zb = fd(S, F_zb_cell);
    const double* zb3 = fd(S, F_zb3_cell);
    const double fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    double zz, w;
    col_rd2<LP>(fd(S, F_zz), fd(S, wf), c, k, L, zz, w);
    const double w_in = w;  // (MD: levels 0 and L keep the tend_w just loaded)
    // (the point's cprMask byte loaded with the columns: tested after a lane condition it
    // was loaded under a divergent branch and waited for there)
    const uint8_t cpr = MD ? 0 : ((const uint8_t*)S.f[F_cprMask])[p];
    const double zz_m = lvl_dn<LP>(zz, k);
    int e_[NF];
    double ut_[NF], utm_[NF], zb_[NF], zb3_[NF], sgn_[NF];
    row_ld(eoc, e_);
    row_ld(sgn, sgn_);
#pragma unroll
    for (int i = 0; i < NF; i += 2) gather2s<LP>(ut_f, e_[i], e_[i + 1], k, ut_[i], ut_[i + 1]);
#pragma unroll
    for (int i = 0; i < NF; i++) {
        ut_[i] = ldz(k <= L, ut_[i]);
        gather2<LP>(zb, c * 10 + i, zb3, c * 10 + i, k, zb_[i], zb3_[i]);  // (one 16-B load)
    }
#pragma unroll
    for (int i = 0; i < NF; i++) utm_[i] = lvl_dn<LP>(ut_[i], k);
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        double flux = sgn_[i] * (fzm * ut_[i] + fzp * utm_[i]);
        const double t = (zb_[i] + copysign(1.0, ut_[i]) * zb3_[i]) * flux;
        if constexpr (SUM) sum = add_if(i < ne, sum, t);
        else w = sub_if(i < ne, w, t);
    }
    for (int i = NF; i < ne; i++) {
        int iEdge = eoc[i];
        double ut = col_rd<LP>(ut_f, iEdge, k, L);
        double ut_m = lvl_dn<LP>(ut, k);
        double flux = sgn[i] * (fzm * ut + fzp * ut_m);
        size_t q = ((size_t)c * 10 + i) * LP + lpos(LP, k);
        if constexpr (SUM) sum += (zb[q] + copysign(1.0, ut) * zb3[q]) * flux;
        else w -= (zb[q] + copysign(1.0, ut) * zb3[q]) * flux;
    }
    if constexpr (SUM) w = w - sum;
    w *= (fzm * zz + fzp * zz_m);
    if (MD) {  // (every level written: 0 and L with their loaded values, the padding with zeros)
        if (fi(S, F_bdyMaskCell)[c] <= kRelaxZone) colk(fw(S, wf), c) = (k >= 1 && k < L) ? w : PADW(w_in);
    } else if ((k <= L) & (fi(S, F_bdyMaskCell)[c] <= kRelaxZone) & (cpr != 0)) {
        colk(fw(S, wf), c) = w;
        if (k == L) keep_put<LP>(S, F_w, KC, c, w);  // (w's level L changes: its keep tail too)
    } else if ((k > L) & (fi(S, F_bdyMaskCell)[c] <= kRelaxZone)) {
        colk(fw(S, wf), c) = 0.0;  // (the padding's content: the column's last line written whole)
    }
}
template <int LP>
static hipError_t smlstep_lp(const DevState& S, hipStream_t st, int exact) {
    const bool md = S.physics == 2;
    auto run = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (nb && md) k_set_smlstep<LP, true, false><<<nb, 256, 0, st>>>(X);
        else if (nb && !exact) k_set_smlstep<LP, false, true><<<nb, 256, 0, st>>>(X);
        else if (nb) k_set_smlstep<LP, false, false><<<nb, 256, 0, st>>>(X);
    };
    if (md) {
        HALO_RUN(S, st, run, F_tend_u);
        HALO_WROTE(S, F_tend_w);
    } else {
        HALO_RUN(S, st, run, F_u_tend);
        HALO_WROTE(S, F_w);
    }
    return hipGetLastError();
}
hipError_t launch_set_smlstep(const DevState& S, hipStream_t st, int exact) {
    MPAS_LP_DISPATCH(S.LP, smlstep_lp, S, st, exact);
}

// ---------------------------------------------------------------- divergence damping
// (kernel body: k_cols.h divdamp_body)
template <int LP, int EPW, bool OLD0, bool DIVB = false, bool TME = false>
__global__ __launch_bounds__(256) void k_div_damp(DevState S, double coef_divdamp) {
    divdamp_body<LP, EPW, OLD0, DIVB, TME>(S, coef_divdamp, this_blk());
}
double divdamp_coef(double dts) {  // :1736-1738
    double smdiv = kSmdiv;
    double rdts = 1.0 / dts;
    return 2.0 * smdiv * kLenDisp * rdts;
}
template <int LP>
static hipError_t divdamp_div_lp(const DevState& S, hipStream_t st, double dts, int tme) {
    if (S.physics || (tme && S.halo)) return hipErrorInvalidValue;  // (the fused path's; srk3 never asks otherwise)
    const double coef_divdamp = divdamp_coef(dts);
    auto run = [&](const DevState& X) {
        const int nb = col_blocks_n<LP, 2>(X, KE);
        if (nb && tme) k_div_damp<LP, 2, false, true, true><<<nb, 256, 0, st>>>(X, coef_divdamp);
        else if (nb) k_div_damp<LP, 2, false, true><<<nb, 256, 0, st>>>(X, coef_divdamp);
    };
    if (!S.halo) {
        run(S);
        return hipGetLastError();
    }
    // decomposed: div (X_dvB) at the cells of the edges, and the ring-1 redundancy of
    // divdamp_lp (the launch after the exchange also updates the ghost edges of owned cells)
    if (!(S.ring1 && S.nERing >= S.nEO)) return hipErrorInvalidValue;
    auto run1 = [&](const DevState& X) {
        DevState Y = X;
        if (!X.interior) Y.nEO = S.nERing;
        run(Y);
    };
    HALO_RUN(S, st, run1, X_dvB, F_theta_m);
    S.halo->wrote_ring1({F_ru_p});
    return hipGetLastError();
}
hipError_t launch_div_damping_div(const DevState& S, hipStream_t st, double dts, int tme) {
    MPAS_LP_DISPATCH(S.LP, divdamp_div_lp, S, st, dts, tme);
}
template <int LP>
static hipError_t divdamp_lp(const DevState& S, hipStream_t st, double dts, int old_zero) {
    double coef_divdamp = divdamp_coef(dts);
    auto run = [&](const DevState& X) {
#define MPAS_DIVDAMP(EPW)                                                                    \
    do {                                                                                     \
        const int nb = col_blocks_n<LP, EPW>(X, KE);                                         \
        if (nb && old_zero) k_div_damp<LP, EPW, true><<<nb, 256, 0, st>>>(X, coef_divdamp);  \
        else if (nb) k_div_damp<LP, EPW, false><<<nb, 256, 0, st>>>(X, coef_divdamp);        \
    } while (0)
        if (X.epw == 4) MPAS_DIVDAMP(4);
        else if (X.epw == 2) MPAS_DIVDAMP(2);
        else MPAS_DIVDAMP(1);
#undef MPAS_DIVDAMP
    };
    // ring-1 redundancy (reference semantics, where only this task writes ru_p): the launch
    // that may read ghosts (all owned edges, or the boundary ones) also updates the ghost
    // edges of owned cells from the freshly exchanged cell values, exactly as their owners
    // do, so the acoustic step's gathers of ru_p need no exchange (7 per RK3 step fewer)
    const bool r1 = S.halo && S.ring1 && S.nERing >= S.nEO && S.physics == 0;
    auto run1 = [&](const DevState& X) {
        DevState Y = X;
        if (!X.interior) Y.nEO = S.nERing;  // the launch after the exchange (whole or boundary)
        run(Y);
    };
    if (r1) {
        if (old_zero) HALO_RUN(S, st, run1, F_rtheta_pp, F_theta_m);
        else HALO_RUN(S, st, run1, F_rtheta_pp, F_rtheta_pp_old, F_theta_m);
        S.halo->wrote_ring1({F_ru_p});
        return hipGetLastError();
    }
    if (old_zero) HALO_RUN(S, st, run, F_rtheta_pp, F_theta_m);
    else HALO_RUN(S, st, run, F_rtheta_pp, F_rtheta_pp_old, F_theta_m);
    HALO_WROTE(S, F_ru_p);
    return hipGetLastError();
}
hipError_t launch_div_damping(const DevState& S, hipStream_t st, double dts, int old_zero) {
    MPAS_LP_DISPATCH(S.LP, divdamp_lp, S, st, dts, old_zero);
}

// ---------------------------------------------------------------- substep finish
__global__ __launch_bounds__(256) void k_finish_edges(DevState S, int substep, int split, double inv_split) {
    const size_t n = (size_t)S.nEO * S.LP;
    double *ru_save = fw(S, F_ru_save), *u = fw(S, F_u), *ruAvg = fw(S, F_ruAvg), *ruAvgS = fw(S, F_ruAvg_split);
    const double *ru = fd(S, F_ru), *u2 = fd(S, F_u_2);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (plev(S.LP, (int)(i & (size_t)(S.LP - 1))) == S.L) continue;  // (padding copied: zeros, full 64-B sectors)
        if (substep < split) {
            ru_save[i] = ru[i];
            u[i] = u2[i];
        }
        double s = (substep == 1) ? ruAvg[i] : ruAvg[i] + ruAvgS[i];
        ruAvgS[i] = s;
        if (substep == split) ruAvg[i] = s * inv_split;
    }
}
__global__ __launch_bounds__(256) void k_finish_cells(DevState S, int substep, int split, double inv_split) {
    const size_t n = (size_t)S.nCO * S.LP;
    double *wwAvg = fw(S, F_wwAvg), *wwAvgS = fw(S, F_wwAvg_split), *rho_zz = fw(S, F_rho_zz);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (plev(S.LP, (int)(i & (size_t)(S.LP - 1))) == S.L) continue;  // (padding copied: zeros, full 64-B sectors)
        if (substep < split) {
            fw(S, F_rw_save)[i] = fd(S, F_rw)[i];
            fw(S, F_rtheta_p_save)[i] = fd(S, F_rtheta_p)[i];
            fw(S, F_rho_p_save)[i] = fd(S, F_rho_p)[i];
            fw(S, F_w)[i] = fd(S, F_w_2)[i];
            fw(S, F_theta_m)[i] = fd(S, F_theta_m_2)[i];
            rho_zz[i] = fd(S, F_rho_zz_2)[i];
        }
        double s = (substep == 1) ? wwAvg[i] : wwAvg[i] + wwAvgS[i];
        wwAvgS[i] = s;
        if (substep == split) {
            wwAvg[i] = s * inv_split;
            // MPAS-A resets rho_zz of the OLD time level (rho_zz_1); the port has one time
            // level, so the MPAS dynamics (physics = 2) keeps the new rho_zz
            if (S.physics != 2) rho_zz[i] = fd(S, F_rho_zz_old_split)[i];
        }
    }
}
// LP = 64 form of both finish kernels in one launch (blockIdx.y: 0 edges, 1 cells), 16-B
// position pairs.  With substep = split = 1 (atm_srk3) the average is s * 1.0 = s: its
// store back is skipped (the same bits)
__global__ __launch_bounds__(256) void k_finish64(DevState S, int substep, int split, double inv_split, Pair64 q,
                                                  int norz) {
    finish64_body(S, substep, split, inv_split, q, blockIdx.y == 1, (int)blockIdx.x, (int)gridDim.x, norz);
}

hipError_t launch_substep_finish(const DevState& S, hipStream_t st, int substep, int split, int norz) {
    double inv = 1.0 / (double)split;
    if (norz && (S.physics || substep != split || S.LP != 64)) return hipErrorInvalidValue;
    if (S.LP == 64) {
        const int gx = (stream_grid((size_t)S.nEO * 32) + 3) / 4;
        k_finish64<<<dim3(gx, 2), 256, 0, st>>>(S, substep, split, inv, Pair64(S.L), norz);
    } else {
        k_finish_edges<<<stream_grid((size_t)S.nEO * S.LP), 256, 0, st>>>(S, substep, split, inv);
        k_finish_cells<<<stream_grid((size_t)S.nCO * S.LP), 256, 0, st>>>(S, substep, split, inv);
    }
    // what the kernels write for these arguments (a field declared written but untouched
    // would cost every later gather of it a halo exchange): with substep = split = 1, as
    // atm_srk3 calls it, only the averages and (physics != 2) rho_zz
    if (substep < split)
        HALO_WROTE(S, F_ru_save, F_u, F_rw_save, F_rtheta_p_save, F_rho_p_save, F_w, F_theta_m, F_rho_zz);
    HALO_WROTE(S, F_ruAvg, F_ruAvg_split, F_wwAvg, F_wwAvg_split);
    if (substep == split && S.physics != 2 && !norz) HALO_WROTE(S, F_rho_zz);
    return hipGetLastError();
}

// ---------------------------------------------------------------- derived mesh arrays
__global__ __launch_bounds__(256) void k_prepare(DevState S, int* selfc) {
    const size_t n = (size_t)S.nCells * 10;
    const int* eoc = fi(S, F_edgesOnCell);
    const int* coe = fi(S, F_cellsOnEdge);
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < (size_t)S.nVertices * 3; t += (size_t)gridDim.x * 256)
        fw(S, X_ve_dc)[t] = fd(S, F_dcEdge)[fi(S, F_edgesOnVertex)[t]];
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < (size_t)S.nEdges * 24; t += (size_t)gridDim.x * 256) {
        const size_t e = t / 24;
        const int j = (int)(t % 24);
        int v = 0;
        if (j < 2) v = coe[e * 2 + j];
        else if (j < 12) v = fi(S, F_edgesOnEdge)[e * 20 + (j - 2)];
        else if (j < 21) v = fi(S, F_advCellsForEdge)[e * 15 + (j - 12)];
        else if (j == 21) v = fi(S, F_nEdgesOnEdge)[e];
        else if (j == 22) v = fi(S, F_nAdvCellsForEdge)[e];
        ((int*)S.f[X_eB])[t] = v;
    }
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < (size_t)S.nEO * 20; t += (size_t)gridDim.x * 256)
        if (fi(S, F_edgesOnEdge)[t] != fi(S, F_edgesOnEdge_ECP)[t]) atomicAnd(selfc + 2, 0);
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (size_t)gridDim.x * 256) {
        const int e = eoc[t], c = (int)(t / 10), i = (int)(t % 10);
        const int c1 = coe[(size_t)e * 2], c2 = coe[(size_t)e * 2 + 1];
        ((int*)S.f[X_ce_c1])[t] = c1;
        ((int*)S.f[X_ce_c2])[t] = c2;
        ((int*)S.f[X_ce_oth])[t] = (c1 == c) ? c2 : c1;
        ((int*)S.f[X_ce_s1])[t] = (c1 == c) ? 1 : 0;
        if (c < S.nCO && i < fi(S, F_nEdgesOnCell)[c] && i < NF && c1 != c && c2 != c) atomicAnd(selfc, 0);
        if (i < NF) {
            int* r = (int*)S.f[X_cR] + (size_t)c * CREC;
            int* rs = (int*)S.f[X_cRs] + (size_t)c * CREC;
            r[i] = rs[i] = e;
            r[NF + i] = c1;
            r[2 * NF + i] = c2;
            rs[NF + i] = (c1 == c) ? c2 : c1;
            rs[2 * NF + i] = (c1 == c) ? 1 : 0;
            if (i == 0) {
                r[3 * NF] = rs[3 * NF] = fi(S, F_nEdgesOnCell)[c];
                r[3 * NF + 1] = rs[3 * NF + 1] = 0;
            }
        }
        fw(S, X_ce_dv)[t] = fd(S, F_dvEdge)[e];
        fw(S, X_ce_dc)[t] = fd(S, F_dcEdge)[e];
        fw(S, X_ce_idc)[t] = fd(S, F_invDcEdge)[e];
        fw(S, X_ce_msd2)[t] = fd(S, F_meshScalingDel2)[e];
        fw(S, X_ce_msd4)[t] = fd(S, F_meshScalingDel4)[e];
        if (i == 0) {  // X_wfl (k_dyn_A): the literal flux_arr of :1174-1205 on the zeroed w
            const int ne = fi(S, F_nEdgesOnCell)[c];
            const int el = ne > 0 ? eoc[t + ne - 1] : S.nEdges;
            const int na = fi(S, F_nAdvCellsForEdge)[el];
            const double* ac = fd(S, F_adv_coefs) + (size_t)el * 15;
            const double* ac3 = fd(S, F_adv_coefs_3rd) + (size_t)el * 15;
            for (int q = 0; q < 2; q++) {
                const double sg = q == 0 ? 1.0 : -1.0, w_zeroed = 0.0;
                double flux_arr = 0.0;
                for (int j = 0; j < na; j++) {
                    double scalar_weight = ac[j] + sg * ac3[j];
                    flux_arr += scalar_weight * w_zeroed;
                }
                fw(S, X_wfl)[(size_t)c * 2 + q] = flux_arr;
            }
        }
    }
}
// edge ownership of the deferred damping (k_acoustic MODE 2): the lowest cell * 16 + slot
// listing each edge (slots < nEdgesOnCell, owned cells), the owning slots per cell as a
// bit mask, and the edges no cell lists; the div buffers' zero-slot rows hold the div the
// damping computes there, -(0.0 - 0.0) = -0.0
__global__ __launch_bounds__(256) void k_own_init(DevState S) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t <= (size_t)S.nEdges; t += stride)
        ((int*)S.f[X_eowner])[t] = 0x7fffffff;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t <= (size_t)S.nCells; t += stride)
        ((int*)S.f[X_eown])[t] = 0;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < (size_t)S.LP; t += stride) {
        fw(S, X_dvA)[(size_t)S.nCells * S.LP + t] = -0.0;
        fw(S, X_dvB)[(size_t)S.nCells * S.LP + t] = -0.0;
    }
}
__global__ __launch_bounds__(256) void k_own_min(DevState S) {
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < (size_t)S.nCO * 10; t += (size_t)gridDim.x * 256) {
        const int c = (int)(t / 10), i = (int)(t % 10), e = fi(S, F_edgesOnCell)[t];
        if (i < fi(S, F_nEdgesOnCell)[c] && e >= 0 && e < S.nEdges) atomicMin((int*)S.f[X_eowner] + e, c * 16 + i);
    }
}
__global__ __launch_bounds__(256) void k_own_bits(DevState S, int* norph) {
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < (size_t)S.nCO * 10; t += (size_t)gridDim.x * 256) {
        const int c = (int)(t / 10), i = (int)(t % 10), e = fi(S, F_edgesOnCell)[t];
        if (i < fi(S, F_nEdgesOnCell)[c] && e >= 0 && e < S.nEdges && fi(S, X_eowner)[e] == c * 16 + i)
            atomicOr((int*)S.f[X_eown] + c, 1 << i);
    }
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < (size_t)S.nEO; t += (size_t)gridDim.x * 256)
        if (fi(S, X_eowner)[t] == 0x7fffffff) ((int*)S.f[X_orph])[atomicAdd(norph, 1)] = (int)t;
}

// derived mesh arrays; decides S.selfc (synchronous: runs once after each mesh upload)
hipError_t launch_prepare(DevState& S, hipStream_t st) {
    int* flag = nullptr;  // [0] selfc, [1] orphan edges, [2] eoe_same
    hipError_t e = hipMalloc(&flag, 3 * sizeof(int));
    if (e != hipSuccess) return e;
    const int init[3] = {1, 0, 1};
    int host[3] = {0, 0, 0};
    e = hipMemcpyAsync(flag, init, sizeof(init), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        k_prepare<<<stream_grid((size_t)S.nCells * 10), 256, 0, st>>>(S, flag);
        const int g = stream_grid((size_t)S.nCells * 10 > (size_t)S.nEdges ? (size_t)S.nCells * 10 : (size_t)S.nEdges + 1);
        k_own_init<<<g, 256, 0, st>>>(S);
        k_own_min<<<g, 256, 0, st>>>(S);
        k_own_bits<<<g, 256, 0, st>>>(S, flag + 1);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(host, flag, sizeof(host), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(flag);
    if (e == hipSuccess) {
        S.selfc = host[0];
        S.n_orph = host[1];
        S.eoe_same = host[2];
    }
    return e;
}

// ---------------------------------------------------------------- synthetic fill
__global__ __launch_bounds__(256) void k_fill(void* dst, int fid, int kind, long n, int W, int levels, int LP,
                                              int dist, double lo, double hi, uint64_t seed, const int* gid) {
    double* d = (double*)dst;
    const size_t total = (size_t)n * W * levels;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (size_t)gridDim.x * 256) {
        int k = (int)(t % levels);
        size_t r = t / levels;
        int i = (int)(r % W);
        long e = (long)(r / W);
        const long g = gid ? (long)gid[e] : e;  // the global entity id: same value on every rank
        double v = mpas_synth_value(seed, (uint32_t)fid, (uint64_t)g, (uint32_t)k, (uint32_t)i, dist, lo, hi);
        if (kind == K_ZV) d[k] = v;
        else if (kind == K_C3V) d[vidx(W, LP, e, i, k)] = v;
        else d[(size_t)e * LP + lpos(LP, k)] = v;
    }
}
hipError_t launch_fill_synthetic(const DevState& S, hipStream_t st, uint64_t seed) {
    for (int f = 0; f < F_COUNT; f++) {
        const FieldInfo& fi_ = kFields[f];
        if (fi_.dist == D_M) continue;
        long n = 0;
        int W = 1;
        const int* gid = nullptr;
        switch (fi_.kind) {
            case K_C3: n = S.nCells; gid = S.gid[0]; break;
            case K_E3: n = S.nEdges; gid = S.gid[1]; break;
            case K_V3: n = S.nVertices; gid = S.gid[2]; break;
            case K_C3V: n = S.nCells; W = fi_.width; gid = S.gid[0]; break;
            case K_ZV: n = 1; break;
            default: continue;
        }
        size_t total = (size_t)n * W * (S.L + 1);
        k_fill<<<stream_grid(total), 256, 0, st>>>(S.f[f], f, fi_.kind, n, W, S.L + 1, S.LP, fi_.dist, fi_.lo, fi_.hi, seed,
                                                   gid);
    }
    return hipGetLastError();
}

}  // namespace mpas

namespace mpas {
// ---------------------------------------------------------------- device-resident views
// mpas_upload / mpas_download of a 3-D field from / to a strided view in device memory
// (a Legion instance in framebuffer memory, a torch tensor): element (entity e, level k,
// component i) at byte offset e*se + k*sl + i*sc of the view, to / from the LP-padded
// column layout; one thread per element, the levels of a column on consecutive threads.
// Only levels 0..L of entities 0..n-1 move (padding and the zero slot keep their zeros).
template <class T>
__global__ __launch_bounds__(256) void k_view_copy(T* dev, char* view, int n, int W, int L, int LP, int64_t se,
                                                  int64_t sl, int64_t sc, int to_dev) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t per = (size_t)W * (L + 1);
    if (t >= (size_t)n * per) return;
    const int e = (int)(t / per), r = (int)(t % per), i = r / (L + 1), k = r % (L + 1);
    T* d = dev + vidx(W, LP, e, i, k);
    T* v = (T*)(view + (int64_t)e * se + (int64_t)k * sl + (int64_t)i * sc);
    if (to_dev) *d = *v;
    else *v = *d;
}
hipError_t launch_view_copy(void* dev, void* view, int elem, int n, int W, int L, int LP, int64_t se, int64_t sl,
                            int64_t sc, int to_dev, hipStream_t st) {
    const size_t total = (size_t)n * W * (L + 1);
    if (!total) return hipSuccess;
    const int nb = (int)((total + 255) / 256);
    if (elem == 8) k_view_copy<double><<<nb, 256, 0, st>>>((double*)dev, (char*)view, n, W, L, LP, se, sl, sc, to_dev);
    else k_view_copy<uint8_t><<<nb, 256, 0, st>>>((uint8_t*)dev, (char*)view, n, W, L, LP, se, sl, sc, to_dev);
    return hipGetLastError();
}
#if MPAS_BOUNDS
// bounds-checked build: read field u `col` columns past its last row (the zero slot) --
// the check must report it (tests/test_gpu_bounds.py)
template <int LP>
__global__ __launch_bounds__(256) void k_bounds_probe(DevState S, int col) {
    const int k = (int)(threadIdx.x % LP);
    const double x = colk(fd(S, F_u), S.nEdges + col);
    if (x == 12345.678) colk(fw(S, F_tend_u), 0) = x;  // (keeps the load)
}
template <int LP>
static hipError_t bounds_probe_lp(const DevState& S, hipStream_t st, int col) {
    k_bounds_probe<LP><<<1, LP, 0, st>>>(S, col);
    return hipGetLastError();
}
hipError_t launch_bounds_probe(const DevState& S, hipStream_t st, int col) {
    MPAS_LP_DISPATCH(S.LP, bounds_probe_lp, S, st, col);
}
#endif

// ---------------------------------------------------------------- keep tails (mpas_dev.h)
// (plain arguments -- the column base, n, no: a runtime field id / kind into DevState made the
// compiler index a scratch copy of the struct and select n from it, and that select came out
// wrong for the third kind, ROCm 7.2 hipcc -O3: vertex tails were read at the cell offset)
template <int LP>
__global__ __launch_bounds__(256) void k_keep_refresh(double* f, int n, int L) {
    const int i = (int)(blockIdx.x * 256 + threadIdx.x);
    if (i > n) return;
    const double* col = f + (size_t)i * LP;
    double* t = f + (size_t)(n + 1) * LP;
    t[i] = col[lpos(LP, L)];
    t[(size_t)n + 1 + i] = col[lpos(LP, 0)];
}
template <int LP>
__global__ __launch_bounds__(256) void k_keep_check(const double* f, int n, int no, int L, int fid, int lev0, int* flag) {
    const int i = (int)(blockIdx.x * 256 + threadIdx.x);
    if (i >= no) return;
    const double a = f[(size_t)i * LP + lpos(LP, lev0 ? 0 : L)];
    const double b = f[(size_t)(n + 1) * LP + (lev0 ? (size_t)n + 1 : 0) + i];
    if (__builtin_bit_cast(uint64_t, a) != __builtin_bit_cast(uint64_t, b)) {
        atomicAdd(flag + 6, 1);
        atomicMin(flag + 7, i);
        if (atomicCAS(flag, 0, 2 * fid + lev0 + 1) == 0) {
            flag[1] = i;  // (the first mismatch found: entity and both values, for the message)
            ((double*)(flag + 2))[0] = a;
            ((double*)(flag + 2))[1] = b;
        }
    }
}
static inline int keep_n(const DevState& S, int kind) { return kind == KC ? S.nCells : kind == KE ? S.nEdges : S.nVertices; }
template <int LP>
static hipError_t keep_refresh_lp(const DevState& S, hipStream_t st, int f, int kind) {
    const int n = keep_n(S, kind);
    k_keep_refresh<LP><<<(n + 256) / 256, 256, 0, st>>>((double*)S.f[f], n, S.L);
    return hipGetLastError();
}
hipError_t launch_keep_refresh(const DevState& S, hipStream_t st, int f, int kind) {
    MPAS_LP_DISPATCH(S.LP, keep_refresh_lp, S, st, f, kind);
}
template <int LP>
static hipError_t keep_check_lp(const DevState& S, hipStream_t st, int f, int kind, int lev0, int* flag) {
    const int no = kind == KC ? S.nCO : kind == KE ? S.nEO : S.nVO;
    if (no > 0)
        k_keep_check<LP><<<(no + 255) / 256, 256, 0, st>>>((const double*)S.f[f], keep_n(S, kind), no, S.L, f, lev0, flag);
    return hipGetLastError();
}
hipError_t launch_keep_check(const DevState& S, hipStream_t st, int f, int kind, int lev0, int* flag) {
    MPAS_LP_DISPATCH(S.LP, keep_check_lp, S, st, f, kind, lev0, flag);
}

}  // namespace mpas
