// k_transport.hip -- monotonic scalar transport for gfx950.
//
// The reference has no scalar transport: it declares scalars:double[8] per cell point
// (data_structures.rg:36; nScalars = 8, constants.rg:42) and never touches it.  This is
// the flux-corrected transport MPAS-A runs in its last RK stage (atm_advance_scalars_mono
// of MPAS-Model mpas_atm_time_integration.F; Zalesak 1979, Skamarock & Gassmann 2011),
// statement for statement as oracle/mpas_oracle.c ora_mpas_advance_scalars_mono states it
// (parity unpinned; pinned by its properties in tests/test_transport.py).  mpas mode only.
//
// Three launches, separated where the data flow needs a grid-wide barrier:
//   k_tr_edge    per edge: the antidiffusive flux A = high-order - upwind flux of each
//                scalar and level (X_Ah, E3 x 8)
//   k_tr_bounds  per cell: the upwind update su, the bounds of the old values around the
//                cell, and R+ / R- (X_su, X_Rp, X_Rm, C3V x 8)
//   k_tr_update  per cell: every A scaled by min(R- of its source, R+ of its receiver),
//                s_new = su - dt div(scaled A) / rho_new  (scalars)
// Column slot = (entity, scalar): the 8 scalars of an entity are 8 consecutive columns,
// so the 8 wavefronts of an entity read the same connectivity, mass fluxes and densities
// (one HBM fetch, then L2 hits).  One wavefront per column at 57 levels (LP = 64); the
// vertical neighbours are lane shuffles.
#include "mpas_dev.h"
#include "mpas_halo.h"

namespace mpas {

constexpr int NSC = 8;            // nScalars (constants.rg:42)
constexpr double kCoef3 = 0.25;   // config_coef_3rd_order

__device__ __forceinline__ double tr_flux3(double q_im2, double q_im1, double q_i, double q_ip1, double ua) {
    const double f4 = ua * (7. * (q_i + q_im1) - (q_ip1 + q_im2)) / 12.0;
    return f4 + kCoef3 * fabs(ua) * ((q_ip1 - q_im2) - 3. * (q_i - q_im1)) / 12.0;
}

// entity and scalar of this lane's column slot
template <int LP>
__device__ __forceinline__ void tr_slot(const DevState& S, int kind, int& ent, int& isc) {
    const int slot = col_of<LP>(xcd_block(S.xcd));
    ent = (slot >> 3) + S.lo[kind];
    isc = slot & (NSC - 1);
}

// level k of the column of scalar isc of entity ent in a x8 field (64-bit offsets: the
// edge scratch exceeds 4 GiB on the largest meshes)
template <int LP>
__device__ __forceinline__ size_t tr_at(int ent, int isc, int k) {
    return ((size_t)ent * NSC + isc) * LP + lpos(LP, k);
}

// interface k of a column: upwind (lo) and antidiffusive (A) vertical flux of the lane's
// level; no flux through interfaces 0 and L
template <int LP>
__device__ __forceinline__ void tr_vflux(double s, double w, int k, int L, double fzm, double fzp, double& lo,
                                         double& A) {
    const double sm1 = lvl_dn<LP>(s, k), sm2 = lvl_dn2<LP>(s, k), sp1 = lvl_up<LP>(s, k);
    const double hi = (k >= 2 && k <= L - 2) ? tr_flux3(sm2, sm1, s, sp1, w) : w * (fzm * s + fzp * sm1);
    const double l = fmax(w, 0.0) * sm1 + fmin(w, 0.0) * s;
    const bool in = k >= 1 && k <= L - 1;
    lo = in ? l : 0.0;
    A = in ? hi - l : 0.0;
}

template <int LP>
__global__ __launch_bounds__(256) void k_tr_edge(DevState S) {
    int e, isc;
    tr_slot<LP>(S, KE, e, isc);
    const int L = S.L, k = (int)(threadIdx.x % LP);
    if (e >= S.nEO) return;
    const int* rec = fi(S, X_eB) + (size_t)e * 24;  // cellsOnEdge(2) .. advCellsForEdge(9) @12, nAdv @22
    const int c1 = rec[0], c2 = rec[1], na = rec[22];
    int adv[AF];
    double ac[AF], ac3[AF];
#pragma unroll
    for (int j = 0; j < AF; j++) adv[j] = rec[12 + j];
    row_ld(fd(S, F_adv_coefs) + (size_t)e * 15, ac);
    row_ld(fd(S, F_adv_coefs_3rd) + (size_t)e * 15, ac3);
    const double dv = fd(S, F_dvEdge)[e];
    const double* so = fd(S, F_scalars_old);
    const double u = colk(fd(S, F_ruAvg), e);
    double x[AF];
#pragma unroll
    for (int j = 0; j < AF; j++) x[j] = colk(so, adv[j] * NSC + isc);
    const double s1 = colk(so, c1 * NSC + isc), s2 = colk(so, c2 * NSC + isc);
    const double sgn = copysign(1.0, u);
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < AF; j++) acc = add_if(j < na, acc, (ac[j] + sgn * ac3[j]) * x[j]);
    for (int j = AF; j < na; j++) {  // lists longer than the reference's 9 (width 15)
        const int cj = fi(S, F_advCellsForEdge)[(size_t)e * 15 + j];
        const double wgt = fd(S, F_adv_coefs)[(size_t)e * 15 + j] + sgn * fd(S, F_adv_coefs_3rd)[(size_t)e * 15 + j];
        acc = acc + wgt * colk(so, cj * NSC + isc);
    }
    const double lo = dv * (fmax(u, 0.0) * s1 + fmin(u, 0.0) * s2);
    if (k != L) fw(S, X_Ah)[tr_at<LP>(e, isc, k)] = PADW(u * acc - lo);
}

// the first NF edge slots of a cell: edge, cells of the edge, "cell is cellsOnEdge(0)",
// the other cell, dvEdge (the per-cell copies of k_prepare)
struct TrSlots {
    int e[NF], c1[NF], c2[NF], oth[NF], s1[NF];
    double dv[NF];
};
__device__ __forceinline__ void tr_slots(const DevState& S, int c, TrSlots& t) {
    const size_t r = (size_t)c * 10;
    row_ld(fi(S, F_edgesOnCell) + r, t.e);
    row_ld(fi(S, X_ce_c1) + r, t.c1);
    row_ld(fi(S, X_ce_c2) + r, t.c2);
    row_ld(fi(S, X_ce_oth) + r, t.oth);
    row_ld(fi(S, X_ce_s1) + r, t.s1);
    row_ld(fd(S, X_ce_dv) + r, t.dv);
}

// one edge slot of k_tr_bounds: the upwind flux's contribution, the antidiffusive in/out
// sums and the other cell's value in the bounds
template <int LP>
__device__ __forceinline__ void tr_bound_slot(bool on, int s1f, double dv, double u, double x1, double x2, double A,
                                              double& hlo, double& pin, double& pout, double& smax, double& smin) {
    const double sg = s1f ? 1.0 : -1.0;
    const double lo = dv * (fmax(u, 0.0) * x1 + fmin(u, 0.0) * x2);
    hlo = add_if(on, hlo, sg * lo);
    const double a = -sg * A;
    pin = add_if(on, pin, fmax(a, 0.0));
    pout = sub_if(on, pout, fmin(a, 0.0));
    const double xo = s1f ? x2 : x1;
    smax = on ? fmax(smax, xo) : smax;
    smin = on ? fmin(smin, xo) : smin;
}

template <int LP, bool SELF>
__global__ __launch_bounds__(256) void k_tr_bounds(DevState S, double dt) {
    int c, isc;
    tr_slot<LP>(S, KC, c, isc);
    const int L = S.L, k = (int)(threadIdx.x % LP);
    if (c >= S.nCO) return;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    TrSlots t;
    tr_slots(S, c, t);
    const double invA = fd(S, F_invAreaCell)[c];
    const double rdzw = fd(S, F_rdzw)[k], fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double *so = fd(S, F_scalars_old), *ru = fd(S, F_ruAvg);
    const double* Ah = fd(S, X_Ah);
    const double s = colk(so, c * NSC + isc);
    const double w = colk(fd(S, F_wwAvg), c), r_o = colk(fd(S, F_rho_zz_old_split), c), r_n = colk(fd(S, F_rho_zz), c);
    double u_[NF], x1_[NF], x2_[NF], A_[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        u_[i] = colk(ru, t.e[i]);
        A_[i] = Ah[tr_at<LP>(t.e[i], isc, k)];
        if constexpr (SELF) {
            const double xo = colk(so, t.oth[i] * NSC + isc);
            x1_[i] = t.s1[i] ? s : xo;
            x2_[i] = t.s1[i] ? xo : s;
        } else {
            x1_[i] = colk(so, t.c1[i] * NSC + isc);
            x2_[i] = colk(so, t.c2[i] * NSC + isc);
        }
    }
    double hlo = 0.0, pin = 0.0, pout = 0.0, smax = s, smin = s;
#pragma unroll
    for (int i = 0; i < NF; i++)
        tr_bound_slot<LP>(i < ne, t.s1[i], t.dv[i], u_[i], x1_[i], x2_[i], A_[i], hlo, pin, pout, smax, smin);
    for (int i = NF; i < ne; i++) {  // cells with more than NF edges
        const size_t r = (size_t)c * 10 + i;
        const int e = fi(S, F_edgesOnCell)[r], c1 = fi(S, X_ce_c1)[r], c2 = fi(S, X_ce_c2)[r];
        tr_bound_slot<LP>(true, fi(S, X_ce_s1)[r], fd(S, X_ce_dv)[r], colk(ru, e), colk(so, c1 * NSC + isc),
                          colk(so, c2 * NSC + isc), Ah[tr_at<LP>(e, isc, k)], hlo, pin, pout, smax, smin);
    }
    const double sm1 = lvl_dn<LP>(s, k), sp1 = lvl_up<LP>(s, k);
    smax = k > 0 ? fmax(smax, sm1) : smax;
    smin = k > 0 ? fmin(smin, sm1) : smin;
    smax = k < L - 1 ? fmax(smax, sp1) : smax;
    smin = k < L - 1 ? fmin(smin, sp1) : smin;
    double lob, Ab;
    tr_vflux<LP>(s, w, k, L, fzm, fzp, lob, Ab);
    const double lot = lvl_up<LP>(lob, k), At = lvl_up<LP>(Ab, k);
    const double su = (s * r_o - dt * (hlo * invA + (lot - lob) * rdzw)) / r_n;
    smax = fmax(smax, su);
    smin = fmin(smin, su);
    const double pin_t = dt * (pin * invA + (fmax(Ab, 0.0) - fmin(At, 0.0)) * rdzw);
    const double pout_t = dt * (pout * invA + (fmax(At, 0.0) - fmin(Ab, 0.0)) * rdzw);
    const double qin = (smax - su) * r_n, qout = (su - smin) * r_n;
    const double Rp = pin_t > 0.0 ? fmin(1.0, qin / pin_t) : 0.0;
    const double Rm = pout_t > 0.0 ? fmin(1.0, qout / pout_t) : 0.0;
    if (k < L || k > L) {
        const size_t o = tr_at<LP>(c, isc, k);
        fw(S, X_Rp)[o] = PADW(Rp);
        fw(S, X_Rm)[o] = PADW(Rm);
        fw(S, X_su)[o] = PADW(su);
    }
}

template <int LP>
__global__ __launch_bounds__(256) void k_tr_update(DevState S, double dt) {
    int c, isc;
    tr_slot<LP>(S, KC, c, isc);
    const int L = S.L, k = (int)(threadIdx.x % LP);
    if (c >= S.nCO) return;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    TrSlots t;
    tr_slots(S, c, t);
    const double invA = fd(S, F_invAreaCell)[c];
    const double rdzw = fd(S, F_rdzw)[k], fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double *Ah = fd(S, X_Ah), *Rp = fd(S, X_Rp), *Rm = fd(S, X_Rm);
    const size_t o = tr_at<LP>(c, isc, k);
    const double s = colk(fd(S, F_scalars_old), c * NSC + isc);
    const double w = colk(fd(S, F_wwAvg), c), r_n = colk(fd(S, F_rho_zz), c);
    const double su = fd(S, X_su)[o], rp = Rp[o], rm = Rm[o];
    double A_[NF], p1_[NF], m1_[NF], p2_[NF], m2_[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        A_[i] = Ah[tr_at<LP>(t.e[i], isc, k)];
        p1_[i] = Rp[tr_at<LP>(t.c1[i], isc, k)];
        m1_[i] = Rm[tr_at<LP>(t.c1[i], isc, k)];
        p2_[i] = Rp[tr_at<LP>(t.c2[i], isc, k)];
        m2_[i] = Rm[tr_at<LP>(t.c2[i], isc, k)];
    }
    double hc = 0.0;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        const double sg = t.s1[i] ? 1.0 : -1.0;
        const double C = A_[i] >= 0.0 ? fmin(m1_[i], p2_[i]) : fmin(p1_[i], m2_[i]);
        hc = add_if(i < ne, hc, sg * (C * A_[i]));
    }
    for (int i = NF; i < ne; i++) {
        const size_t r = (size_t)c * 10 + i;
        const int e = fi(S, F_edgesOnCell)[r], c1 = fi(S, X_ce_c1)[r], c2 = fi(S, X_ce_c2)[r];
        const double sg = fi(S, X_ce_s1)[r] ? 1.0 : -1.0;
        const double A = Ah[tr_at<LP>(e, isc, k)];
        const double C = A >= 0.0 ? fmin(Rm[tr_at<LP>(c1, isc, k)], Rp[tr_at<LP>(c2, isc, k)])
                                  : fmin(Rp[tr_at<LP>(c1, isc, k)], Rm[tr_at<LP>(c2, isc, k)]);
        hc = hc + sg * (C * A);
    }
    double lo, A;
    tr_vflux<LP>(s, w, k, L, fzm, fzp, lo, A);
    const double rp_b = lvl_dn<LP>(rp, k), rm_b = lvl_dn<LP>(rm, k);
    const double fcb = (k >= 1 && k <= L - 1) ? (A >= 0.0 ? fmin(rm_b, rp) : fmin(rp_b, rm)) * A : 0.0;
    const double fct = lvl_up<LP>(fcb, k);
    const double sn = su - dt * (hc * invA + (fct - fcb) * rdzw) / r_n;
    if (k < L) colk(fw(S, F_scalars), c * NSC + isc) = sn;
}

template <int LP>
static hipError_t transport_lp(const DevState& S, hipStream_t st, double dt) {
    constexpr int COLS = 256 / LP;
    const long ne = (long)(S.nEO - S.lo[KE]) * NSC, nc = (long)(S.nCO - S.lo[KC]) * NSC;
    const int nEB = (int)((ne + COLS - 1) / COLS), nCB = (int)((nc + COLS - 1) / COLS);
    if (nEB > 0) k_tr_edge<LP><<<nEB, 256, 0, st>>>(S);
    if (nCB > 0) {
        if (S.selfc) k_tr_bounds<LP, true><<<nCB, 256, 0, st>>>(S, dt);
        else k_tr_bounds<LP, false><<<nCB, 256, 0, st>>>(S, dt);
        k_tr_update<LP><<<nCB, 256, 0, st>>>(S, dt);
    }
    return hipGetLastError();
}
hipError_t launch_advance_scalars_mono(const DevState& S, hipStream_t st, double dt) {
    if (S.halo) return hipErrorNotSupported;  // single subdomain only
    MPAS_LP_DISPATCH(S.LP, transport_lp, S, st, dt);
}

}  // namespace mpas
