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
// Column slot = (entity, scalar pair): the 8 scalars of an entity are 8 consecutive
// columns; a wavefront computes two of them (one 16-B lane load fetches a gathered column
// pair: the gathers cost per load instruction), and the 4 wavefronts of an
// entity read the same connectivity, mass fluxes and densities (one HBM fetch, then L2
// hits).  One wavefront per column pair at 57 levels (LP = 64); the vertical neighbours
// are lane shuffles.
#include "mpas_dev.h"
#include "mpas_halo.h"

namespace mpas {

constexpr int NSC = 8;            // nScalars (constants.rg:42)
constexpr double kCoef3 = 0.25;   // config_coef_3rd_order

__device__ __forceinline__ double tr_flux3(double q_im2, double q_im1, double q_i, double q_ip1, double ua) {
    const double f4 = ua * (7. * (q_i + q_im1) - (q_ip1 + q_im2)) / 12.0;
    return f4 + kCoef3 * fabs(ua) * ((q_ip1 - q_im2) - 3. * (q_i - q_im1)) / 12.0;
}

// entity and scalar pair of this lane's column slot: a wavefront computes two scalars,
// 2p and 2p+1, of one entity (their columns are adjacent, so one 16-B lane load fetches
// both: ld2 below)
// Slot order (option "trorder"): 0 entity-major (the 4 pairs of an entity in adjacent
// slots: they share its connectivity and mass-flux loads), 1 pair-major (all entities for
// pair 0, then pair 1, ...: a quarter of the per-entity footprint in L2, so the entities
// in flight span 4x the mesh and share more neighbour columns)
template <int LP>
__device__ __forceinline__ void tr_slot(const DevState& S, int kind, int& ent, int& p) {
    const int slot = col_of<LP>(xcd_block(S.xcd));
    if (S.tro) {
        const int n = (kind == KC ? S.nCO : S.nEO) - S.lo[kind];
        const int q = slot / n;
        ent = slot - q * n + S.lo[kind];
        p = q * 2;
        if (q >= NSC / 2) ent = 0x7fffffff;  // past the grid's last slot (caller returns)
    } else {
        ent = (slot >> 2) + S.lo[kind];
        p = (slot & 3) * 2;
    }
}

// level k of columns ia and ib of field f (64-bit column ids: the edge scratch exceeds
// 4 GiB on the largest meshes).  At LP = 64 one 16-B load per lane (lanes 0-31 the level
// pair k & 31 of column ia, lanes 32-63 that of column ib, the lpos layout) and a
// permlane32 swap (gather2 of mpas_dev.h); two loads below LP 64.
template <int LP>
__device__ __forceinline__ void ld2(const double* f, size_t ia, size_t ib, int k, double& a, double& b) {
    if constexpr (LP == 64) {
        const double2 t = *(const double2*)((const char*)f + (k >= 32 ? ib : ia) * 512 + (size_t)(k & 31) * 16);
        double x = t.x, y = t.y;
        swap_halves(x, y);
        a = x;
        b = y;
    } else {
        a = f[ia * LP + lpos(LP, k)];
        b = f[ib * LP + lpos(LP, k)];
    }
}
// the inverse: store a (column ia) and b (column ib) at every level of the lane; at
// LP = 64 one 16-B store per lane (every lane of the wavefront must take part)
template <int LP>
__device__ __forceinline__ void st2(double* f, size_t ia, size_t ib, int k, double a, double b) {
    if constexpr (LP == 64) {
        swap_halves(a, b);
        *(double2*)((char*)f + (k >= 32 ? ib : ia) * 512 + (size_t)(k & 31) * 16) = make_double2(a, b);
    } else {
        f[ia * LP + lpos(LP, k)] = a;
        f[ib * LP + lpos(LP, k)] = b;
    }
}
__device__ __forceinline__ size_t col8(int ent, int i) { return (size_t)ent * NSC + i; }

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
    int e, p;
    tr_slot<LP>(S, KE, e, p);
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
    double xa[AF], xb[AF], s1a, s1b, s2a, s2b;
#pragma unroll
    for (int j = 0; j < AF; j++) ld2<LP>(so, col8(adv[j], p), col8(adv[j], p + 1), k, xa[j], xb[j]);
    // the upwind flux's two cells are normally advCellsForEdge(0) and (1) (MPAS's list
    // construction): take their columns from the list; gather them only where they are not
    // (wave-uniform branch, the same column either way)
    if (na >= 2 && adv[0] == c1 && adv[1] == c2) {
        s1a = xa[0], s1b = xb[0], s2a = xa[1], s2b = xb[1];
    } else {
        ld2<LP>(so, col8(c1, p), col8(c1, p + 1), k, s1a, s1b);
        ld2<LP>(so, col8(c2, p), col8(c2, p + 1), k, s2a, s2b);
    }
    const double sgn = copysign(1.0, u);
    double acca = 0.0, accb = 0.0;
#pragma unroll
    for (int j = 0; j < AF; j++) {
        const double wgt = ac[j] + sgn * ac3[j];
        acca = add_if(j < na, acca, wgt * xa[j]);
        accb = add_if(j < na, accb, wgt * xb[j]);
    }
    for (int j = AF; j < na; j++) {  // lists longer than the reference's 9 (width 15)
        const int cj = fi(S, F_advCellsForEdge)[(size_t)e * 15 + j];
        const double wgt = fd(S, F_adv_coefs)[(size_t)e * 15 + j] + sgn * fd(S, F_adv_coefs_3rd)[(size_t)e * 15 + j];
        double ya, yb;
        ld2<LP>(so, col8(cj, p), col8(cj, p + 1), k, ya, yb);
        acca = acca + wgt * ya;
        accb = accb + wgt * yb;
    }
    const double loa = dv * (fmax(u, 0.0) * s1a + fmin(u, 0.0) * s2a);
    const double lob = dv * (fmax(u, 0.0) * s1b + fmin(u, 0.0) * s2b);
    st2<LP>(fw(S, X_Ah), col8(e, p), col8(e, p + 1), k, PADW(u * acca - loa), PADW(u * accb - lob));
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

// one scalar's running sums of k_tr_bounds
struct TrAcc {
    double hlo = 0.0, pin = 0.0, pout = 0.0, smax, smin;
};
// one edge slot of k_tr_bounds for one scalar: the upwind flux's contribution, the
// antidiffusive in/out sums and the other cell's value in the bounds
__device__ __forceinline__ void tr_bound_slot(bool on, int s1f, double dv, double u, double x1, double x2, double A,
                                              TrAcc& r) {
    const double sg = s1f ? 1.0 : -1.0;
    const double lo = dv * (fmax(u, 0.0) * x1 + fmin(u, 0.0) * x2);
    r.hlo = add_if(on, r.hlo, sg * lo);
    const double a = -sg * A;
    r.pin = add_if(on, r.pin, fmax(a, 0.0));
    r.pout = sub_if(on, r.pout, fmin(a, 0.0));
    const double xo = s1f ? x2 : x1;
    r.smax = on ? fmax(r.smax, xo) : r.smax;
    r.smin = on ? fmin(r.smin, xo) : r.smin;
}

// the rest of k_tr_bounds for one scalar: vertical bounds and fluxes, su, R+ / R-
template <int LP>
__device__ __forceinline__ void tr_bound_fin(TrAcc& r, double s, double w, double r_o, double r_n, double invA,
                                             double rdzw, double fzm, double fzp, double dt, int k, int L,
                                             double& Rp, double& Rm, double& su) {
    const double sm1 = lvl_dn<LP>(s, k), sp1 = lvl_up<LP>(s, k);
    r.smax = k > 0 ? fmax(r.smax, sm1) : r.smax;
    r.smin = k > 0 ? fmin(r.smin, sm1) : r.smin;
    r.smax = k < L - 1 ? fmax(r.smax, sp1) : r.smax;
    r.smin = k < L - 1 ? fmin(r.smin, sp1) : r.smin;
    double lob, Ab;
    tr_vflux<LP>(s, w, k, L, fzm, fzp, lob, Ab);
    const double lot = lvl_up<LP>(lob, k), At = lvl_up<LP>(Ab, k);
    su = (s * r_o - dt * (r.hlo * invA + (lot - lob) * rdzw)) / r_n;
    r.smax = fmax(r.smax, su);
    r.smin = fmin(r.smin, su);
    const double pin_t = dt * (r.pin * invA + (fmax(Ab, 0.0) - fmin(At, 0.0)) * rdzw);
    const double pout_t = dt * (r.pout * invA + (fmax(At, 0.0) - fmin(Ab, 0.0)) * rdzw);
    const double qin = (r.smax - su) * r_n, qout = (su - r.smin) * r_n;
    Rp = pin_t > 0.0 ? fmin(1.0, qin / pin_t) : 0.0;
    Rm = pout_t > 0.0 ? fmin(1.0, qout / pout_t) : 0.0;
}

template <int LP, bool SELF>
__global__ __launch_bounds__(256) void k_tr_bounds(DevState S, double dt) {
    int c, p;
    tr_slot<LP>(S, KC, c, p);
    const int L = S.L, k = (int)(threadIdx.x % LP);
    if (c >= S.nCO) return;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    TrSlots t;
    tr_slots(S, c, t);
    const double invA = fd(S, F_invAreaCell)[c];
    const double rdzw = fd(S, F_rdzw)[k], fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double *so = fd(S, F_scalars_old), *ru = fd(S, F_ruAvg);
    const double* Ah = fd(S, X_Ah);
    double sa, sb;
    ld2<LP>(so, col8(c, p), col8(c, p + 1), k, sa, sb);
    const double w = colk(fd(S, F_wwAvg), c), r_o = colk(fd(S, F_rho_zz_old_split), c), r_n = colk(fd(S, F_rho_zz), c);
    double u_[NF], x1a[NF], x2a[NF], x1b[NF], x2b[NF], Aa[NF], Ab[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        u_[i] = colk(ru, t.e[i]);
        ld2<LP>(Ah, col8(t.e[i], p), col8(t.e[i], p + 1), k, Aa[i], Ab[i]);
        if constexpr (SELF) {
            double xa, xb;
            ld2<LP>(so, col8(t.oth[i], p), col8(t.oth[i], p + 1), k, xa, xb);
            x1a[i] = t.s1[i] ? sa : xa;
            x2a[i] = t.s1[i] ? xa : sa;
            x1b[i] = t.s1[i] ? sb : xb;
            x2b[i] = t.s1[i] ? xb : sb;
        } else {
            ld2<LP>(so, col8(t.c1[i], p), col8(t.c1[i], p + 1), k, x1a[i], x1b[i]);
            ld2<LP>(so, col8(t.c2[i], p), col8(t.c2[i], p + 1), k, x2a[i], x2b[i]);
        }
    }
    TrAcc ra, rb;
    ra.smax = ra.smin = sa;
    rb.smax = rb.smin = sb;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        tr_bound_slot(i < ne, t.s1[i], t.dv[i], u_[i], x1a[i], x2a[i], Aa[i], ra);
        tr_bound_slot(i < ne, t.s1[i], t.dv[i], u_[i], x1b[i], x2b[i], Ab[i], rb);
    }
    for (int i = NF; i < ne; i++) {  // cells with more than NF edges
        const size_t r = (size_t)c * 10 + i;
        const int e = fi(S, F_edgesOnCell)[r], c1 = fi(S, X_ce_c1)[r], c2 = fi(S, X_ce_c2)[r];
        const int s1f = fi(S, X_ce_s1)[r];
        const double dv = fd(S, X_ce_dv)[r], u = colk(ru, e);
        double y1a, y1b, y2a, y2b, Ba, Bb;
        ld2<LP>(so, col8(c1, p), col8(c1, p + 1), k, y1a, y1b);
        ld2<LP>(so, col8(c2, p), col8(c2, p + 1), k, y2a, y2b);
        ld2<LP>(Ah, col8(e, p), col8(e, p + 1), k, Ba, Bb);
        tr_bound_slot(true, s1f, dv, u, y1a, y2a, Ba, ra);
        tr_bound_slot(true, s1f, dv, u, y1b, y2b, Bb, rb);
    }
    double Rpa, Rma, sua, Rpb, Rmb, sub;
    tr_bound_fin<LP>(ra, sa, w, r_o, r_n, invA, rdzw, fzm, fzp, dt, k, L, Rpa, Rma, sua);
    tr_bound_fin<LP>(rb, sb, w, r_o, r_n, invA, rdzw, fzm, fzp, dt, k, L, Rpb, Rmb, sub);
    // level L and the padding levels of the scratch are never read
    st2<LP>(fw(S, X_Rp), col8(c, p), col8(c, p + 1), k, Rpa, Rpb);
    st2<LP>(fw(S, X_Rm), col8(c, p), col8(c, p + 1), k, Rma, Rmb);
    st2<LP>(fw(S, X_su), col8(c, p), col8(c, p + 1), k, sua, sub);
}

// the limited update of one scalar
template <int LP>
__device__ __forceinline__ double tr_update_fin(double hc, double s, double w, double su, double rp, double rm,
                                                double r_n, double invA, double rdzw, double fzm, double fzp,
                                                double dt, int k, int L) {
    double lo, A;
    tr_vflux<LP>(s, w, k, L, fzm, fzp, lo, A);
    const double rp_b = lvl_dn<LP>(rp, k), rm_b = lvl_dn<LP>(rm, k);
    const double fcb = (k >= 1 && k <= L - 1) ? (A >= 0.0 ? fmin(rm_b, rp) : fmin(rp_b, rm)) * A : 0.0;
    const double fct = lvl_up<LP>(fcb, k);
    return su - dt * (hc * invA + (fct - fcb) * rdzw) / r_n;
}
__device__ __forceinline__ double tr_limited(double A, double m1, double p2, double p1, double m2) {
    return (A >= 0.0 ? fmin(m1, p2) : fmin(p1, m2)) * A;
}

template <int LP, bool SELF>
__global__ __launch_bounds__(256) void k_tr_update(DevState S, double dt) {
    int c, p;
    tr_slot<LP>(S, KC, c, p);
    const int L = S.L, k = (int)(threadIdx.x % LP);
    if (c >= S.nCO) return;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    TrSlots t;
    tr_slots(S, c, t);
    const double invA = fd(S, F_invAreaCell)[c];
    const double rdzw = fd(S, F_rdzw)[k], fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double *Ah = fd(S, X_Ah), *Rp = fd(S, X_Rp), *Rm = fd(S, X_Rm);
    const size_t ca = col8(c, p), cb = col8(c, p + 1);
    double sa, sb, sua, sub, rpa, rpb, rma, rmb;
    ld2<LP>(fd(S, F_scalars_old), ca, cb, k, sa, sb);
    ld2<LP>(fd(S, X_su), ca, cb, k, sua, sub);
    ld2<LP>(Rp, ca, cb, k, rpa, rpb);
    ld2<LP>(Rm, ca, cb, k, rma, rmb);
    const double w = colk(fd(S, F_wwAvg), c), r_n = colk(fd(S, F_rho_zz), c);
    double Aa[NF], Ab[NF], p1a[NF], p1b[NF], m1a[NF], m1b[NF], p2a[NF], p2b[NF], m2a[NF], m2b[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        ld2<LP>(Ah, col8(t.e[i], p), col8(t.e[i], p + 1), k, Aa[i], Ab[i]);
        if constexpr (SELF) {  // the cell is one of the two: gather only the other
            double qa, qb, na, nb;
            ld2<LP>(Rp, col8(t.oth[i], p), col8(t.oth[i], p + 1), k, qa, qb);
            ld2<LP>(Rm, col8(t.oth[i], p), col8(t.oth[i], p + 1), k, na, nb);
            const bool f = t.s1[i];
            p1a[i] = f ? rpa : qa, p1b[i] = f ? rpb : qb, m1a[i] = f ? rma : na, m1b[i] = f ? rmb : nb;
            p2a[i] = f ? qa : rpa, p2b[i] = f ? qb : rpb, m2a[i] = f ? na : rma, m2b[i] = f ? nb : rmb;
        } else {
            ld2<LP>(Rp, col8(t.c1[i], p), col8(t.c1[i], p + 1), k, p1a[i], p1b[i]);
            ld2<LP>(Rm, col8(t.c1[i], p), col8(t.c1[i], p + 1), k, m1a[i], m1b[i]);
            ld2<LP>(Rp, col8(t.c2[i], p), col8(t.c2[i], p + 1), k, p2a[i], p2b[i]);
            ld2<LP>(Rm, col8(t.c2[i], p), col8(t.c2[i], p + 1), k, m2a[i], m2b[i]);
        }
    }
    double hca = 0.0, hcb = 0.0;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        const double sg = t.s1[i] ? 1.0 : -1.0;
        hca = add_if(i < ne, hca, sg * tr_limited(Aa[i], m1a[i], p2a[i], p1a[i], m2a[i]));
        hcb = add_if(i < ne, hcb, sg * tr_limited(Ab[i], m1b[i], p2b[i], p1b[i], m2b[i]));
    }
    for (int i = NF; i < ne; i++) {
        const size_t r = (size_t)c * 10 + i;
        const int e = fi(S, F_edgesOnCell)[r], c1 = fi(S, X_ce_c1)[r], c2 = fi(S, X_ce_c2)[r];
        const double sg = fi(S, X_ce_s1)[r] ? 1.0 : -1.0;
        double Ba, Bb, q1a, q1b, n1a, n1b, q2a, q2b, n2a, n2b;
        ld2<LP>(Ah, col8(e, p), col8(e, p + 1), k, Ba, Bb);
        ld2<LP>(Rp, col8(c1, p), col8(c1, p + 1), k, q1a, q1b);
        ld2<LP>(Rm, col8(c1, p), col8(c1, p + 1), k, n1a, n1b);
        ld2<LP>(Rp, col8(c2, p), col8(c2, p + 1), k, q2a, q2b);
        ld2<LP>(Rm, col8(c2, p), col8(c2, p + 1), k, n2a, n2b);
        hca = hca + sg * tr_limited(Ba, n1a, q2a, q1a, n2a);
        hcb = hcb + sg * tr_limited(Bb, n1b, q2b, q1b, n2b);
    }
    const double na = tr_update_fin<LP>(hca, sa, w, sua, rpa, rma, r_n, invA, rdzw, fzm, fzp, dt, k, L);
    const double nb = tr_update_fin<LP>(hcb, sb, w, sub, rpb, rmb, r_n, invA, rdzw, fzm, fzp, dt, k, L);
    if (k < L) {  // level L of scalars keeps its value (the oracle writes levels 0..L-1)
        double* sn = fw(S, F_scalars);
        sn[ca * LP + lpos(LP, k)] = na;
        sn[cb * LP + lpos(LP, k)] = nb;
    }
}

template <int LP>
static hipError_t transport_lp(const DevState& S, hipStream_t st, double dt) {
    constexpr int COLS = 256 / LP;  // column slots per block; a slot = one entity, two scalars
    auto blocks = [](const DevState& X, int kind) {
        const int end = kind == KC ? X.nCO : X.nEO;
        const long n = (long)(end - X.lo[kind]) * (NSC / 2);
        return n > 0 ? (int)((n + COLS - 1) / COLS) : 0;
    };
    // decomposed meshes: the gathered fields are exchanged first (HALO_RUN: scalars_old
    // on two rings for the adv lists, A on the ghost edges of owned cells, R+/R- on the
    // neighbour cells); the x8 fields move as 8 columns per entity (mpas_halo.hip)
    auto ke = [&](const DevState& X) {
        const int nb = blocks(X, KE);
        if (nb) k_tr_edge<LP><<<nb, 256, 0, st>>>(X);
    };
    HALO_RUN(S, st, ke, F_scalars_old, F_ruAvg);
    HALO_WROTE(S, X_Ah);
    auto kb = [&](const DevState& X) {
        const int nb = blocks(X, KC);
        if (nb && X.selfc) k_tr_bounds<LP, true><<<nb, 256, 0, st>>>(X, dt);
        else if (nb) k_tr_bounds<LP, false><<<nb, 256, 0, st>>>(X, dt);
    };
    HALO_RUN(S, st, kb, F_scalars_old, F_ruAvg, X_Ah);
    HALO_WROTE(S, X_Rp, X_Rm, X_su);
    auto ku = [&](const DevState& X) {
        const int nb = blocks(X, KC);
        if (nb && X.selfc) k_tr_update<LP, true><<<nb, 256, 0, st>>>(X, dt);
        else if (nb) k_tr_update<LP, false><<<nb, 256, 0, st>>>(X, dt);
    };
    HALO_RUN(S, st, ku, X_Ah, X_Rp, X_Rm);
    HALO_WROTE(S, F_scalars);
    return hipGetLastError();
}
hipError_t launch_advance_scalars_mono(const DevState& S, hipStream_t st, double dt) {
    MPAS_LP_DISPATCH(S.LP, transport_lp, S, st, dt);
}

}  // namespace mpas
