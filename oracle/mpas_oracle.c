/* mpas_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
 * RK3 dynamics hot path (alexaiken/mpas-regent), used as the parity checker by
 * tests/, __graft_entry__.smoke() and the cpu_baseline leg of bench.py.  Nothing in
 * the product (mpas-regent_amd/) links, loads or calls this file.
 *
 * PARITY UNPINNED: the reference is Regent source that cannot be compiled or run here
 * (no Regent/Legion/Terra) and it ships no tests, fixtures or golden
 * vectors.  This restatement follows the Regent text line by line; every
 * function cites the lines it follows.  Undefined behaviour in the reference is
 * resolved by the written policies of SURVEY §8.0 ("ref" mode):
 *   Q1  raw ids are used as offsets; every entity array has one extra all-zero row n
 *       (the "zero slot", never written); any other out-of-range entity -> 0.0.
 *   Q2  never-written fields are inputs (zero in a literal "ref" state).
 *   OOB levels (k < 0 or k > nVertLevels) read 0.0.
 *   pow(x, 2.0) is evaluated as x*x; pow of compile-time constants is folded.
 *   min(a,b) := a < b ? a : b, max(a,b) := a > b ? a : b.
 *   Loops run entity-outer / level-inner, which the loop-order note of SURVEY §8.0
 *   shows equivalent to Legion's point order for every task on the path.
 * Layout (the reference's int2d region indexing): a cell field f is f[cell*(L+1)+k]
 * for k = 0..L; C3V fields are f[(cell*(L+1)+k)*W + i]; 2-D mesh fields f[e*W + i].
 * Build with -ffp-contract=off so that every a*b+c rounds twice, as written.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "mpas_synth.h"

/* ---------------- field registry ---------------- */
enum {
#define MPAS_FIELD(name, KIND, W, D, LO, HI) F_##name,
#include "mpas_fields.def"
#undef MPAS_FIELD
    F_COUNT
};

typedef struct {
    int32_t nCells, nEdges, nVertices, L; /* L = nVertLevels */
    void* f[F_COUNT];                     /* host arrays, reference layout */
} ora_state;

/* constants.rg:27-66 */
static const double rgas = 287.0;
#define CP (7.0 * 287.0 / 2.0)
static const double gravity = 9.80616;
static const double omega_c = 7.29212E-5;
static const double config_epssm = 0.1;
static const double prandtl = 1.0;
static const int nRelaxZone = 5;
static const double config_smdiv = 0.1;
static const double config_len_disp = 120000.0;
static const double config_visc4_2dsmag = 0.05;
static const double config_smagorinsky_coef = 0.125;
static const double config_del4u_div_factor = 10.0;
static const int config_number_rayleigh_damp_u_levels = 6;
static const double config_rayleigh_damp_u_timescale_days = 5.0;
static const double seconds_per_day = 86400.0;
static const double sphere_radius = 6371229.0;

#define D(name) ((double*)S->f[F_##name])
#define I(name) ((int32_t*)S->f[F_##name])
#define B(name) ((uint8_t*)S->f[F_##name])
#define LV (S->L + 1)
#define NSC 8 /* nScalars, constants.rg:42 */

static inline double dmin(double a, double b) { return a < b ? a : b; }
static inline double dmax(double a, double b) { return a > b ? a : b; }

/* Q1/OOB read policy */
static inline double rc(const ora_state* S, const double* f, long i, long k) {
    if (i < 0 || i > S->nCells || k < 0 || k > S->L) return 0.0;
    return f[i * LV + k];
}
static inline double re(const ora_state* S, const double* f, long i, long k) {
    if (i < 0 || i > S->nEdges || k < 0 || k > S->L) return 0.0;
    return f[i * LV + k];
}
static inline double rv(const ora_state* S, const double* f, long i, long k) {
    if (i < 0 || i > S->nVertices || k < 0 || k > S->L) return 0.0;
    return f[i * LV + k];
}
static inline double rz(const ora_state* S, const double* f, long k) {
    if (k < 0 || k > S->L) return 0.0;
    return f[k];
}
static inline double rc2(const ora_state* S, const double* f, long i, int W, int c) {
    if (i < 0 || i > S->nCells || c < 0 || c >= W) return 0.0;
    return f[i * W + c];
}
static inline double re2(const ora_state* S, const double* f, long i, int W, int c) {
    if (i < 0 || i > S->nEdges || c < 0 || c >= W) return 0.0;
    return f[i * W + c];
}
static inline double rv2(const ora_state* S, const double* f, long i, int W, int c) {
    if (i < 0 || i > S->nVertices || c < 0 || c >= W) return 0.0;
    return f[i * W + c];
}
static inline int ic2(const ora_state* S, const int32_t* f, long i, int W, int c) {
    if (i < 0 || i > S->nCells || c < 0 || c >= W) return 0;
    return f[i * W + c];
}
static inline int ie2(const ora_state* S, const int32_t* f, long i, int W, int c) {
    if (i < 0 || i > S->nEdges || c < 0 || c >= W) return 0;
    return f[i * W + c];
}
static inline int iv2(const ora_state* S, const int32_t* f, long i, int W, int c) {
    if (i < 0 || i > S->nVertices || c < 0 || c >= W) return 0;
    return f[i * W + c];
}
static inline double rc3v(const ora_state* S, const double* f, long i, long k, int c) {
    if (i < 0 || i > S->nCells || k < 0 || k > S->L || c < 0 || c >= 10) return 0.0;
    return f[(i * LV + k) * 10 + c];
}
#define CW(f, i, k) (f)[(long)(i) * LV + (k)] /* own-point write/read */

/* flux4/flux3, dynamics_tasks.rg:780-789 */
static inline double flux4(double q_im2, double q_im1, double q_i, double q_ip1, double ua) {
    return ua * (7. * (q_i + q_im1) - (q_ip1 + q_im2)) / 12.0;
}
static inline double flux3(double q_im2, double q_im1, double q_i, double q_ip1, double ua, double coef3) {
    return flux4(q_im2, q_im1, q_i, q_ip1, ua) + coef3 * fabs(ua) * ((q_ip1 - q_im2) - 3. * (q_i - q_im1)) / 12.0;
}
/* rayleigh_damp_coef, dynamics_tasks.rg:791-796 */
static inline double rayleigh_damp_coef(const ora_state* S, double vertLevel) {
    double inv = 1.0 / ((double)config_number_rayleigh_damp_u_levels *
                        (config_rayleigh_damp_u_timescale_days * seconds_per_day));
    return (double)(vertLevel - (S->L - config_number_rayleigh_damp_u_levels)) * inv;
}

/* ===================== atm_compute_solve_diagnostics, dynamics_tasks.rg:328-454 */
void ora_atm_compute_solve_diagnostics(ora_state* S, int hollingsworth, int rk_step) {
    const int L = S->L, nC = S->nCells, nE = S->nEdges, nV = S->nVertices;
    double *u = D(u), *h = D(h), *h_edge = D(h_edge), *ke_edge = D(ke_edge);
    double *dcEdge = D(dcEdge), *dvEdge = D(dvEdge);
    int32_t* cellsOnEdge = I(cellsOnEdge);
    /* :346-353 */
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) {
        int cell1 = ie2(S, cellsOnEdge, e, 2, 0), cell2 = ie2(S, cellsOnEdge, e, 2, 1);
        for (int k = 0; k < L; k++) {
            CW(h_edge, e, k) = 0.5 * (rc(S, h, cell1, k) + rc(S, h, cell2, k));
            double efac = re2(S, dcEdge, e, 1, 0) * re2(S, dvEdge, e, 1, 0);
            double uu = CW(u, e, k);
            CW(ke_edge, e, k) = efac * (uu * uu);
        }
    }
    /* :356-366 */
    double *vort = D(vorticity);
#pragma omp parallel for schedule(static)
    for (long v = 0; v < nV; v++) {
        for (int k = 0; k < L; k++) {
            CW(vort, v, k) = 0.0;
            for (int i = 0; i < 3; i++) {
                int iEdge = iv2(S, I(edgesOnVertex), v, 3, i);
                double s = rv2(S, D(edgesOnVertexSign), v, 3, i) * re2(S, dcEdge, iEdge, 1, 0);
                CW(vort, v, k) += s * re(S, u, iEdge, k);
            }
            CW(vort, v, k) *= rv2(S, D(invAreaTriangle), v, 1, 0);
        }
    }
    /* :369-379 (Q9: divergence += s + u, literal) */
    double *div = D(divergence), *ke = D(ke);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        for (int k = 0; k < L; k++) {
            CW(div, c, k) = 0.0;
            for (int i = 0; i < ne; i++) {
                int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
                double s = rc2(S, D(edgesOnCellSign), c, 10, i) * re2(S, dvEdge, iEdge, 1, 0);
                CW(div, c, k) += s + re(S, u, iEdge, k);
            }
            double r = rc2(S, D(invAreaCell), c, 1, 0);
            CW(div, c, k) *= r;
        }
        /* :382-390 */
        for (int k = 0; k < L; k++) {
            CW(ke, c, k) = 0.0;
            for (int i = 0; i < ne; i++) {
                int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
                CW(ke, c, k) += 0.25 * re(S, ke_edge, iEdge, k);
            }
            CW(ke, c, k) *= rc2(S, D(invAreaCell), c, 1, 0);
        }
    }
    if (hollingsworth) { /* :392-418 */
        double* ke_vertex = D(ke_vertex);
#pragma omp parallel for schedule(static)
        for (long v = 0; v < nV; v++) {
            double r = 0.25 * rv2(S, D(invAreaTriangle), v, 1, 0);
            for (int k = 0; k < L; k++) {
                CW(ke_vertex, v, k) = (re(S, ke_edge, iv2(S, I(edgesOnVertex), v, 3, 0), k) +
                                       re(S, ke_edge, iv2(S, I(edgesOnVertex), v, 3, 1), k) +
                                       re(S, ke_edge, iv2(S, I(edgesOnVertex), v, 3, 2), k)) * r;
            }
        }
        double ke_fact = 1.0 - 0.375;
#pragma omp parallel for schedule(static)
        for (long c = 0; c < nC; c++) {
            for (int k = 0; k < L; k++) CW(ke, c, k) *= ke_fact;
            double r = rc2(S, D(invAreaCell), c, 1, 0);
            int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
            for (int k = 0; k < L; k++) {
                for (int i = 0; i < ne; i++) {
                    int iVertex = ic2(S, I(verticesOnCell), c, 10, i);
                    int j = ic2(S, I(kiteForCell), c, 10, i);
                    CW(ke, c, k) += (1.0 - ke_fact) * rv2(S, D(kiteAreasOnVertex), iVertex, 3, j) *
                                    rv(S, ke_vertex, iVertex, k) * r;
                }
            }
        }
    }
    /* :422-439 (Q23: starts at i = 1) */
    int reconstruct_v = 1;
    if (rk_step != -1 && rk_step != 2) reconstruct_v = 0;
    if (reconstruct_v) {
        double* vv = D(v);
#pragma omp parallel for schedule(static)
        for (long e = 0; e < nE; e++) {
            int neoe = ie2(S, I(nEdgesOnEdge), e, 1, 0);
            for (int k = 0; k < L; k++) {
                CW(vv, e, k) = 0;
                for (int i = 1; i < neoe; i++) {
                    int eoe = ie2(S, I(edgesOnEdge_ECP), e, 20, i);
                    CW(vv, e, k) += re2(S, D(weightsOnEdge), e, 20, i) * re(S, u, eoe, k);
                }
            }
        }
    }
    /* :443-445 */
    double* pv_vertex = D(pv_vertex);
#pragma omp parallel for schedule(static)
    for (long v = 0; v < nV; v++)
        for (int k = 0; k < L; k++) CW(pv_vertex, v, k) = rv2(S, D(fVertex), v, 1, 0) + CW(vort, v, k);
    /* :449-451 */
    double* pv_edge = D(pv_edge);
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) {
        int v1 = ie2(S, I(verticesOnEdge), e, 2, 0), v2 = ie2(S, I(verticesOnEdge), e, 2, 1);
        for (int k = 0; k < L; k++) CW(pv_edge, e, k) = 0.5 * (rv(S, pv_vertex, v1, k) + rv(S, pv_vertex, v2, k));
    }
}

/* ===================== atm_compute_moist_coefficients, dynamics_tasks.rg:460-502 */
void ora_atm_compute_moist_coefficients(ora_state* S) {
    const int L = S->L, nC = S->nCells;
    double *qtot = D(qtot), *cqw = D(cqw);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        for (int k = 0; k < L; k++) CW(qtot, c, k) = 0.0; /* :473-482 */
        for (int k = 0; k < L; k++) {                      /* :484-489 */
            if (k > 0) {
                double qtotal = 0.5 * (CW(qtot, c, k) + CW(qtot, c, k - 1));
                CW(cqw, c, k) = 1.0 / (1.0 + qtotal);
            }
        }
    }
    /* :491-501 edge loop body is commented out in the reference: nothing to do */
}

/* ===================== atm_compute_vert_imp_coefs, dynamics_tasks.rg:513-592 */
void ora_atm_compute_vert_imp_coefs(ora_state* S, double dts) {
    const int L = S->L, nC = S->nCells;
    double dtseps = .5 * dts * (1.0 + config_epssm);
    double rcv = rgas / (CP - rgas);
    double c2 = CP * rcv;
    double *rdzu = D(rdzu), *rdzw = D(rdzw), *fzm = D(fzm), *fzp = D(fzp), *cofrz = D(cofrz);
    for (int k = 0; k < L; k++) cofrz[k] = dtseps * rdzw[k]; /* :537-539 */
    double *zz = D(zz), *cofwr = D(cofwr), *cofwz = D(cofwz), *coftz = D(coftz), *cofwt = D(cofwt);
    double *cqw = D(cqw), *exner = D(exner), *theta_m = D(theta_m), *qtot = D(qtot);
    double *rho_base = D(rho_base), *rtheta_base = D(rtheta_base), *rtheta_p = D(rtheta_p);
    double *exner_base = D(exner_base);
    double *a_tri = D(a_tri), *b_tri = D(b_tri), *c_tri = D(c_tri), *alpha_tri = D(alpha_tri);
    double* gamma_tri = D(gamma_tri);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        CW(gamma_tri, c, 0) = 0.0; /* :541-547 */
        for (int k = 0; k < L; k++) { /* :550-564 */
            if (k > 0)
                CW(cofwr, c, k) = .5 * dtseps * gravity * (fzm[k] * CW(zz, c, k) + fzp[k] * CW(zz, c, k - 1));
            CW(coftz, c, k) = 0.0;
            if (k > 0) {
                CW(cofwz, c, k) = dtseps * c2 * (fzm[k] * CW(zz, c, k) + fzp[k] * CW(zz, c, k - 1)) * rdzu[k] *
                                  CW(cqw, c, k) * (fzm[k] * CW(exner, c, k) + fzp[k] * CW(exner, c, k - 1));
                CW(coftz, c, k) = dtseps * (fzm[k] * CW(theta_m, c, k) + fzp[k] * CW(theta_m, c, k - 1));
            }
            double qtotal = CW(qtot, c, k);
            CW(cofwt, c, k) = .5 * dtseps * rcv * CW(zz, c, k) * gravity * CW(rho_base, c, k) / (1.0 + qtotal) *
                              CW(exner, c, k) / ((CW(rtheta_base, c, k) + CW(rtheta_p, c, k)) * CW(exner_base, c, k));
        }
        for (int k = 1; k < L; k++) { /* :566-578 */
            CW(a_tri, c, k) = -1.0 * CW(cofwz, c, k) * CW(coftz, c, k - 1) * rdzw[k - 1] * CW(zz, c, k - 1) +
                              CW(cofwr, c, k) * cofrz[k - 1] -
                              CW(cofwt, c, k - 1) * CW(coftz, c, k - 1) * rdzw[k - 1];
            CW(b_tri, c, k) = 1.0 +
                              CW(cofwz, c, k) * (CW(coftz, c, k) * rdzw[k] * CW(zz, c, k) +
                                                 CW(coftz, c, k) * rdzw[k - 1] * CW(zz, c, k - 1)) -
                              CW(coftz, c, k) * (CW(cofwt, c, k) * rdzw[k] - CW(cofwt, c, k) * rdzw[k - 1]) +
                              CW(cofwr, c, k) * ((cofrz[k] - cofrz[k - 1]));
            CW(c_tri, c, k) = -1.0 * CW(cofwz, c, k) * rc(S, coftz, c, k + 1) * rdzw[k] * CW(zz, c, k) -
                              CW(cofwr, c, k) * cofrz[k] + CW(cofwt, c, k) * rc(S, coftz, c, k + 1) * rdzw[k];
        }
        for (int k = 1; k < L; k++) /* :580-585 (Q17: gamma of the previous call) */
            CW(alpha_tri, c, k) = 1.0 / (CW(b_tri, c, k) - CW(a_tri, c, k) * CW(gamma_tri, c, k - 1));
        for (int k = 1; k < L; k++) /* :587-591 */
            CW(gamma_tri, c, k) = CW(c_tri, c, k) * CW(alpha_tri, c, k);
    }
}

/* ===================== atm_rk_integration_setup, dynamics_tasks.rg:747-778 */
void ora_atm_rk_integration_setup(ora_state* S) {
    const int L = S->L;
#pragma omp parallel for schedule(static)
    for (long e = 0; e < S->nEdges; e++)
        for (int k = 0; k < L; k++) {
            CW(D(ru_save), e, k) = CW(D(ru), e, k);
            CW(D(u_2), e, k) = CW(D(u), e, k);
        }
#pragma omp parallel for schedule(static)
    for (long c = 0; c < S->nCells; c++)
        for (int k = 0; k < L; k++) {
            CW(D(rw_save), c, k) = CW(D(rw), c, k);
            CW(D(rtheta_p_save), c, k) = CW(D(rtheta_p), c, k);
            CW(D(rho_p_save), c, k) = CW(D(rho_p), c, k);
            CW(D(w_2), c, k) = CW(D(w), c, k);
            CW(D(theta_m_2), c, k) = CW(D(theta_m), c, k);
            CW(D(rho_zz_2), c, k) = CW(D(rho_zz), c, k);
            CW(D(rho_zz_old_split), c, k) = CW(D(rho_zz), c, k);
        }
}

/* ===================== atm_compute_dyn_tend_work, dynamics_tasks.rg:814-1480
 * horiz_mixing: 0 = "2d_smagorinsky", 1 = "2d_fixed", other = neither.
 * The v_mom/v_theta_eddy_visc2 branches (:1094-1146, :1304-1315, :1430-1475) are dead
 * code under constants.rg:47-48 (both 0.0) and are not restated.                    */
static void dyn_tend_impl(ora_state* S, int rk_step, double dt, int horiz_mixing, double config_mpas_cam_coef,
                          int config_mix_full, int config_rayleigh_damp_u, int mpas) {
    (void)config_mix_full;
    const int L = S->L, nC = S->nCells, nE = S->nEdges, nV = S->nVertices;
    double prandtl_inv = 1.0 / prandtl;
    double invDt = 1.0 / dt;
    double r_earth = sphere_radius;
    double inv_r_earth = 1.0 / r_earth;
    double h_mom_eddy_visc4 = 0.0, h_theta_eddy_visc4 = 0.0;
    double *u = D(u), *v = D(v), *kdiff = D(kdiff), *ru = D(ru), *rw = D(rw);
    int32_t *nEdgesOnCell = I(nEdgesOnCell), *edgesOnCell = I(edgesOnCell), *cellsOnEdge = I(cellsOnEdge);
    double *eocs = D(edgesOnCell_sign), *dvEdge = D(dvEdge), *invAreaCell = D(invAreaCell);
    double *invDcEdge = D(invDcEdge);
    double *fzm = D(fzm), *fzp = D(fzp), *rdzw = D(rdzw), *rdzu = D(rdzu);

    if (rk_step == 0) {
        if (horiz_mixing == 0) { /* :861-890 (Q11: only d_diag[k] of the own level is used) */
            double c_s = config_smagorinsky_coef;
            double cs_l2 = (c_s * config_len_disp) * (c_s * config_len_disp); /* pow(c_s*len,2.0) */
            double cap = (0.01 * (config_len_disp * config_len_disp)) * invDt;
#pragma omp parallel for schedule(static)
            for (long c = 0; c < nC; c++) {
                int ne = ic2(S, nEdgesOnCell, c, 1, 0);
                for (int k = 0; k < L; k++) {
                    double d_diag = 0.0, d_off_diag = 0.0;
                    for (int iEdge = 0; iEdge < ne; iEdge++) {
                        int e = ic2(S, edgesOnCell, c, 10, iEdge);
                        d_diag += rc2(S, D(defc_a), c, 10, iEdge) * re(S, u, e, k) - rc2(S, D(defc_b), c, 10, iEdge) * re(S, v, e, k);
                        d_off_diag += rc2(S, D(defc_b), c, 10, iEdge) * re(S, u, e, k) + rc2(S, D(defc_a), c, 10, iEdge) * re(S, v, e, k);
                    }
                    CW(kdiff, c, k) = dmin(cs_l2 * sqrt(d_diag * d_diag + d_off_diag * d_off_diag), cap);
                }
            }
            h_mom_eddy_visc4 = config_visc4_2dsmag * (config_len_disp * config_len_disp * config_len_disp);
            h_theta_eddy_visc4 = h_mom_eddy_visc4;
        } else if (horiz_mixing == 1) {
#pragma omp parallel for schedule(static)
            for (long c = 0; c < nC; c++)
                for (int k = 0; k < L; k++) CW(kdiff, c, k) = 0.0;
        }
        if (config_mpas_cam_coef > 0.0) { /* :898-916 */
#pragma omp parallel for schedule(static)
            for (long c = 0; c < nC; c++)
                for (int k = 0; k < L; k++)
                    if (k >= L - 2 && k <= L) {
                        int p = k - (L - 2);
                        CW(kdiff, c, k) = dmax(CW(kdiff, c, k), pow(2, p) * 2.0833 * config_len_disp * config_mpas_cam_coef);
                    }
        }
    }

    double* h_divergence = D(h_divergence);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) { /* :924-938 */
        int ne = ic2(S, nEdgesOnCell, c, 1, 0);
        for (int k = 0; k < L; k++) {
            CW(h_divergence, c, k) = 0.0;
            for (int i = 0; i < ne; i++) {
                int iEdge = ic2(S, edgesOnCell, c, 10, i);
                double edge_sign = rc2(S, eocs, c, 10, i) * re2(S, dvEdge, iEdge, 1, 0);
                CW(h_divergence, c, k) += edge_sign * re(S, ru, iEdge, k);
            }
        }
        for (int k = 0; k < L; k++) {
            double r = rc2(S, invAreaCell, c, 1, 0);
            CW(h_divergence, c, k) *= r;
        }
    }

    double *tend_rho = D(tend_rho), *dpdz = D(dpdz);
    if (rk_step == 0) { /* :942-951 */
#pragma omp parallel for schedule(static)
        for (long c = 0; c < nC; c++)
            for (int k = 0; k < L; k++) {
                if (mpas) /* MPAS-A: the physics tendency outside the vertical flux divergence */
                    CW(tend_rho, c, k) = -CW(h_divergence, c, k) - rdzw[k] * (rc(S, rw, c, k + 1) - CW(rw, c, k)) +
                                         CW(D(tend_rho_physics), c, k);
                else
                    CW(tend_rho, c, k) = -CW(h_divergence, c, k) -
                                         rdzw[k] * (rc(S, rw, c, k + 1) - CW(rw, c, k) + CW(D(tend_rho_physics), c, k));
                CW(dpdz, c, k) = -gravity * (CW(D(rho_base), c, k) * (CW(D(qtot), c, k)) +
                                             CW(D(rho_p_save), c, k) * (1.0 + CW(D(qtot), c, k)));
            }
    }

    /* -------- U section -------- */
    double *tend_u_euler = D(tend_u_euler), *wduz = D(wduz), *tend_u = D(tend_u), *q = D(q);
    double *pressure_p = D(pressure_p), *zz = D(zz), *zxu = D(zxu), *cqu = D(cqu);
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) { /* :958-981 */
        int cell1 = ie2(S, cellsOnEdge, e, 2, 0), cell2 = ie2(S, cellsOnEdge, e, 2, 1);
        for (int k = 0; k < L; k++) {
            if (rk_step == 0) {
                CW(tend_u_euler, e, k) =
                    -CW(cqu, e, k) * ((rc(S, pressure_p, cell2, k) - rc(S, pressure_p, cell1, k)) * re2(S, invDcEdge, e, 1, 0) /
                                          (0.5 * (rc(S, zz, cell2, k) + rc(S, zz, cell1, k))) -
                                      0.5 * CW(zxu, e, k) * (rc(S, dpdz, cell1, k) + rc(S, dpdz, cell2, k)));
            }
            CW(wduz, e, k) = 0.0;
            if (k == 1 || k == L - 1)
                CW(wduz, e, k) = 0.5 * (rc(S, rw, cell1, k) + rc(S, rw, cell2, k)) *
                                 (fzm[k] * CW(u, e, k) + fzp[k] * re(S, u, e, k - 1));
            if (k > 1 && k < L - 1)
                CW(wduz, e, k) = flux3(re(S, u, e, k - 2), re(S, u, e, k - 1), CW(u, e, k), re(S, u, e, k + 1),
                                       0.5 * (rc(S, rw, cell1, k) + rc(S, rw, cell2, k)), 1.0);
        }
    }
    double *pv_edge = D(pv_edge), *rho_edge = D(rho_edge), *ke = D(ke), *w = D(w);
    double *cosA = D(angleEdge), *latE = D(latEdge); /* cos() taken below, glibc */
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) { /* :983-1019 */
        int cell1 = ie2(S, cellsOnEdge, e, 2, 0), cell2 = ie2(S, cellsOnEdge, e, 2, 1);
        int neoe = ie2(S, I(nEdgesOnEdge), e, 1, 0);
        for (int k = 0; k < L; k++) {
            /* (mpas: wduz(nVertLevels) = 0, MPAS-A's top boundary; the reference reads the
             * never-written level-L slot) */
            const double wduz_p = (mpas && k + 1 == L) ? 0.0 : re(S, wduz, e, k + 1);
            CW(tend_u, e, k) = -rdzw[k] * (wduz_p - CW(wduz, e, k));
            CW(q, e, k) = 0.0;
            for (int j = 0; j < neoe; j++) { /* Q10: each term accumulated nVertLevels times */
                int eoe = ie2(S, I(edgesOnEdge), e, 20, j);
                for (int kk = 0; kk < (mpas ? 1 : L); kk++) { /* (mpas: once) */
                    double workpv = 0.5 * (CW(pv_edge, e, k) + re(S, pv_edge, eoe, k));
                    CW(q, e, k) += re2(S, D(weightsOnEdge), e, 20, j) * re(S, u, eoe, k) * workpv;
                }
            }
            CW(tend_u, e, k) += CW(rho_edge, e, k) * (CW(q, e, k) - (rc(S, ke, cell2, k) - rc(S, ke, cell1, k)) * re2(S, invDcEdge, e, 1, 0)) -
                                CW(u, e, k) * 0.5 * (rc(S, h_divergence, cell1, k) + rc(S, h_divergence, cell2, k));
            /* Q12: -= (A) - (B), literal; mpas: tend_u - A - B */
            const double cA = (2.0 * omega_c * cos(re2(S, cosA, e, 1, 0)) * cos(re2(S, latE, e, 1, 0)) * CW(rho_edge, e, k) * 0.25 *
                               (rc(S, w, cell1, k) + rc(S, w, cell1, k + 1) + rc(S, w, cell2, k) + rc(S, w, cell2, k + 1)));
            const double cB = (CW(u, e, k) * 0.25 * (rc(S, w, cell1, k) + rc(S, w, cell1, k + 1) + rc(S, w, cell2, k) + rc(S, w, cell2, k + 1)) *
                               CW(rho_edge, e, k) * inv_r_earth);
            if (mpas)
                CW(tend_u, e, k) = CW(tend_u, e, k) - cA - cB;
            else
                CW(tend_u, e, k) -= cA - cB;
        }
    }

    double *delsq_u = D(delsq_u), *divergence = D(divergence), *vorticity = D(vorticity);
    double *delsq_vorticity = D(delsq_vorticity), *delsq_divergence = D(delsq_divergence);
    if (rk_step == 0) { /* :1025-1091 */
#pragma omp parallel for schedule(static)
        for (long e = 0; e < nE; e++) {
            int cell1 = ie2(S, cellsOnEdge, e, 2, 0), cell2 = ie2(S, cellsOnEdge, e, 2, 1);
            int vertex1 = ie2(S, I(verticesOnEdge), e, 2, 0), vertex2 = ie2(S, I(verticesOnEdge), e, 2, 1);
            double r_dc = re2(S, invDcEdge, e, 1, 0);
            double r_dv = dmin(re2(S, D(invDvEdge), e, 1, 0), 4 * r_dc);
            for (int k = 0; k < L; k++) {
                CW(delsq_u, e, k) = 0.0;
                double u_diffusion = (rc(S, divergence, cell2, k) - rc(S, divergence, cell1, k)) * r_dc -
                                     (rv(S, vorticity, vertex2, k) - rv(S, vorticity, vertex1, k)) * r_dv;
                CW(delsq_u, e, k) += u_diffusion;
                double kdiffu = 0.5 * (rc(S, kdiff, cell1, k) + rc(S, kdiff, cell2, k));
                CW(tend_u_euler, e, k) += CW(rho_edge, e, k) * kdiffu * u_diffusion * re2(S, D(meshScalingDel2), e, 1, 0);
            }
        }
        if (h_mom_eddy_visc4 > 0.0) {
#pragma omp parallel for schedule(static)
            for (long vx = 0; vx < nV; vx++)
                for (int k = 0; k < L; k++) {
                    CW(delsq_vorticity, vx, k) = 0.0;
                    for (int i = 0; i < 3; i++) {
                        int iEdge = iv2(S, I(edgesOnVertex), vx, 3, i);
                        double edge_sign = rv2(S, D(invAreaTriangle), vx, 1, 0) * re2(S, D(dcEdge), iEdge, 1, 0) *
                                           rv2(S, D(edgesOnVertex_sign), vx, 3, i);
                        CW(delsq_vorticity, vx, k) += edge_sign * re(S, delsq_u, iEdge, k);
                    }
                }
#pragma omp parallel for schedule(static)
            for (long c = 0; c < nC; c++) {
                int ne = ic2(S, nEdgesOnCell, c, 1, 0);
                for (int k = 0; k < L; k++) {
                    CW(delsq_divergence, c, k) = 0.0;
                    double r = rc2(S, invAreaCell, c, 1, 0);
                    for (int i = 0; i < ne; i++) {
                        int iEdge = ic2(S, edgesOnCell, c, 10, i);
                        double edge_sign = r * re2(S, dvEdge, iEdge, 1, 0) * rc2(S, eocs, c, 10, i);
                        CW(delsq_divergence, c, k) += edge_sign * re(S, delsq_u, iEdge, k);
                    }
                }
            }
#pragma omp parallel for schedule(static)
            for (long e = 0; e < nE; e++) {
                int cell1 = ie2(S, cellsOnEdge, e, 2, 0), cell2 = ie2(S, cellsOnEdge, e, 2, 1);
                int vertex1 = ie2(S, I(verticesOnEdge), e, 2, 0), vertex2 = ie2(S, I(verticesOnEdge), e, 2, 1);
                double u_mix_scale = re2(S, D(meshScalingDel4), e, 1, 0) * h_mom_eddy_visc4;
                double r_dc = u_mix_scale * config_del4u_div_factor * re2(S, invDcEdge, e, 1, 0);
                double r_dv = u_mix_scale * dmin(re2(S, D(invDvEdge), e, 1, 0), 4 * re2(S, invDcEdge, e, 1, 0));
                for (int k = 0; k < L; k++) {
                    double u_diffusion = CW(rho_edge, e, k) *
                                         ((rc(S, delsq_divergence, cell2, k) - rc(S, delsq_divergence, cell1, k)) * r_dc -
                                          (rv(S, delsq_vorticity, vertex2, k) - rv(S, delsq_vorticity, vertex1, k)) * r_dv);
                    CW(tend_u_euler, e, k) -= u_diffusion;
                }
            }
        }
    }
    if (config_rayleigh_damp_u) { /* :1152-1159 */
#pragma omp parallel for schedule(static)
        for (long e = 0; e < nE; e++)
            for (int k = 0; k < L; k++)
                if (k > L - config_number_rayleigh_damp_u_levels + 1)
                    CW(tend_u, e, k) -= CW(rho_edge, e, k) * CW(u, e, k) * rayleigh_damp_coef(S, k);
    }
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) /* :1161-1163 */
        for (int k = 0; k < L; k++) CW(tend_u, e, k) += CW(tend_u_euler, e, k) + CW(D(tend_ru_physics), e, k);

    /* -------- W section --------
     * tw: where the w tendency accumulates (the state w in the reference, Q8; tend_w in
     * mpas mode); wr: the w the tendency is computed from (the reference reads its own
     * partial tendency there, Q8/Q13; mpas mode the state w)                          */
    double* tw = mpas ? D(tend_w) : w;
    double* wr = mpas ? w : tw;
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) /* :1170-1172 */
        for (int k = 0; k < (mpas ? L + 1 : L); k++) CW(tw, c, k) = 0.0;
    double *ru_edge_w = D(ru_edge_w), *flux_arr = D(flux_arr);
    double *adv_coefs = D(adv_coefs), *adv_coefs_3rd = D(adv_coefs_3rd);
    int32_t *nAdv = I(nAdvCellsForEdge), *advCells = I(advCellsForEdge);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) { /* :1174-1197 (Q13) */
        int ne = ic2(S, nEdgesOnCell, c, 1, 0);
        for (int k = 0; k < L; k++) {
            for (int i = 0; i < ne; i++) {
                int iEdge = ic2(S, edgesOnCell, c, 10, i);
                if (k > 0) CW(ru_edge_w, c, k) = fzm[k] * re(S, ru, iEdge, k) + fzp[k] * re(S, ru, iEdge, k - 1);
                CW(flux_arr, c, k) = 0.0;
                int na = ie2(S, nAdv, iEdge, 1, 0);
                for (int j = 0; j < na; j++) {
                    int iAdvCell = ie2(S, advCells, iEdge, 15, j);
                    if (k > 0) {
                        double scalar_weight = re2(S, adv_coefs, iEdge, 15, j) +
                                               copysign(1.0, CW(ru_edge_w, c, k)) * re2(S, adv_coefs_3rd, iEdge, 15, j);
                        CW(flux_arr, c, k) += scalar_weight * rc(S, wr, iAdvCell, k);
                    }
                }
                /* mpas: the edge's flux enters before the next edge overwrites flux_arr */
                if (mpas && k > 0) CW(tw, c, k) -= rc2(S, eocs, c, 10, i) * CW(ru_edge_w, c, k) * CW(flux_arr, c, k);
            }
        }
    }
    if (!mpas) {
#pragma omp parallel for schedule(static)
        for (long c = 0; c < nC; c++) { /* :1199-1205 */
            int ne = ic2(S, nEdgesOnCell, c, 1, 0);
            for (int k = 0; k < L; k++)
                for (int i = 0; i < ne; i++)
                    if (k > 0) CW(w, c, k) -= rc2(S, eocs, c, 10, i) * CW(ru_edge_w, c, k) * CW(flux_arr, c, k);
        }
    }
    double *rho_zz = D(rho_zz), *uRZ = D(uReconstructZonal), *uRM = D(uReconstructMeridional);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) { /* :1208-1218 (mpas: added after the area scaling below) */
        double coslat = cos(rc2(S, D(lat), c, 1, 0));
        for (int k = 1; k < (mpas ? 1 : L); k++) {
            double a = fzm[k] * CW(uRZ, c, k) + fzp[k] * CW(uRZ, c, k - 1);
            double b = fzm[k] * CW(uRM, c, k) + fzp[k] * CW(uRM, c, k - 1);
            CW(w, c, k) += (CW(rho_zz, c, k) * fzm[k] + CW(rho_zz, c, k - 1) * fzp[k]) * ((a * a) + (b * b)) / r_earth +
                           2.0 * omega_c * coslat * (fzm[k] * CW(uRZ, c, k) + fzp[k] * CW(uRZ, c, k - 1)) *
                               (CW(rho_zz, c, k) * fzm[k] + CW(rho_zz, c, k - 1) * fzp[k]);
        }
    }
    double *delsq_w = D(delsq_w), *tend_w_euler = D(tend_w_euler);
    double *msd2 = D(meshScalingDel2), *msd4 = D(meshScalingDel4);
    if (rk_step == 0) { /* :1224-1274 */
#pragma omp parallel for schedule(static)
        for (long c = 0; c < nC; c++) {
            int ne = ic2(S, nEdgesOnCell, c, 1, 0);
            for (int k = 0; k < L; k++) {
                CW(delsq_w, c, k) = 0.0;
                CW(tend_w_euler, c, k) = 0.0;
                double r_areaCell = rc2(S, invAreaCell, c, 1, 0);
                for (int i = 0; i < ne; i++) {
                    int iEdge = ic2(S, edgesOnCell, c, 10, i);
                    double edge_sign = 0.5 * r_areaCell * rc2(S, eocs, c, 10, i) * re2(S, dvEdge, iEdge, 1, 0) * re2(S, invDcEdge, iEdge, 1, 0);
                    int cell1 = ie2(S, cellsOnEdge, iEdge, 2, 0), cell2 = ie2(S, cellsOnEdge, iEdge, 2, 1);
                    if (k > 0) {
                        double w_turb_flux = edge_sign * (re(S, rho_edge, iEdge, k) + re(S, rho_edge, iEdge, k - 1)) *
                                             (rc(S, wr, cell2, k) - rc(S, wr, cell1, k));
                        CW(delsq_w, c, k) += w_turb_flux;
                        w_turb_flux *= re2(S, msd2, iEdge, 1, 0) * 0.25 *
                                       (rc(S, kdiff, cell1, k) + rc(S, kdiff, cell2, k) + rc(S, kdiff, cell1, k - 1) + rc(S, kdiff, cell2, k - 1));
                        CW(tend_w_euler, c, k) += w_turb_flux;
                    }
                }
            }
        }
        if (h_mom_eddy_visc4 > 0.0) {
#pragma omp parallel for schedule(static)
            for (long c = 0; c < nC; c++) {
                int ne = ic2(S, nEdgesOnCell, c, 1, 0);
                double r_areaCell = h_mom_eddy_visc4 * rc2(S, invAreaCell, c, 1, 0);
                for (int k = 0; k < L; k++)
                    for (int i = 0; i < ne; i++) {
                        int iEdge = ic2(S, edgesOnCell, c, 10, i);
                        int cell1 = ie2(S, cellsOnEdge, iEdge, 2, 0), cell2 = ie2(S, cellsOnEdge, iEdge, 2, 1);
                        double edge_sign = re2(S, msd4, iEdge, 1, 0) * r_areaCell * re2(S, dvEdge, iEdge, 1, 0) *
                                           rc2(S, eocs, c, 10, i) * re2(S, invDcEdge, iEdge, 1, 0);
                        if (k > 0) CW(tend_w_euler, c, k) -= edge_sign * (rc(S, delsq_w, cell2, k) - rc(S, delsq_w, cell1, k));
                    }
            }
        }
    }
    double *wdwz = D(wdwz), *cqw = D(cqw);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        for (int k = 0; k < L; k++) { /* :1277-1287 */
            CW(wdwz, c, k) = 0.0;
            if (k == 1 || k == L - 1)  /* (nVertLevels = 1: level -1 reads 0, the level policy) */
                CW(wdwz, c, k) = 0.25 * (CW(rw, c, k) + rc(S, rw, c, k - 1)) * (CW(wr, c, k) + rc(S, wr, c, k - 1));
            if (k > 1 && k < L - 1)
                CW(wdwz, c, k) = flux3(CW(wr, c, k - 2), CW(wr, c, k - 1), CW(wr, c, k), rc(S, wr, c, k + 1),
                                       0.5 * (CW(rw, c, k) + CW(rw, c, k - 1)), 1.0);
        }
        const double coslat = cos(rc2(S, D(lat), c, 1, 0));
        for (int k = 0; k < L; k++) { /* :1289-1302 (Q14 literal) */
            /* mpas: wdwz(nVertLevels) = 0; tend_w = hflux invAreaCell + curvature - d(wdwz)/dz */
            const double wdwz_p = (mpas && k + 1 == L) ? 0.0 : rc(S, wdwz, c, k + 1);
            if (k > 0 && mpas) {
                double a = fzm[k] * CW(uRZ, c, k) + fzp[k] * CW(uRZ, c, k - 1);
                double b = fzm[k] * CW(uRM, c, k) + fzp[k] * CW(uRM, c, k - 1);
                double curv = (CW(rho_zz, c, k) * fzm[k] + CW(rho_zz, c, k - 1) * fzp[k]) * ((a * a) + (b * b)) / r_earth +
                              2.0 * omega_c * coslat * (fzm[k] * CW(uRZ, c, k) + fzp[k] * CW(uRZ, c, k - 1)) *
                                  (CW(rho_zz, c, k) * fzm[k] + CW(rho_zz, c, k - 1) * fzp[k]);
                CW(tw, c, k) = CW(tw, c, k) * rc2(S, invAreaCell, c, 1, 0) + curv - rdzu[k] * (wdwz_p - CW(wdwz, c, k));
            } else if (k > 0) {
                CW(w, c, k) *= rc2(S, invAreaCell, c, 1, 0) - rdzu[k] * (wdwz_p - CW(wdwz, c, k));
            }
            if (rk_step == 0 && k > 0)
                CW(tend_w_euler, c, k) -= CW(cqw, c, k) * (rdzu[k] * (CW(pressure_p, c, k) - CW(pressure_p, c, k - 1)) -
                                                           (fzm[k] * CW(dpdz, c, k) + fzp[k] * CW(dpdz, c, k - 1)));
        }
        for (int k = 1; k < L; k++) CW(tw, c, k) += CW(tend_w_euler, c, k); /* :1318-1322 */
    }

    /* -------- theta section -------- */
    double *tend_theta = D(tend_theta), *theta_m = D(theta_m), *ru_save = D(ru_save), *tms = D(theta_m_save);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) { /* :1328-1344 */
        int ne = ic2(S, nEdgesOnCell, c, 1, 0);
        for (int k = 0; k < L; k++) {
            CW(tend_theta, c, k) = 0.0;
            for (int i = 0; i < ne; i++) {
                int iEdge = ic2(S, edgesOnCell, c, 10, i);
                CW(flux_arr, c, k) = 0.0;
                int na = ie2(S, nAdv, iEdge, 1, 0);
                for (int j = 0; j < na; j++) {
                    int iAdvCell = ie2(S, advCells, iEdge, 15, j);
                    double scalar_weight = re2(S, adv_coefs, iEdge, 15, j) +
                                           copysign(1.0, re(S, ru, iEdge, k)) * re2(S, adv_coefs_3rd, iEdge, 15, j);
                    CW(flux_arr, c, k) += scalar_weight * rc(S, theta_m, iAdvCell, k);
                }
                CW(tend_theta, c, k) -= rc2(S, eocs, c, 10, i) * re(S, ru, iEdge, k) * CW(flux_arr, c, k);
            }
        }
    }
    if (rk_step > 0) { /* :1347-1360 */
#pragma omp parallel for schedule(static)
        for (long c = 0; c < nC; c++) {
            int ne = ic2(S, nEdgesOnCell, c, 1, 0);
            for (int k = 0; k < L; k++)
                for (int i = 0; i < ne; i++) {
                    int iEdge = ic2(S, edgesOnCell, c, 10, i);
                    int cell1 = ie2(S, cellsOnEdge, iEdge, 2, 0), cell2 = ie2(S, cellsOnEdge, iEdge, 2, 1);
                    double flux = rc2(S, eocs, c, 10, i) * re2(S, dvEdge, iEdge, 1, 0) *
                                  (re(S, ru_save, iEdge, k) - re(S, ru, iEdge, k)) * 0.5 *
                                  (rc(S, tms, cell2, k) + rc(S, tms, cell1, k));
                    CW(tend_theta, c, k) -= flux;
                }
        }
    }
    double *delsq_theta = D(delsq_theta), *tend_theta_euler = D(tend_theta_euler);
    if (rk_step == 0) { /* :1364-1401 */
#pragma omp parallel for schedule(static)
        for (long c = 0; c < nC; c++) {
            int ne = ic2(S, nEdgesOnCell, c, 1, 0);
            double r_areaCell = rc2(S, invAreaCell, c, 1, 0);
            for (int k = 0; k < L; k++) {
                CW(delsq_theta, c, k) = 0.0;
                CW(tend_theta_euler, c, k) = 0.0;
                for (int i = 0; i < ne; i++) {
                    int iEdge = ic2(S, edgesOnCell, c, 10, i);
                    double edge_sign = r_areaCell * rc2(S, eocs, c, 10, i) * re2(S, dvEdge, iEdge, 1, 0) * re2(S, invDcEdge, iEdge, 1, 0);
                    double pr_scale = prandtl_inv * re2(S, msd2, iEdge, 1, 0);
                    int cell1 = ie2(S, cellsOnEdge, iEdge, 2, 0), cell2 = ie2(S, cellsOnEdge, iEdge, 2, 1);
                    double theta_turb_flux = edge_sign * (rc(S, theta_m, cell2, k) - rc(S, theta_m, cell1, k)) * re(S, rho_edge, iEdge, k);
                    CW(delsq_theta, c, k) += theta_turb_flux;
                    theta_turb_flux *= 0.5 * (rc(S, kdiff, cell1, k) + rc(S, kdiff, cell2, k)) * pr_scale;
                    CW(tend_theta_euler, c, k) += theta_turb_flux;
                }
            }
        }
        if (h_theta_eddy_visc4 > 0.0) {
#pragma omp parallel for schedule(static)
            for (long c = 0; c < nC; c++) {
                int ne = ic2(S, nEdgesOnCell, c, 1, 0);
                double r_areaCell = h_theta_eddy_visc4 * prandtl_inv * rc2(S, invAreaCell, c, 1, 0);
                for (int k = 0; k < L; k++)
                    for (int i = 0; i < ne; i++) {
                        int iEdge = ic2(S, edgesOnCell, c, 10, i);
                        double edge_sign = re2(S, msd4, iEdge, 1, 0) * r_areaCell * re2(S, dvEdge, iEdge, 1, 0) *
                                           rc2(S, eocs, c, 10, i) * re2(S, invDcEdge, iEdge, 1, 0);
                        int cell1 = ie2(S, cellsOnEdge, iEdge, 2, 0), cell2 = ie2(S, cellsOnEdge, iEdge, 2, 1);
                        CW(tend_theta_euler, c, k) -= edge_sign * (rc(S, delsq_theta, cell2, k) - rc(S, delsq_theta, cell1, k));
                    }
            }
        }
    }
    double *wdtz = D(wdtz), *rw_save = D(rw_save);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        for (int k = 0; k < L; k++) { /* :1406-1420 (Q15 literal order) */
            CW(wdtz, c, k) = 0.0;
            if (mpas) { /* MPAS-A: 3rd-order flux of theta_m by rw plus the rtheta_pp redefinition term */
                if (k == 1)
                    CW(wdtz, c, k) = CW(rw, c, k) * (fzm[k] * CW(theta_m, c, k) + fzp[k] * CW(theta_m, c, k - 1)) +
                                     (CW(rw_save, c, k) - CW(rw, c, k)) * (fzm[k] * CW(tms, c, k) + fzp[k] * CW(tms, c, k - 1));
                if (k > 1 && k < L - 1)
                    CW(wdtz, c, k) = flux3(CW(theta_m, c, k - 2), CW(theta_m, c, k - 1), CW(theta_m, c, k),
                                           CW(theta_m, c, k + 1), CW(rw, c, k), 0.25) +
                                     (CW(rw_save, c, k) - CW(rw, c, k)) * (fzm[k] * CW(tms, c, k) + fzp[k] * CW(tms, c, k - 1));
                if (k == L - 1)  /* (nVertLevels = 1: level k - 1 = -1 reads 0, the level policy) */
                    CW(wdtz, c, k) = CW(rw_save, c, k) * (fzm[k] * CW(theta_m, c, k) + fzp[k] * rc(S, theta_m, c, k - 1));
                continue;
            }
            if (k > 0 && k < L - 1)
                CW(wdtz, c, k) = ((CW(rw_save, c, k) - CW(rw, c, k)) * (fzm[k] * CW(tms, c, k) + fzp[k] * CW(tms, c, k - 1)));
            if (k == 1) CW(wdtz, c, k) += CW(rw, c, k) * (fzm[k] * CW(theta_m, c, k) + fzp[k] * CW(theta_m, c, k - 1));
            if (k == L - 1) CW(wdtz, c, k) = CW(rw_save, c, k) * (fzm[k] * CW(tms, c, k) + fzp[k] * rc(S, tms, c, k - 1));
        }
        for (int k = 0; k < L; k++) { /* :1422-1427 */
            const double wdtz_p = (mpas && k + 1 == L) ? 0.0 : rc(S, wdtz, c, k + 1);
            if (mpas)
                CW(tend_theta, c, k) = CW(tend_theta, c, k) * rc2(S, invAreaCell, c, 1, 0) - rdzw[k] * (wdtz_p - CW(wdtz, c, k));
            else
                CW(tend_theta, c, k) *= rc2(S, invAreaCell, c, 1, 0) - rdzw[k] * (wdtz_p - CW(wdtz, c, k));
            CW(D(tend_rtheta_adv), c, k) = CW(tend_theta, c, k);
            CW(D(rthdynten), c, k) = CW(tend_theta, c, k) / CW(rho_zz, c, k);
            CW(tend_theta, c, k) += CW(rho_zz, c, k) * CW(D(rt_diabatic_tend), c, k);
        }
        for (int k = 0; k < L; k++) /* :1477-1479 */
            CW(tend_theta, c, k) += CW(tend_theta_euler, c, k) + CW(D(tend_rtheta_physics), c, k);
    }
}

void ora_atm_compute_dyn_tend_work(ora_state* S, int rk_step, double dt, int horiz_mixing, double config_mpas_cam_coef,
                                   int config_mix_full, int config_rayleigh_damp_u) {
    dyn_tend_impl(S, rk_step, dt, horiz_mixing, config_mpas_cam_coef, config_mix_full, config_rayleigh_damp_u, 0);
}

/* ===================== atm_set_smlstep_pert_variables_work, dynamics_tasks.rg:1503-1528
 * The iteration space "points of cpr" is the explicit mask cprMask[cell][k] (Q6);
 * "{iCell, iCell.y}" (:1522) is read as {iCell.x, iCell.y} (Q22).                    */
void ora_atm_set_smlstep_pert_variables_work(ora_state* S) {
    const int L = S->L, nC = S->nCells;
    double *w = D(w), *zz = D(zz), *u_tend = D(u_tend), *fzm = D(fzm), *fzp = D(fzp);
    uint8_t* mask = B(cprMask);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        for (int k = 0; k <= L; k++) {
            if (!mask[c * LV + k]) continue;
            if (ic2(S, I(bdyMaskCell), c, 1, 0) <= nRelaxZone) {
                for (int i = 0; i < ne; i++) {
                    int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
                    double flux = rc2(S, D(edgesOnCell_sign), c, 10, i) *
                                  (rz(S, fzm, k) * re(S, u_tend, iEdge, k) + rz(S, fzp, k) * re(S, u_tend, iEdge, k - 1));
                    CW(w, c, k) -= (rc3v(S, D(zb_cell), c, k, i) + copysign(1.0, re(S, u_tend, iEdge, k)) * rc3v(S, D(zb3_cell), c, k, i)) * flux;
                }
                CW(w, c, k) *= (rz(S, fzm, k) * CW(zz, c, k) + rz(S, fzp, k) * rc(S, zz, c, k - 1));
            }
        }
    }
}

/* ===================== atm_advance_acoustic_step_work, dynamics_tasks.rg:1546-1705
 * Q18 (ru_p update commented out), Q19 (rs/ts reset per point), Q20 (k-1 values read
 * after their update), Q21 (no back substitution) are all literal.
 * "{iCell, 0}" at :1638 is read as {iCell.x, 0} (Q22).                               */
void ora_atm_advance_acoustic_step_work(ora_state* S, double dts, int small_step) {
    const int L = S->L, nC = S->nCells;
    double epssm = config_epssm;
    double rcv = rgas / (CP - rgas);
    double c2 = CP * rcv;
    (void)c2;
    double resm = (1.0 - epssm) / (1.0 + epssm);
    double *rtheta_pp_old = D(rtheta_pp_old), *rtheta_pp = D(rtheta_pp), *rho_pp = D(rho_pp);
    double *wwAvg = D(wwAvg), *rw_p = D(rw_p);
    double *cofrz = D(cofrz), *rdzw = D(rdzw), *fzm = D(fzm), *fzp = D(fzp);
    double *zz = D(zz), *theta_m = D(theta_m), *ru_p = D(ru_p), *coftz = D(coftz), *w = D(w);
    /* :1581-1613: both edge-loop bodies are commented out in the reference */
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        double rs[128], ts[128];
        for (int k = 0; k < L; k++) /* :1615-1623 */
            CW(rtheta_pp_old, c, k) = (small_step == 0) ? 0 : CW(rtheta_pp, c, k);
        for (int k = 0; k <= L; k++) /* :1625-1630 */
            if (small_step == 0) {
                CW(wwAvg, c, k) = 0;
                CW(rw_p, c, k) = 0;
            }
        for (int k = 0; k < L; k++) { /* :1632-1704 */
            if (small_step == 0) {
                CW(rho_pp, c, k) = 0;
                CW(rtheta_pp, c, k) = 0;
            }
            if (rc2(S, D(specZoneMaskCell), c, 1, 0) == 0.0) {
                for (int i = 0; i < L; i++) {
                    ts[i] = 0;
                    rs[i] = 0;
                }
                for (int i = 0; i < ne; i++) {
                    int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
                    int cell1 = ie2(S, I(cellsOnEdge), iEdge, 2, 0), cell2 = ie2(S, I(cellsOnEdge), iEdge, 2, 1);
                    double flux = rc2(S, D(edgesOnCellSign), c, 10, i) * dts * re2(S, D(dvEdge), iEdge, 1, 0) *
                                  re(S, ru_p, iEdge, k) * rc2(S, D(invAreaCell), c, 1, 0);
                    rs[k] -= flux;
                    ts[k] -= flux * 0.5 * (rc(S, theta_m, cell2, k) + rc(S, theta_m, cell1, k));
                }
                rs[k] = CW(rho_pp, c, k) + dts * CW(D(tend_rho), c, k) + rs[k] -
                        cofrz[k] * resm * (rc(S, rw_p, c, k + 1) - CW(rw_p, c, k));
                ts[k] = CW(rtheta_pp, c, k) + dts * CW(theta_m, c, k) + ts[k] -
                        resm * rdzw[k] * (rc(S, coftz, c, k + 1) * rc(S, rw_p, c, k + 1) - CW(coftz, c, k) * CW(rw_p, c, k));
                if (k > 0) {
                    double tsm = ts[k - 1], rsm = rs[k - 1];
                    CW(wwAvg, c, k) += 0.5 * (1.0 - epssm) * CW(rw_p, c, k);
                    CW(rw_p, c, k) += dts * CW(w, c, k) -
                                      CW(D(cofwz), c, k) * ((CW(zz, c, k) * ts[k] - CW(zz, c, k - 1) * tsm) +
                                                            resm * (CW(zz, c, k) * CW(rtheta_pp, c, k) - CW(zz, c, k - 1) * CW(rtheta_pp, c, k - 1))) -
                                      CW(D(cofwr), c, k) * ((rs[k] + rsm) + resm * (CW(rho_pp, c, k) + CW(rho_pp, c, k - 1))) +
                                      CW(D(cofwt), c, k) * (ts[k] + resm * CW(rtheta_pp, c, k)) +
                                      CW(D(cofwt), c, k - 1) * (tsm + resm * CW(rtheta_pp, c, k - 1));
                    CW(rw_p, c, k) -= CW(D(a_tri), c, k) * CW(rw_p, c, k - 1);
                    CW(rw_p, c, k) *= CW(D(alpha_tri), c, k);
                }
                if (k > 0) { /* :1681-1690 */
                    CW(rw_p, c, k) += (CW(D(rw_save), c, k) - CW(D(rw), c, k)) -
                                      dts * CW(D(dss), c, k) * (fzm[k] * CW(zz, c, k) + fzp[k] * CW(zz, c, k - 1)) *
                                          (fzm[k] * CW(D(rho_zz), c, k) + fzp[k] * CW(D(rho_zz), c, k - 1)) * CW(w, c, k);
                    CW(rw_p, c, k) /= (1.0 + dts * CW(D(dss), c, k));
                    CW(rw_p, c, k) -= (CW(D(rw_save), c, k) - CW(D(rw), c, k));
                    CW(wwAvg, c, k) += 0.5 * (1.0 + epssm) * CW(rw_p, c, k);
                }
                CW(rho_pp, c, k) = rs[k] - cofrz[k] * (rc(S, rw_p, c, k + 1) - CW(rw_p, c, k));
                CW(rtheta_pp, c, k) = ts[k] - rdzw[k] * (rc(S, coftz, c, k + 1) * rc(S, rw_p, c, k + 1) - CW(coftz, c, k) * CW(rw_p, c, k));
            } else { /* :1698-1703 */
                CW(rho_pp, c, k) = CW(rho_pp, c, k) + dts * CW(D(tend_rho), c, k);
                CW(rtheta_pp, c, k) = CW(rtheta_pp, c, k) + dts * CW(theta_m, c, k);
                CW(rw_p, c, k) = CW(rw_p, c, k) + dts * CW(w, c, k);
                CW(wwAvg, c, k) = CW(wwAvg, c, k) + 0.5 * (1.0 + epssm) * CW(rw_p, c, k);
            }
        }
    }
}

/* ===================== atm_divergence_damping_3d, dynamics_tasks.rg:1726-1763
 * cellOne/cellTwo are the rects built from cellsOnEdge (mesh_loading.rg:422-425);
 * isShared is read at level 0 of the whole cell field (Q6).                          */
void ora_atm_divergence_damping_3d(ora_state* S, double dts) {
    const int L = S->L;
    double smdiv = config_smdiv;
    double rdts = 1.0 / dts;
    double coef_divdamp = 2.0 * smdiv * config_len_disp * rdts;
    double *ru_p = D(ru_p), *rtp = D(rtheta_pp), *rtpo = D(rtheta_pp_old), *tm = D(theta_m);
#pragma omp parallel for schedule(static)
    for (long e = 0; e < S->nEdges; e++) {
        int cell1 = ie2(S, I(cellsOnEdge), e, 2, 0), cell2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        if (!(ic2(S, I(isShared), cell1, 1, 0) && ic2(S, I(isShared), cell2, 1, 0))) {
            for (int k = 0; k < L; k++) {
                double divCell1 = -(rc(S, rtp, cell1, k) - rc(S, rtpo, cell1, k));
                double divCell2 = -(rc(S, rtp, cell2, k) - rc(S, rtpo, cell2, k));
                CW(ru_p, e, k) += coef_divdamp * (divCell2 - divCell1) * (1.0 - re2(S, D(specZoneMaskEdge), e, 1, 0)) /
                                  (rc(S, tm, cell1, k) + rc(S, tm, cell2, k));
            }
        }
    }
}

/* ===================== atm_rk_dynamics_substep_finish, dynamics_tasks.rg:1951-2007 */
void ora_atm_rk_dynamics_substep_finish(ora_state* S, int dynamics_substep, int dynamics_split) {
    const int L = S->L;
    double inv_dynamics_split = 1.0 / (double)dynamics_split;
    if (dynamics_substep < dynamics_split) {
#pragma omp parallel for schedule(static)
        for (long e = 0; e < S->nEdges; e++)
            for (int k = 0; k < L; k++) {
                CW(D(ru_save), e, k) = CW(D(ru), e, k);
                CW(D(u), e, k) = CW(D(u_2), e, k);
            }
#pragma omp parallel for schedule(static)
        for (long c = 0; c < S->nCells; c++)
            for (int k = 0; k < L; k++) {
                CW(D(rw_save), c, k) = CW(D(rw), c, k);
                CW(D(rtheta_p_save), c, k) = CW(D(rtheta_p), c, k);
                CW(D(rho_p_save), c, k) = CW(D(rho_p), c, k);
                CW(D(w), c, k) = CW(D(w_2), c, k);
                CW(D(theta_m), c, k) = CW(D(theta_m_2), c, k);
                CW(D(rho_zz), c, k) = CW(D(rho_zz_2), c, k);
            }
    }
#pragma omp parallel for schedule(static)
    for (long e = 0; e < S->nEdges; e++)
        for (int k = 0; k < L; k++) {
            if (dynamics_substep == 1) CW(D(ruAvg_split), e, k) = CW(D(ruAvg), e, k);
            else CW(D(ruAvg_split), e, k) = CW(D(ruAvg), e, k) + CW(D(ruAvg_split), e, k);
            if (dynamics_substep == dynamics_split) CW(D(ruAvg), e, k) = CW(D(ruAvg_split), e, k) * inv_dynamics_split;
        }
#pragma omp parallel for schedule(static)
    for (long c = 0; c < S->nCells; c++)
        for (int k = 0; k < L; k++) {
            if (dynamics_substep == 1) CW(D(wwAvg_split), c, k) = CW(D(wwAvg), c, k);
            else CW(D(wwAvg_split), c, k) = CW(D(wwAvg), c, k) + CW(D(wwAvg_split), c, k);
            if (dynamics_substep == dynamics_split) {
                CW(D(wwAvg), c, k) = CW(D(wwAvg_split), c, k) * inv_dynamics_split;
                CW(D(rho_zz), c, k) = CW(D(rho_zz_old_split), c, k);
            }
        }
}


/* ===================== atm_recover_large_step_variables_work, dynamics_tasks.rg:1766-1872
 * Not called by atm_srk3 (Q7, rk_timestep.rg:460); restated for the operator API.
 * Literal: Q24 (ru = ru_save * ru_p, flux2 = a * (b), the exner exponent placement);
 * the level-0 flux term of the w recovery is added at EVERY level iteration of the cell
 * (:1851-1854 write cr[{iCell.x, 0}].w inside the loop over all points), i.e. nVertLevels
 * times; "{iCell, 0}" (:1856) is {iCell.x, 0} (Q22).  Every loop covers levels
 * 0..nVertLevels-1.  The zero slot of rho_zz (the "garbage cell", :1790-1792) is set to
 * 1.0 at those levels.                                                                  */
void ora_atm_recover_large_step_variables_work(ora_state* S, int ns, int rk_step, double dt) {
    const int L = S->L, nC = S->nCells, nE = S->nEdges;
    const double rcv = rgas / (CP - rgas);
    const int p0 = 100000;
    double *rho_zz = D(rho_zz), *w = D(w), *ru = D(ru);
    for (int k = 0; k < L; k++) CW(rho_zz, nC, k) = 1.0;
    const double invNs = 1 / (double)ns;
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++)
        for (int k = 0; k < L; k++) {
            CW(D(rho_p), c, k) = CW(D(rho_p_save), c, k) + CW(D(rho_pp), c, k);
            CW(rho_zz, c, k) = CW(D(rho_p), c, k) + CW(D(rho_base), c, k);
            CW(w, c, k) = 0.0;
            CW(D(wwAvg), c, k) *= invNs;
            CW(D(wwAvg), c, k) += CW(D(rw_save), c, k);
            CW(D(rw), c, k) = CW(D(rw_save), c, k) + CW(D(rw_p), c, k);
            CW(w, c, k) = CW(D(rw), c, k) / (rz(S, D(fzm), k) * CW(D(zz), c, k) + rz(S, D(fzp), k) * rc(S, D(zz), c, k - 1));
            if (k == L) CW(w, c, k) = 0.0;
            if (rk_step == 2) {
                CW(D(rtheta_p), c, k) = CW(D(rtheta_p_save), c, k) + CW(D(rtheta_pp), c, k) -
                                        dt * CW(rho_zz, c, k) * CW(D(rt_diabatic_tend), c, k);
                CW(D(theta_m), c, k) = (CW(D(rtheta_p), c, k) + CW(D(rtheta_base), c, k)) / CW(rho_zz, c, k);
                CW(D(exner), c, k) = CW(D(zz), c, k) * (rgas / p0) * pow((CW(D(rtheta_p), c, k) + CW(D(rtheta_base), c, k)), rcv);
                CW(D(pressure_p), c, k) = CW(D(zz), c, k) * rgas *
                                          (CW(D(exner), c, k) * CW(D(rtheta_p), c, k) +
                                           CW(D(rtheta_base), c, k) * (CW(D(exner), c, k) - CW(D(exner_base), c, k)));
            } else {
                CW(D(rtheta_p), c, k) = CW(D(rtheta_p_save), c, k) + CW(D(rtheta_pp), c, k);
                CW(D(theta_m), c, k) = (CW(D(rtheta_p), c, k) + CW(D(rtheta_base), c, k)) / CW(rho_zz, c, k);
            }
        }
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) {
        int cell1 = ie2(S, I(cellsOnEdge), e, 2, 0), cell2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        for (int k = 0; k < L; k++) {
            CW(D(ruAvg), e, k) *= invNs;
            CW(D(ruAvg), e, k) += CW(D(ru_save), e, k);
            CW(ru, e, k) = CW(D(ru_save), e, k) * CW(D(ru_p), e, k);
            CW(D(u), e, k) = 2 * CW(ru, e, k) / (rc(S, rho_zz, cell1, k) + rc(S, rho_zz, cell2, k));
        }
    }
    const double cf1 = rz(S, D(cf1), 0), cf2 = rz(S, D(cf2), 0), cf3 = rz(S, D(cf3), 0);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        if (ic2(S, I(bdyMaskCell), c, 1, 0) > nRelaxZone) continue;
        const int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        for (int k = 0; k < L; k++)
            for (int i = 0; i < ne; i++) {
                int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
                double sg = rc2(S, D(edgesOnCell_sign), c, 10, i);
                double flux = (cf1 * re(S, ru, iEdge, 0) + cf2 * re(S, ru, iEdge, 1) + cf3 * re(S, ru, iEdge, 2));
                CW(w, c, 0) += sg * (rc3v(S, D(zb_cell), c, 0, i) + copysign(1.0, flux) * rc3v(S, D(zb3_cell), c, 0, i)) * flux;
                double flux2 = rz(S, D(fzm), k) * re(S, ru, iEdge, k) * (rz(S, D(fzp), k) * re(S, ru, iEdge, k - 1));
                CW(w, c, k) += sg * (rc3v(S, D(zb_cell), c, k, i) + copysign(1.0, flux2) * rc3v(S, D(zb3_cell), c, k, i)) * flux2;
            }
        for (int k = 0; k < L; k++) {
            if (k == 0) CW(w, c, 0) /= (cf1 * CW(rho_zz, c, 0) + cf2 * rc(S, rho_zz, c, 1) + cf3 * rc(S, rho_zz, c, 2));
            if (k > 0) CW(w, c, k) /= (rz(S, D(fzm), k) * CW(rho_zz, c, k) + rz(S, D(fzp), k) * CW(rho_zz, c, k - 1));
        }
    }
}

/* ===================== atm_compute_output_diagnostics, dynamics_tasks.rg:729-746 (the
 * theta statement :740 is commented out in the reference; theta is left as it is)   */
void ora_atm_compute_output_diagnostics(ora_state* S) {
    const int L = S->L, nC = S->nCells;
    double *rho = D(rho), *pressure = D(pressure);
    const double *rho_zz = D(rho_zz), *zz = D(zz), *pb = D(pressure_base), *pp = D(pressure_p);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++)
        for (int k = 0; k < L; k++) {
            CW(rho, c, k) = CW(rho_zz, c, k) * CW(zz, c, k);
            CW(pressure, c, k) = CW(pb, c, k) + CW(pp, c, k);
        }
}

/* ===================== mpas_reconstruct_2d, dynamics_tasks.rg:1893-1948 (levels
 * 0..nVertLevels-1 of every cell; includeHalos does not change the range there).   */
void ora_mpas_reconstruct_2d(ora_state* S, int includeHalos, int on_a_sphere) {
    const int L = S->L, nC = S->nCells;
    (void)includeHalos;
    double *X = D(uReconstructX), *Y = D(uReconstructY), *Z = D(uReconstructZ), *u = D(u);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        const int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        for (int k = 0; k < L; k++) {
            CW(X, c, k) = 0.0;
            CW(Y, c, k) = 0.0;
            CW(Z, c, k) = 0.0;
        }
        for (int k = 0; k < L; k++)
            for (int i = 0; i < ne; i++) {
                int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
                CW(X, c, k) += rc2(S, D(coeffs_reconstruct), c, 30, i * 3 + 0) * re(S, u, iEdge, k);
                CW(Y, c, k) += rc2(S, D(coeffs_reconstruct), c, 30, i * 3 + 1) * re(S, u, iEdge, k);
                CW(Z, c, k) += rc2(S, D(coeffs_reconstruct), c, 30, i * 3 + 2) * re(S, u, iEdge, k);
            }
        if (on_a_sphere) {
            double clat = cos(rc2(S, D(lat), c, 1, 0)), slat = sin(rc2(S, D(lat), c, 1, 0));
            double clon = cos(rc2(S, D(lon), c, 1, 0)), slon = sin(rc2(S, D(lon), c, 1, 0));
            for (int k = 0; k < L; k++) {
                CW(D(uReconstructZonal), c, k) = -CW(X, c, k) * slon + CW(Y, c, k) * clon;
                CW(D(uReconstructMeridional), c, k) = -(CW(X, c, k) * clon + CW(Y, c, k) * slon) * slat + CW(Z, c, k) * clat;
            }
        } else {
            for (int k = 0; k < L; k++) {
                CW(D(uReconstructZonal), c, k) = CW(X, c, k);
                CW(D(uReconstructMeridional), c, k) = CW(Y, c, k);
            }
        }
    }
}

/* ===================== summarize_timestep, rk_timestep.rg:29-359: the values the
 * reference prints.  out[0..24]: five records {value, index, k, lat_deg, lon_deg} for
 * min w, max w, min u, max u, max wind speed (first point in cell-major, level-minor
 * order; comparisons strict against the 1e20 / -1e20 start; the lat/lon of the max
 * records are read at level k, i.e. 0.0 for k > 0 (2-D data at level > 0, Q2)); out[25],
 * out[26]: NaN seen in w, u; out[27..30]: the fold min/max of w and of u from 0.0
 * (regentlib min/max, a < b ? a : b).  detailed / global_vel select the two blocks
 * (the reference tests constants.config_print_detailed_minmax_vel for the first and its
 * argument for the second; both are false on the path, rk_timestep.rg:492).         */
static void ora_rec(double* r, double val, long idx, long k, double lat, double lon) {
    const double pi_const = 2.0 * asin(1.0);
    r[0] = val;
    r[1] = (double)idx;
    r[2] = (double)k;
    double la = lat * (180.0 / pi_const), lo = lon * (180.0 / pi_const);
    if (lo > 180.0) lo -= 360.0;
    r[3] = la;
    r[4] = lo;
}
void ora_summarize_timestep(ora_state* S, int detailed, int global_vel, double* out) {
    const int L = S->L, nC = S->nCells, nE = S->nEdges;
    double *w = D(w), *u = D(u), *v = D(v), *latc = D(lat), *lonc = D(lon), *late = D(latEdge), *lone = D(lonEdge);
    for (int i = 0; i < 31; i++) out[i] = 0.0;
    if (detailed) {
        double mn = 1.0e20, mx = -1.0e20, la = 0, lo = 0, la2 = 0, lo2 = 0;
        long im = -1, km = -1, ix = -1, kx = -1;
        for (long c = 0; c < nC; c++)
            for (int k = 0; k < L; k++) {
                double x = CW(w, c, k);
                if (x < mn) { mn = x; im = c; km = k; la = latc[c]; lo = lonc[c]; }
            }
        for (long c = 0; c < nC; c++)
            for (int k = 0; k < L; k++) {
                double x = CW(w, c, k);
                if (x > mx) { mx = x; ix = c; kx = k; la2 = k == 0 ? latc[c] : 0.0; lo2 = k == 0 ? lonc[c] : 0.0; }
            }
        ora_rec(out + 0, mn, im, km, la, lo);
        ora_rec(out + 5, mx, ix, kx, la2, lo2);
        mn = 1.0e20; mx = -1.0e20; im = km = ix = kx = -1; la = lo = la2 = lo2 = 0;
        for (long e = 0; e < nE; e++)
            for (int k = 0; k < L; k++) {
                double x = CW(u, e, k);
                if (x < mn) { mn = x; im = e; km = k; la = late[e]; lo = lone[e]; }
            }
        for (long e = 0; e < nE; e++)
            for (int k = 0; k < L; k++) {
                double x = CW(u, e, k);
                if (x > mx) { mx = x; ix = e; kx = k; la2 = k == 0 ? late[e] : 0.0; lo2 = k == 0 ? lone[e] : 0.0; }
            }
        ora_rec(out + 10, mn, im, km, la, lo);
        ora_rec(out + 15, mx, ix, kx, la2, lo2);
        mx = -1.0e20; ix = kx = -1; la = lo = 0;
        for (long e = 0; e < nE; e++)
            for (int k = 0; k < L; k++) {
                double spd = sqrt(CW(u, e, k) * CW(u, e, k) + CW(v, e, k) * CW(v, e, k));
                if (spd > mx) { mx = spd; ix = e; kx = k; la = late[e]; lo = lone[e]; }
            }
        ora_rec(out + 20, mx, ix, kx, la, lo);
        for (long c = 0; c < nC; c++)
            for (int k = 0; k < L; k++)
                if (isnan(CW(w, c, k))) out[25] = 1.0;
        for (long e = 0; e < nE; e++)
            for (int k = 0; k < L; k++)
                if (isnan(CW(u, e, k))) out[26] = 1.0;
    }
    if (global_vel) {
        double mn = 0.0, mx = 0.0;
        for (long c = 0; c < nC; c++)
            for (int k = 0; k < L; k++) {
                mn = dmin(mn, CW(w, c, k));
                mx = dmax(mx, CW(w, c, k));
            }
        out[27] = mn;
        out[28] = mx;
        mn = 0.0;
        mx = 0.0;
        for (long e = 0; e < nE; e++)
            for (int k = 0; k < L; k++) {
                mn = dmin(mn, CW(u, e, k));
                mx = dmax(mx, CW(u, e, k));
            }
        out[29] = mn;
        out[30] = mx;
    }
}

/* ===================== atm_srk3, rk_timestep.rg:361-500
 * schedule 0: the reference's own driver, with Q4 (rk_sub_timestep[rk_step] truncated
 *             into dyn_tend's int rk_step) and Q5 (n+1 acoustic substeps);
 * schedule 1: dyn_tend gets rk_step = 0,1,2 (the MPAS schedule, SURVEY §8.5 bench).   */
void ora_atm_srk3(ora_state* S, double dt, int schedule) {
    int number_of_sub_steps = 2;
    int dynamics_split = 1;
    double dt_dynamics = dt;
    double rk_sub_timestep[3] = {dt_dynamics / 3, dt_dynamics / number_of_sub_steps, dt_dynamics / number_of_sub_steps};
    int number_sub_steps[3];
    number_sub_steps[0] = (number_of_sub_steps / 2 > 1) ? number_of_sub_steps / 2 : 1;
    number_sub_steps[1] = number_sub_steps[0];
    number_sub_steps[2] = number_of_sub_steps;
    ora_atm_rk_integration_setup(S);
    ora_atm_compute_moist_coefficients(S);
    ora_atm_compute_vert_imp_coefs(S, rk_sub_timestep[0]);
    for (int rk_step = 0; rk_step < 3; rk_step++) {
        if (rk_step == 1) ora_atm_compute_vert_imp_coefs(S, rk_sub_timestep[rk_step]);
        int dyn_rk = schedule == 0 ? (int)rk_sub_timestep[rk_step] : rk_step;
        ora_atm_compute_dyn_tend_work(S, dyn_rk, dt, 0, 0.0, 0, 0);
        ora_atm_set_smlstep_pert_variables_work(S);
        for (int small_step = 0; small_step < number_sub_steps[rk_step] + 1; small_step++) {
            ora_atm_advance_acoustic_step_work(S, rk_sub_timestep[rk_step], small_step);
            ora_atm_divergence_damping_3d(S, rk_sub_timestep[rk_step]);
        }
        ora_atm_compute_solve_diagnostics(S, 0, rk_step);
    }
    ora_atm_rk_dynamics_substep_finish(S, 1, dynamics_split);
}

/* ===================== one-time tasks of atm_core_init (atm_core.rg:22-42) on the device
 * atm_compute_damping_coefs, dynamics_tasks.rg:274-300: dss of the upper damping layer
 * (pow(x, 2.0) evaluated as x * x, the policy of DESIGN.md §2) */
void ora_atm_compute_damping_coefs(ora_state* S, double config_zd, double config_xnutr) {
    const int L = S->L, nC = S->nCells;
    const double pii = acos(-1.0), dx_scale_power = 1.0;
    double *dss = D(dss), *zgrid = D(zgrid);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++)
        for (int k = 0; k < L; k++) {
            CW(dss, c, k) = 0.0;
            const double zt = CW(zgrid, c, L);
            const double z = 0.5 * (CW(zgrid, c, k) + CW(zgrid, c, k + 1));
            if (z > config_zd) {
                const double sn = sin(0.5 * pii * (z - config_zd) / (zt - config_zd));
                CW(dss, c, k) = config_xnutr * (sn * sn);
                CW(dss, c, k) /= pow(rc2(S, D(meshDensity), c, 1, 0), (0.25 * dx_scale_power));
            }
        }
}

/* ---- the mesh tasks of atm_core_init (atm_core.rg:22-39) ----
 * Ids are compared as the arrays hold them (raw); reads through an id follow the Q1
 * policy (ic2/ie2/iv2: outside [0, n] reads 0).  Out-of-range list writes the reference
 * leaves undefined are bounded: the cell list of atm_adv_coef_compression is capped at
 * maxEdges - 1 in both of its loops (the reference caps only the second, :175) and
 * deriv_two(iCell * FIFTEEN + s) past the array's 30 entries reads 0.0. */
#define MAXEDGES 10
#define VERTEXDEGREE 3

/* atm_compute_signs, dynamics_tasks.rg:46-130.  zb_cell / zb3_cell copy er.zb / er.zb3
 * (:88-110), which init_atm_case_jw writes (init_atm_cases.rg:657-660); the state keeps no
 * er.zb, the host that builds the initial state uploads the copy, so they stay as given.  kiteForCell keeps its value when no cellsOnVertex(j),
 * j = 1..vertexDegree-1, matches (the loop breaks only on a match). */
void ora_atm_compute_signs(ora_state* S) {
    const int nC = S->nCells, nE = S->nEdges, nV = S->nVertices, L = S->L;
    int32_t *eov = I(edgesOnVertex), *eoc = I(edgesOnCell), *voc = I(verticesOnCell), *kite = I(kiteForCell);
    double *eovs = D(edgesOnVertexSign), *eocs = D(edgesOnCellSign);
#pragma omp parallel for schedule(static)
    for (long v = 0; v < nV; v++)
        for (int i = 0; i < VERTEXDEGREE; i++) {
            const int e = eov[v * VERTEXDEGREE + i];
            if (e <= nE) eovs[v * VERTEXDEGREE + i] = (v == ie2(S, I(verticesOnEdge), e, 2, 1)) ? 1.0 : -1.0;
            else eovs[v * VERTEXDEGREE + i] = 0.0;
        }
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        if (ne > MAXEDGES) ne = MAXEDGES;
        for (int i = 0; i < ne; i++) {
            const int e = eoc[c * MAXEDGES + i];
            if (e <= nE) eocs[c * MAXEDGES + i] = (c == ie2(S, I(cellsOnEdge), e, 2, 0)) ? 1.0 : -1.0;
            else eocs[c * MAXEDGES + i] = 0.0;
        }
        for (int i = 0; i < ne; i++) {
            const int iVtx = voc[c * MAXEDGES + i];
            if (iVtx <= nV) {
                for (int j = 1; j < VERTEXDEGREE; j++)
                    if (c == iv2(S, I(cellsOnVertex), iVtx, VERTEXDEGREE, j)) {
                        kite[c * MAXEDGES + i] = j;
                        break;
                    }
            } else {
                kite[c * MAXEDGES + i] = 1;
            }
        }
    }
}

/* atm_adv_coef_compression, dynamics_tasks.rg:133-269 (nAdvCellsForEdge = n is the index
 * of the list's last cell, so the coefficient loops over j < n never see it; pow(dc, 2)
 * as dc * dc) */
void ora_atm_adv_coef_compression(ora_state* S) {
    const int nC = S->nCells, nE = S->nEdges;
    int32_t *nadv = I(nAdvCellsForEdge), *advc = I(advCellsForEdge);
    double *ac = D(adv_coefs), *ac3 = D(adv_coefs_3rd), *d2 = D(deriv_two);
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) {
        nadv[e] = 0;
        const int cell1 = ie2(S, I(cellsOnEdge), e, 2, 0), cell2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        if (!(cell1 <= nC || cell2 <= nC)) continue;
        int cl[MAXEDGES];
        cl[0] = cell1;
        cl[1] = cell2;
        int n = 1;
        const int ne1 = ic2(S, I(nEdgesOnCell), cell1, 1, 0), ne2 = ic2(S, I(nEdgesOnCell), cell2, 1, 0);
        for (int i = 0; i < ne1; i++) {
            const int cc = ic2(S, I(cellsOnCell), cell1, MAXEDGES, i);
            if (cc != cell2 && n < MAXEDGES - 1) cl[++n] = cc;
        }
        for (int ic = 0; ic < ne2; ic++) {
            const int cc = ic2(S, I(cellsOnCell), cell2, MAXEDGES, ic);
            int add = 1;
            for (int i = 0; i < n; i++)
                if (cl[i] == cc) add = 0;
            if (add && n < MAXEDGES - 1) cl[++n] = cc;
        }
        nadv[e] = n;
        for (int i = 0; i < n; i++) advc[e * 15 + i] = cl[i];
        double* a = ac + e * 15;
        double* a3 = ac3 + e * 15;
        for (int j = 0; j < 15; j++) a[j] = a3[j] = 0.0;
        const double* dt2 = d2 + e * 30;
#define D2(idx) ((idx) < 30 ? dt2[(idx)] : 0.0)
        int j_in = 0;
        for (int j = 0; j < n; j++)
            if (cl[j] == cell1) j_in = j;
        a[j_in] += dt2[0];
        a3[j_in] += dt2[0];
        for (int ic = 0; ic < ne1; ic++) {
            j_in = 0;
            for (int j = 0; j < n; j++)
                if (cl[j] == ic2(S, I(cellsOnCell), cell1, MAXEDGES, ic)) j_in = j;
            a[j_in] += D2(ic * 15 + 0);
            a3[j_in] += D2(ic * 15 + 0);
        }
        j_in = 0;
        for (int j = 0; j < n; j++)
            if (cl[j] == cell2) j_in = j;
        a[j_in] += dt2[1];
        a3[j_in] += dt2[1];
        for (int ic = 0; ic < ne2; ic++) {
            j_in = 0;
            for (int j = 0; j < n; j++)
                if (cl[j] == ic2(S, I(cellsOnCell), cell2, MAXEDGES, ic)) j_in = j;
            a[j_in] += D2(ic * 15 + 1);
            a3[j_in] += D2(ic * 15 + 1);
        }
#undef D2
        const double dc = re2(S, D(dcEdge), e, 1, 0), dv = re2(S, D(dvEdge), e, 1, 0);
        for (int j = 0; j < n; j++) {
            a[j] = -1.0 * (dc * dc) * a[j] / 12;
            a3[j] = -1.0 * (dc * dc) * a3[j] / 12;
        }
        j_in = 0;
        for (int j = 0; j < n; j++)
            if (cl[j] == cell1) j_in = j;
        a[j_in] += 0.5;
        j_in = 0;
        for (int j = 0; j < n; j++)
            if (cl[j] == cell2) j_in = j;
        a[j_in] += 0.5;
        for (int j = 0; j < n; j++) {
            a[j] *= dv;
            a3[j] *= dv;
        }
    }
}

/* atm_couple_coef_3rd_order, dynamics_tasks.rg:303-325 (zb3_cell at level 0 only) */
void ora_atm_couple_coef_3rd_order(ora_state* S, double config_coef_3rd_order) {
    const int nC = S->nCells, nE = S->nEdges;
    double *ac3 = D(adv_coefs_3rd), *zb3 = D(zb3_cell);
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++)
        for (int i = 0; i < 15; i++) ac3[e * 15 + i] *= config_coef_3rd_order;
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++)
        for (int j = 0; j < MAXEDGES; j++) zb3[(c * LV + 0) * MAXEDGES + j] *= config_coef_3rd_order;
}

/* atm_compute_mesh_scaling, dynamics_tasks.rg:595-646: the del2 / del4 scaling of each
 * edge (cellOne / cellTwo = the cells of cellsOnEdge(0/1), data_structures.rg:486-487).
 * The regional-relaxation factors it also writes are read by no task of the path. */
void ora_atm_compute_mesh_scaling(ora_state* S, int config_h_ScaleWithMesh) {
    const int nE = S->nEdges;
    double *d2 = D(meshScalingDel2), *d4 = D(meshScalingDel4), *md = D(meshDensity);
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) {
        d2[e] = 1.0;
        d4[e] = 1.0;
        if (config_h_ScaleWithMesh) {
            const int c1 = ie2(S, I(cellsOnEdge), e, 2, 0), c2 = ie2(S, I(cellsOnEdge), e, 2, 1);
            const double avg = (rc2(S, md, c1, 1, 0) + rc2(S, md, c2, 1, 0)) / 2.0;
            d2[e] = 1.0 / pow(avg, 0.25);
            d4[e] = 1.0 / pow(avg, 0.75);
        }
    }
}

/* atm_init_coupled_diagnostics, dynamics_tasks.rg:651-726: rho_zz /= zz, ru from u, rw
 * from w and the slope flux of ru, then rho_p, rtheta_base/_p, exner(_base), pressure */
void ora_atm_init_coupled_diagnostics(ora_state* S) {
    const int L = S->L, nC = S->nCells, nE = S->nEdges;
    const double rgas_ = rgas, rcv = rgas / (CP - rgas), p0 = 100000;
    double *rho_zz = D(rho_zz), *zz = D(zz), *ru = D(ru), *rw = D(rw), *fzm = D(fzm), *fzp = D(fzp);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++)
        for (int k = 0; k < L; k++) CW(rho_zz, c, k) /= CW(zz, c, k);
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) {
        const int cell1 = ie2(S, I(cellsOnEdge), e, 2, 0), cell2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        for (int k = 0; k < L; k++)
            CW(ru, e, k) = 0.5 * CW(D(u), e, k) * (rc(S, rho_zz, cell1, k) + rc(S, rho_zz, cell2, k));
    }
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        for (int k = 0; k < L; k++) {
            CW(rw, c, k) = 0;
            if (k > 0)
                CW(rw, c, k) = CW(D(w), c, k) * (rz(S, fzp, k) * CW(rho_zz, c, k - 1) + rz(S, fzm, k) * CW(rho_zz, c, k)) *
                               (rz(S, fzp, k) * CW(zz, c, k - 1) + rz(S, fzm, k) * CW(zz, c, k));
        }
        const int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        for (int k = 1; k < L; k++)
            for (int i = 0; i < ne; i++) {
                const int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
                const double flux = rz(S, fzm, k) * re(S, ru, iEdge, k) + rz(S, fzp, k) * re(S, ru, iEdge, k - 1);
                CW(rw, c, k) -= rc2(S, D(edgesOnCellSign), c, 10, i) *
                                (rc3v(S, D(zb_cell), c, k, i) + copysign(1.0, flux) * rc3v(S, D(zb3_cell), c, k, i)) * flux *
                                (rz(S, fzp, k) * CW(zz, c, k - 1) + rz(S, fzm, k) * CW(zz, c, k));
            }
        for (int k = 0; k < L; k++) {
            CW(D(rho_p), c, k) = CW(rho_zz, c, k) - CW(D(rho_base), c, k);
            CW(D(rtheta_base), c, k) = CW(D(theta_base), c, k) * CW(D(rho_base), c, k);
            CW(D(rtheta_p), c, k) = CW(D(theta_m), c, k) * CW(D(rho_p), c, k) +
                                    CW(D(rho_base), c, k) * (CW(D(theta_m), c, k) - CW(D(theta_base), c, k));
            CW(D(exner), c, k) = pow(CW(zz, c, k) * (rgas_ / p0) * (CW(D(rtheta_p), c, k) + CW(D(rtheta_base), c, k)), rcv);
            CW(D(exner_base), c, k) = pow(CW(zz, c, k) * (rgas_ / p0) * (CW(D(rtheta_base), c, k)), rcv);
            CW(D(pressure_p), c, k) = CW(zz, c, k) * rgas_ *
                                      (CW(D(exner), c, k) * CW(D(rtheta_p), c, k) +
                                       CW(D(rtheta_base), c, k) * (CW(D(exner), c, k) - CW(D(exner_base), c, k)));
            CW(D(pressure_base), c, k) = CW(zz, c, k) * rgas_ * CW(D(exner_base), c, k) * CW(D(rtheta_base), c, k);
        }
    }
}

/* ===================== the MPAS vertical solver ("physics" mpas)
 * The reference's vertically implicit acoustic step with the statements it keeps as
 * comments restored and its quirks in that solver fixed; every other task is unchanged.
 *   vert_imp (dynamics_tasks.rg:513-592): Q16 b_tri takes cofwt(k-1) * rdzw(k-1); Q17
 *     alpha_tri/gamma_tri are the LU recurrence of this call (gamma(0) = 0, k ascending).
 *   acoustic (:1546-1723): Q18 the ru_p update and the ruAvg accumulation of :1581-1613;
 *     Q19/Q20 rs, ts of every level first and the explicit rw_p part from the old
 *     rho_pp/rtheta_pp of level k-1; Q21 the back substitution of :1674-1677; Q8 the
 *     tendencies dyn_tend produces: tend_ru = tend_u, tend_rt = tend_theta (tend_rw is w,
 *     where dyn_tend leaves it).  The MPAS-A statement order is kept throughout.
 *   recover (:1766-1872): Q24 fixed, w of the interior interfaces (ora_mpas_recover).
 *   srk3: the acoustic loop runs number_sub_steps times (Q5) and recover runs after it
 *     (the call rk_timestep.rg:460 keeps commented, Q7).                               */
void ora_mpas_vert_imp_coefs(ora_state* S, double dts) {
    ora_atm_compute_vert_imp_coefs(S, dts); /* coefficients, a_tri, c_tri as the reference */
    const int L = S->L, nC = S->nCells;
    double *rdzw = D(rdzw), *cofrz = D(cofrz), *zz = D(zz), *cofwr = D(cofwr), *cofwz = D(cofwz);
    double *coftz = D(coftz), *cofwt = D(cofwt), *a_tri = D(a_tri), *b_tri = D(b_tri), *c_tri = D(c_tri);
    double *alpha_tri = D(alpha_tri), *gamma_tri = D(gamma_tri);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        for (int k = 1; k < L; k++) /* Q16 */
            CW(b_tri, c, k) = 1.0 +
                              CW(cofwz, c, k) * (CW(coftz, c, k) * rdzw[k] * CW(zz, c, k) +
                                                 CW(coftz, c, k) * rdzw[k - 1] * CW(zz, c, k - 1)) -
                              CW(coftz, c, k) * (CW(cofwt, c, k) * rdzw[k] - CW(cofwt, c, k - 1) * rdzw[k - 1]) +
                              CW(cofwr, c, k) * ((cofrz[k] - cofrz[k - 1]));
        CW(gamma_tri, c, 0) = 0.0;
        for (int k = 1; k < L; k++) { /* Q17 */
            CW(alpha_tri, c, k) = 1.0 / (CW(b_tri, c, k) - CW(a_tri, c, k) * CW(gamma_tri, c, k - 1));
            CW(gamma_tri, c, k) = CW(c_tri, c, k) * CW(alpha_tri, c, k);
        }
    }
}

/* dyn = 0: physics 1 (dyn_tend's w tendency is in the state w, Q8); dyn = 1: physics 2,
 * the MPAS dynamics (tend_w; the implicit Rayleigh term stays on the state w)        */
static void mpas_acoustic(ora_state* S, double dts, int small_step, int dyn) {
    const int L = S->L, nC = S->nCells, nE = S->nEdges;
    double* tw = dyn ? D(tend_w) : D(w);
    const double epssm = config_epssm, rcv = rgas / (CP - rgas), c2 = CP * rcv;
    const double resm = (1.0 - epssm) / (1.0 + epssm);
    double *rtheta_pp_old = D(rtheta_pp_old), *rtheta_pp = D(rtheta_pp), *rho_pp = D(rho_pp);
    double *wwAvg = D(wwAvg), *rw_p = D(rw_p), *ru_p = D(ru_p), *ruAvg = D(ruAvg);
    double *cofrz = D(cofrz), *rdzw = D(rdzw), *fzm = D(fzm), *fzp = D(fzp);
    double *zz = D(zz), *theta_m = D(theta_m), *coftz = D(coftz), *w = D(w);
    /* :1581-1613 (Q18): horizontal momentum, every edge before any cell */
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) {
        const int cell1 = ie2(S, I(cellsOnEdge), e, 2, 0), cell2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        for (int k = 0; k < L; k++) {
            if (small_step != 0) {
                double pgrad = ((rc(S, rtheta_pp, cell2, k) - rc(S, rtheta_pp, cell1, k)) * re2(S, D(invDcEdge), e, 1, 0)) /
                               (0.5 * (rc(S, zz, cell2, k) + rc(S, zz, cell1, k)));
                pgrad = CW(D(cqu), e, k) * 0.5 * c2 * (rc(S, D(exner), cell1, k) + rc(S, D(exner), cell2, k)) * pgrad;
                pgrad = pgrad + 0.5 * CW(D(zxu), e, k) * gravity * (rc(S, rho_pp, cell1, k) + rc(S, rho_pp, cell2, k));
                CW(ru_p, e, k) = CW(ru_p, e, k) + dts * (CW(D(tend_u), e, k) - (1.0 - re2(S, D(specZoneMaskEdge), e, 1, 0)) * pgrad);
                CW(ruAvg, e, k) = CW(ruAvg, e, k) + CW(ru_p, e, k);
            } else {
                CW(ru_p, e, k) = dts * CW(D(tend_u), e, k);
                CW(ruAvg, e, k) = CW(ru_p, e, k);
            }
        }
    }
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        const int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        double rs[128], ts[128], rtp0[128], rpp0[128], rwp0[129];
        for (int k = 0; k < L; k++) CW(rtheta_pp_old, c, k) = (small_step == 0) ? 0 : CW(rtheta_pp, c, k);
        if (small_step == 0) {
            for (int k = 0; k <= L; k++) {
                CW(wwAvg, c, k) = 0;
                CW(rw_p, c, k) = 0;
            }
            for (int k = 0; k < L; k++) {
                CW(rho_pp, c, k) = 0;
                CW(rtheta_pp, c, k) = 0;
            }
        }
        if (rc2(S, D(specZoneMaskCell), c, 1, 0) != 0.0) { /* specified zone */
            for (int k = 0; k < L; k++) {
                CW(rho_pp, c, k) = CW(rho_pp, c, k) + dts * CW(D(tend_rho), c, k);
                CW(rtheta_pp, c, k) = CW(rtheta_pp, c, k) + dts * CW(D(tend_theta), c, k);
                CW(rw_p, c, k) = CW(rw_p, c, k) + dts * CW(tw, c, k);
                CW(wwAvg, c, k) = CW(wwAvg, c, k) + 0.5 * (1.0 + epssm) * CW(rw_p, c, k);
            }
            continue;
        }
        for (int k = 0; k < L; k++) {
            rtp0[k] = CW(rtheta_pp, c, k);
            rpp0[k] = CW(rho_pp, c, k);
            ts[k] = 0.0;
            rs[k] = 0.0;
        }
        for (int k = 0; k <= L; k++) rwp0[k] = CW(rw_p, c, k);
        for (int i = 0; i < ne; i++) {
            int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
            int cell1 = ie2(S, I(cellsOnEdge), iEdge, 2, 0), cell2 = ie2(S, I(cellsOnEdge), iEdge, 2, 1);
            for (int k = 0; k < L; k++) {
                double flux = rc2(S, D(edgesOnCellSign), c, 10, i) * dts * re2(S, D(dvEdge), iEdge, 1, 0) *
                              re(S, ru_p, iEdge, k) * rc2(S, D(invAreaCell), c, 1, 0);
                rs[k] = rs[k] - flux;
                ts[k] = ts[k] - flux * 0.5 * (rc(S, theta_m, cell2, k) + rc(S, theta_m, cell1, k));
            }
        }
        for (int k = 0; k < L; k++) {
            rs[k] = rpp0[k] + dts * CW(D(tend_rho), c, k) + rs[k] - cofrz[k] * resm * (rwp0[k + 1] - rwp0[k]);
            ts[k] = rtp0[k] + dts * CW(D(tend_theta), c, k) + ts[k] -
                    resm * rdzw[k] * (rc(S, coftz, c, k + 1) * rwp0[k + 1] - CW(coftz, c, k) * rwp0[k]);
        }
        for (int k = 1; k < L; k++) CW(wwAvg, c, k) = CW(wwAvg, c, k) + 0.5 * (1.0 - epssm) * rwp0[k];
        for (int k = 1; k < L; k++)
            CW(rw_p, c, k) = rwp0[k] + dts * CW(tw, c, k) -
                             CW(D(cofwz), c, k) * ((CW(zz, c, k) * ts[k] - CW(zz, c, k - 1) * ts[k - 1]) +
                                                   resm * (CW(zz, c, k) * rtp0[k] - CW(zz, c, k - 1) * rtp0[k - 1])) -
                             CW(D(cofwr), c, k) * ((rs[k] + rs[k - 1]) + resm * (rpp0[k] + rpp0[k - 1])) +
                             CW(D(cofwt), c, k) * (ts[k] + resm * rtp0[k]) + CW(D(cofwt), c, k - 1) * (ts[k - 1] + resm * rtp0[k - 1]);
        for (int k = 1; k < L; k++) /* tridiagonal solve: up ... */
            CW(rw_p, c, k) = (CW(rw_p, c, k) - CW(D(a_tri), c, k) * CW(rw_p, c, k - 1)) * CW(D(alpha_tri), c, k);
        for (int k = L - 1; k >= 0; k--) /* ... and down (Q21) */
            CW(rw_p, c, k) = CW(rw_p, c, k) - CW(D(gamma_tri), c, k) * CW(rw_p, c, k + 1);
        for (int k = 1; k < L; k++) { /* implicit Rayleigh damping of w */
            const double d = CW(D(rw_save), c, k) - CW(D(rw), c, k);
            CW(rw_p, c, k) = (CW(rw_p, c, k) + d -
                              dts * CW(D(dss), c, k) * (fzm[k] * CW(zz, c, k) + fzp[k] * CW(zz, c, k - 1)) *
                                  (fzm[k] * CW(D(rho_zz), c, k) + fzp[k] * CW(D(rho_zz), c, k - 1)) * CW(w, c, k)) /
                                 (1.0 + dts * CW(D(dss), c, k)) -
                             d;
        }
        for (int k = 1; k < L; k++) CW(wwAvg, c, k) = CW(wwAvg, c, k) + 0.5 * (1.0 + epssm) * CW(rw_p, c, k);
        for (int k = 0; k < L; k++) {
            CW(rho_pp, c, k) = rs[k] - cofrz[k] * (rc(S, rw_p, c, k + 1) - CW(rw_p, c, k));
            CW(rtheta_pp, c, k) = ts[k] - rdzw[k] * (rc(S, coftz, c, k + 1) * rc(S, rw_p, c, k + 1) - CW(coftz, c, k) * CW(rw_p, c, k));
        }
    }
}
void ora_mpas_acoustic_step(ora_state* S, double dts, int small_step) { mpas_acoustic(S, dts, small_step, 0); }
void ora_mpas2_acoustic_step(ora_state* S, double dts, int small_step) { mpas_acoustic(S, dts, small_step, 1); }

/* atm_recover_large_step_variables_work (:1766-1872) in the MPAS form: ru = ru_save + ru_p
 * and flux2 = fzm ru(k) + fzp ru(k-1) (Q24), exner = (zz rgas/p0 (rtheta_p + rtheta_base))^rcv,
 * w(0) = 0 and w(L) = 0 with rw, wwAvg, w of the interior interfaces only, the lower
 * boundary flux added to w(0) once per edge.                                         */
void ora_mpas_recover(ora_state* S, int ns, int rk_step, double dt) {
    const int L = S->L, nC = S->nCells, nE = S->nEdges;
    const double rcv = rgas / (CP - rgas), p0 = 1.0e5;
    double *rho_zz = D(rho_zz), *w = D(w), *ru = D(ru);
    for (int k = 0; k < L; k++) CW(rho_zz, nC, k) = 1.0;
    const double invNs = 1 / (double)ns;
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        for (int k = 0; k < L; k++) {
            CW(D(rho_p), c, k) = CW(D(rho_p_save), c, k) + CW(D(rho_pp), c, k);
            CW(rho_zz, c, k) = CW(D(rho_p), c, k) + CW(D(rho_base), c, k);
        }
        CW(w, c, 0) = 0.0;
        for (int k = 1; k < L; k++) {
            CW(D(wwAvg), c, k) = CW(D(rw_save), c, k) + (CW(D(wwAvg), c, k) * invNs);
            CW(D(rw), c, k) = CW(D(rw_save), c, k) + CW(D(rw_p), c, k);
            CW(w, c, k) = CW(D(rw), c, k) / (rz(S, D(fzm), k) * CW(D(zz), c, k) + rz(S, D(fzp), k) * CW(D(zz), c, k - 1));
        }
        CW(w, c, L) = 0.0;
        for (int k = 0; k < L; k++) {
            if (rk_step == 2) {
                CW(D(rtheta_p), c, k) = CW(D(rtheta_p_save), c, k) + CW(D(rtheta_pp), c, k) -
                                        dt * CW(rho_zz, c, k) * CW(D(rt_diabatic_tend), c, k);
                CW(D(theta_m), c, k) = (CW(D(rtheta_p), c, k) + CW(D(rtheta_base), c, k)) / CW(rho_zz, c, k);
                CW(D(exner), c, k) = pow(CW(D(zz), c, k) * (rgas / p0) * (CW(D(rtheta_p), c, k) + CW(D(rtheta_base), c, k)), rcv);
                CW(D(pressure_p), c, k) = CW(D(zz), c, k) * rgas *
                                          (CW(D(exner), c, k) * CW(D(rtheta_p), c, k) +
                                           CW(D(rtheta_base), c, k) * (CW(D(exner), c, k) - CW(D(exner_base), c, k)));
            } else {
                CW(D(rtheta_p), c, k) = CW(D(rtheta_p_save), c, k) + CW(D(rtheta_pp), c, k);
                CW(D(theta_m), c, k) = (CW(D(rtheta_p), c, k) + CW(D(rtheta_base), c, k)) / CW(rho_zz, c, k);
            }
        }
    }
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) {
        int cell1 = ie2(S, I(cellsOnEdge), e, 2, 0), cell2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        for (int k = 0; k < L; k++) {
            CW(D(ruAvg), e, k) = CW(D(ru_save), e, k) + (CW(D(ruAvg), e, k) * invNs);
            CW(ru, e, k) = CW(D(ru_save), e, k) + CW(D(ru_p), e, k);
            CW(D(u), e, k) = 2. * CW(ru, e, k) / (rc(S, rho_zz, cell1, k) + rc(S, rho_zz, cell2, k));
        }
    }
    const double cf1 = rz(S, D(cf1), 0), cf2 = rz(S, D(cf2), 0), cf3 = rz(S, D(cf3), 0);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        if (ic2(S, I(bdyMaskCell), c, 1, 0) > nRelaxZone) continue;
        const int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        for (int i = 0; i < ne; i++) {
            int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
            double sg = rc2(S, D(edgesOnCell_sign), c, 10, i);
            double flux = (cf1 * re(S, ru, iEdge, 0) + cf2 * re(S, ru, iEdge, 1) + cf3 * re(S, ru, iEdge, 2));
            CW(w, c, 0) = CW(w, c, 0) + sg * (rc3v(S, D(zb_cell), c, 0, i) + copysign(1.0, flux) * rc3v(S, D(zb3_cell), c, 0, i)) * flux;
            for (int k = 1; k < L; k++) {
                flux = (rz(S, D(fzm), k) * re(S, ru, iEdge, k) + rz(S, D(fzp), k) * re(S, ru, iEdge, k - 1));
                CW(w, c, k) = CW(w, c, k) + sg * (rc3v(S, D(zb_cell), c, k, i) + copysign(1.0, flux) * rc3v(S, D(zb3_cell), c, k, i)) * flux;
            }
        }
        CW(w, c, 0) = CW(w, c, 0) / (cf1 * CW(rho_zz, c, 0) + cf2 * rc(S, rho_zz, c, 1) + cf3 * rc(S, rho_zz, c, 2));
        for (int k = 1; k < L; k++)
            CW(w, c, k) = CW(w, c, k) / (rz(S, D(fzm), k) * CW(rho_zz, c, k) + rz(S, D(fzp), k) * CW(rho_zz, c, k - 1));
    }
}

/* ===================== the MPAS dynamics (option physics = 2)
 * Every remaining quirk of the RK3 path fixed as MPAS-A (MPAS-Model v7
 * mpas_atm_time_integration.F, not vendored) defines it, on top of the vertical solver
 * above (physics = 1):
 *   setup   (:747-778)  theta_m_save = theta_m (read by dyn_tend rk > 0, never written: Q2)
 *   moist   (:460-502)  cqu = 1/(1 + qtotal of the edge) (the commented edge loop, Q25)
 *   dyn_tend (:814-1480) tend_rho with the physics term outside the flux divergence; the
 *           top wduz/wdwz/wdtz = 0; q summed once (Q10); curvature -A - B (Q12); the w
 *           tendency in its own array tend_w computed from the state w (Q8), the
 *           horizontal w flux accumulated over every edge (Q13), tend_w = flux
 *           invAreaCell + curvature - d(wdwz)/dz (Q14; the curvature is not area-scaled),
 *           wdtz = 3rd-order flux of theta_m by rw + the rtheta_pp term (Q15)
 *           (dyn_tend_impl with mpas = 1)
 *   set_smlstep (:1503-1528) u_tend = tend_u, w_tend = tend_w (Q2/Q8), levels 1..L-1
 *   acoustic tend_rw = tend_w (mpas_acoustic, dyn = 1)
 *   solve_diagnostics (:328-454) h = rho_zz, rho_edge = h_edge (the MPAS-A caller passes
 *           diag%rho_edge as h_edge; Q2); divergence += sign dvEdge u (Q9); v over every
 *           edgesOnEdge entry (Q23)
 *   srk3    mpas_reconstruct_2d after the RK loop (rk_timestep.rg:487, commented); the
 *           substep finish keeps rho_zz (MPAS-A resets rho_zz of the OLD time level,
 *           :2001-2004 writes the only one the port has)                             */
void ora_mpas_rk_integration_setup(ora_state* S) {
    ora_atm_rk_integration_setup(S);
    const int L = S->L;
#pragma omp parallel for schedule(static)
    for (long c = 0; c < S->nCells; c++)
        for (int k = 0; k < L; k++) CW(D(theta_m_save), c, k) = CW(D(theta_m), c, k);
}

void ora_mpas_moist_coefficients(ora_state* S) {
    ora_atm_compute_moist_coefficients(S);
    const int L = S->L;
#pragma omp parallel for schedule(static)
    for (long e = 0; e < S->nEdges; e++) {
        int cell1 = ie2(S, I(cellsOnEdge), e, 2, 0), cell2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        for (int k = 0; k < L; k++) {
            double qtotal = 0.5 * (rc(S, D(qtot), cell1, k) + rc(S, D(qtot), cell2, k));
            CW(D(cqu), e, k) = 1.0 / (1.0 + qtotal);
        }
    }
}

void ora_mpas_dyn_tend(ora_state* S, int rk_step, double dt, int horiz_mixing, double config_mpas_cam_coef,
                       int config_mix_full, int config_rayleigh_damp_u) {
    dyn_tend_impl(S, rk_step, dt, horiz_mixing, config_mpas_cam_coef, config_mix_full, config_rayleigh_damp_u, 1);
}

void ora_mpas_set_smlstep(ora_state* S) {
    const int L = S->L, nC = S->nCells;
    double *tw = D(tend_w), *zz = D(zz), *tu = D(tend_u), *fzm = D(fzm), *fzp = D(fzp);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        if (ic2(S, I(bdyMaskCell), c, 1, 0) > nRelaxZone) continue;
        int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        for (int i = 0; i < ne; i++) {
            int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
            for (int k = 1; k < L; k++) {
                double flux = rc2(S, D(edgesOnCell_sign), c, 10, i) * (fzm[k] * re(S, tu, iEdge, k) + fzp[k] * re(S, tu, iEdge, k - 1));
                CW(tw, c, k) = CW(tw, c, k) - (rc3v(S, D(zb_cell), c, k, i) + copysign(1.0, re(S, tu, iEdge, k)) * rc3v(S, D(zb3_cell), c, k, i)) * flux;
            }
        }
        for (int k = 1; k < L; k++) CW(tw, c, k) = (fzm[k] * CW(zz, c, k) + fzp[k] * CW(zz, c, k - 1)) * CW(tw, c, k);
    }
}

void ora_mpas_solve_diagnostics(ora_state* S, int hollingsworth, int rk_step) {
    const int L = S->L, nC = S->nCells, nE = S->nEdges;
    double *u = D(u), *rho_zz = D(rho_zz), *h_edge = D(h_edge), *rho_edge = D(rho_edge);
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) { /* h = rho_zz; rho_edge is MPAS-A's h_edge */
        int cell1 = ie2(S, I(cellsOnEdge), e, 2, 0), cell2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        for (int k = 0; k < L; k++) {
            CW(h_edge, e, k) = 0.5 * (rc(S, rho_zz, cell1, k) + rc(S, rho_zz, cell2, k));
            CW(rho_edge, e, k) = CW(h_edge, e, k);
        }
    }
    /* the reference's diagnostics; then the fixed divergence (Q9) and v (Q23) */
    double* h = D(h);
    S->f[F_h] = rho_zz; /* (the h the reference reads is rho_zz: h_edge as above) */
    ora_atm_compute_solve_diagnostics(S, hollingsworth, -3); /* -3: no v here */
    S->f[F_h] = h;
    double* div = D(divergence);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) {
        int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        for (int k = 0; k < L; k++) {
            CW(div, c, k) = 0.0;
            for (int i = 0; i < ne; i++) {
                int iEdge = ic2(S, I(edgesOnCell), c, 10, i);
                double s = rc2(S, D(edgesOnCellSign), c, 10, i) * re2(S, D(dvEdge), iEdge, 1, 0);
                CW(div, c, k) += s * re(S, u, iEdge, k);
            }
            CW(div, c, k) *= rc2(S, D(invAreaCell), c, 1, 0);
        }
    }
    if (rk_step == -1 || rk_step == 2) {
        double* vv = D(v);
#pragma omp parallel for schedule(static)
        for (long e = 0; e < nE; e++) {
            int neoe = ie2(S, I(nEdgesOnEdge), e, 1, 0);
            for (int k = 0; k < L; k++) {
                CW(vv, e, k) = 0;
                for (int i = 0; i < neoe; i++) {
                    int eoe = ie2(S, I(edgesOnEdge_ECP), e, 20, i);
                    CW(vv, e, k) += re2(S, D(weightsOnEdge), e, 20, i) * re(S, u, eoe, k);
                }
            }
        }
    }
}

void ora_mpas_substep_finish(ora_state* S, int dynamics_substep, int dynamics_split) {
    const int L = S->L;
    double* keep = (double*)malloc(sizeof(double) * (size_t)(S->nCells + 1) * LV);
    memcpy(keep, D(rho_zz), sizeof(double) * (size_t)(S->nCells + 1) * LV);
    ora_atm_rk_dynamics_substep_finish(S, dynamics_substep, dynamics_split);
    memcpy(D(rho_zz), keep, sizeof(double) * (size_t)(S->nCells + 1) * LV);
    free(keep);
    (void)L;
}

/* surface pressure (MPAS-A's diagnostic, the formula init_atm_case_jw uses,
 * init_atm_cases.rg:519-520): hydrostatic extrapolation of the lowest two levels */
void ora_mpas_surface_pressure(ora_state* S) {
    const int nC = S->nCells;
    const double dz0 = 1.0 / D(rdzw)[0];
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++)
        CW(D(surface_pressure), c, 0) =
            0.5 * dz0 * gravity * (1.25 * (CW(D(rho_zz), c, 0) * (1.0 + CW(D(qtot), c, 0))) -
                                   0.25 * (CW(D(rho_zz), c, 1) * (1.0 + CW(D(qtot), c, 1)))) +
            CW(D(pressure_p), c, 0) + CW(D(pressure_base), c, 0);
}

void ora_mpas_advance_scalars_mono(ora_state* S, double dt);

/* transport != 0: the monotonic scalar transport over the step (scalars_old = scalars
 * at the start, ora_mpas_advance_scalars_mono after the last stage's recover) */
void ora_mpas_srk3_dyn(ora_state* S, double dt, int schedule, int transport, int physics);
void ora_mpas_srk3_ex(ora_state* S, double dt, int schedule, int transport) { ora_mpas_srk3_dyn(S, dt, schedule, transport, 1); }
/* physics 1: the vertical solver only; physics 2: the MPAS dynamics */
void ora_mpas_srk3_dyn(ora_state* S, double dt, int schedule, int transport, int physics) {
    const int md = physics >= 2;
    if (transport) memcpy(D(scalars_old), D(scalars), sizeof(double) * (size_t)(S->nCells + 1) * LV * NSC);
    int number_of_sub_steps = 2;
    double rk_sub_timestep[3] = {dt / 3, dt / number_of_sub_steps, dt / number_of_sub_steps};
    int number_sub_steps[3];
    number_sub_steps[0] = (number_of_sub_steps / 2 > 1) ? number_of_sub_steps / 2 : 1;
    number_sub_steps[1] = number_sub_steps[0];
    number_sub_steps[2] = number_of_sub_steps;
    if (md) {
        ora_mpas_rk_integration_setup(S);
        ora_mpas_moist_coefficients(S);
    } else {
        ora_atm_rk_integration_setup(S);
        ora_atm_compute_moist_coefficients(S);
    }
    ora_mpas_vert_imp_coefs(S, rk_sub_timestep[0]);
    for (int rk_step = 0; rk_step < 3; rk_step++) {
        if (rk_step == 1) ora_mpas_vert_imp_coefs(S, rk_sub_timestep[rk_step]);
        int dyn_rk = schedule == 0 ? (int)rk_sub_timestep[rk_step] : rk_step;
        if (md) {
            ora_mpas_dyn_tend(S, dyn_rk, dt, 0, 0.0, 0, 0);
            ora_mpas_set_smlstep(S);
        } else {
            ora_atm_compute_dyn_tend_work(S, dyn_rk, dt, 0, 0.0, 0, 0);
            ora_atm_set_smlstep_pert_variables_work(S);
        }
        for (int small_step = 0; small_step < number_sub_steps[rk_step]; small_step++) { /* Q5 */
            mpas_acoustic(S, rk_sub_timestep[rk_step], small_step, md);
            ora_atm_divergence_damping_3d(S, rk_sub_timestep[rk_step]);
        }
        ora_mpas_recover(S, number_sub_steps[rk_step], rk_step, dt); /* rk_timestep.rg:460 (Q7) */
        if (md) ora_mpas_solve_diagnostics(S, 0, rk_step);
        else ora_atm_compute_solve_diagnostics(S, 0, rk_step);
    }
    if (transport) ora_mpas_advance_scalars_mono(S, dt);
    if (md) {
        ora_mpas_reconstruct_2d(S, 0, 1); /* rk_timestep.rg:487 (commented in the reference) */
        ora_mpas_substep_finish(S, 1, 1);
    } else {
        ora_atm_rk_dynamics_substep_finish(S, 1, 1);
    }
}
void ora_mpas_srk3(ora_state* S, double dt, int schedule) { ora_mpas_srk3_ex(S, dt, schedule, 0); }

/* ===================== monotonic scalar transport (Q26: the reference
 * has no transport -- only the untouched scalars:double[8], data_structures.rg:36, and
 * nScalars = 8, constants.rg:42 -- so this restates the published algorithm MPAS-A uses,
 * atm_advance_scalars_mono_work of MPAS-Model src/core_atmosphere/dynamics/
 * mpas_atm_time_integration.F (v7/v8; not vendored here): Zalesak (1979) flux-corrected
 * transport as in Skamarock & Gassmann (2011).  PARITY UNPINNED (no reference run); the
 * tests pin it by its defining properties instead: constant preservation under a mass-
 * consistent flow, bounds (no new extrema), conservation of sum(rho s volume).
 *   per scalar i, level k < L, with rho_old = rho_zz_old_split, rho_new = rho_zz, the
 *   stage-averaged mass fluxes ruAvg (edges) and wwAvg (interfaces 1..L-1; 0 and L carry
 *   no flux), coef3 = config_coef_3rd_order = 0.25:
 *   edge high-order flux  u sum_j (adv_coefs_j + sign(u) adv_coefs_3rd_j) s(advCell_j)
 *        (the theta advection of dyn_tend, dynamics_tasks.rg:1333-1340, same coefficients),
 *   edge upwind flux      dvEdge (max(u,0) s(c1) + min(u,0) s(c2)),
 *   interface high-order  flux3(s(k-2), s(k-1), s(k), s(k+1), w, coef3) for 2 <= k <= L-2,
 *                         w (fzm s(k) + fzp s(k-1)) at k = 1 and k = L-1,
 *   interface upwind      max(w,0) s(k-1) + min(w,0) s(k),
 *   antidiffusive flux A = high - upwind; the upwind update su; the bounds of the old
 *   values of the cell (levels k-1..k+1), of the other cell of each edge (level k) and su;
 *   R+ / R- the largest fractions of the incoming / outgoing A the bounds allow; each A
 *   scaled by min(R- of its source, R+ of its receiver); s_new = su - dt div(scaled A) / rho_new.
 * The sign of an edge for a cell is +1 where the cell is cellsOnEdge(0), else -1 (the
 * orientation of edgesOnCellSign, computed here from the ids so the limiter's source /
 * receiver choice and the divergence agree on any mesh).                               */
static inline double scv(const ora_state* S, const double* f, long c, long k, int i) {
    if (c < 0 || c > S->nCells || k < 0 || k > S->L) return 0.0;
    return f[(c * LV + k) * NSC + i];
}
/* interface kk of column c, scalar i: upwind flux (lo) and antidiffusive flux (A) */
static void ora_vflux(const ora_state* S, const double* so, const double* ww, long c, int kk, int i, double* lo, double* A) {
    const int L = S->L;
    if (kk <= 0 || kk >= L) {
        *lo = 0.0;
        *A = 0.0;
        return;
    }
    const double w = rc(S, ww, c, kk);
    const double sm1 = scv(S, so, c, kk - 1, i), s0 = scv(S, so, c, kk, i);
    double hi;
    if (kk >= 2 && kk <= L - 2)
        hi = flux3(scv(S, so, c, kk - 2, i), sm1, s0, scv(S, so, c, kk + 1, i), w, 0.25);
    else
        hi = w * (rz(S, D(fzm), kk) * s0 + rz(S, D(fzp), kk) * sm1);
    *lo = fmax(w, 0.0) * sm1 + fmin(w, 0.0) * s0;
    *A = hi - *lo;
}

void ora_mpas_advance_scalars_mono(ora_state* S, double dt) {
    const int L = S->L, nC = S->nCells, nE = S->nEdges;
    double *so = D(scalars_old), *sn = D(scalars), *ro = D(rho_zz_old_split), *rn = D(rho_zz);
    double *ru = D(ruAvg), *ww = D(wwAvg), *rdzw = D(rdzw);
    const long PE = (long)L * NSC;
    double* Ah = (double*)calloc((size_t)nE * PE, sizeof(double));
    double* Rp = (double*)calloc((size_t)nC * PE, sizeof(double));
    double* Rm = (double*)calloc((size_t)nC * PE, sizeof(double));
    double* su = (double*)calloc((size_t)nC * PE, sizeof(double));
    if (!Ah || !Rp || !Rm || !su) abort();
#pragma omp parallel for schedule(static)
    for (long e = 0; e < nE; e++) { /* edge fluxes */
        const int c1 = ie2(S, I(cellsOnEdge), e, 2, 0), c2 = ie2(S, I(cellsOnEdge), e, 2, 1);
        const int na = ie2(S, I(nAdvCellsForEdge), e, 1, 0);
        const double dv = re2(S, D(dvEdge), e, 1, 0);
        for (int k = 0; k < L; k++) {
            const double u = re(S, ru, e, k);
            for (int i = 0; i < NSC; i++) {
                double acc = 0.0;
                for (int j = 0; j < na; j++) {
                    const double wgt = re2(S, D(adv_coefs), e, 15, j) + copysign(1.0, u) * re2(S, D(adv_coefs_3rd), e, 15, j);
                    acc = acc + wgt * scv(S, so, ie2(S, I(advCellsForEdge), e, 15, j), k, i);
                }
                const double lo = dv * (fmax(u, 0.0) * scv(S, so, c1, k, i) + fmin(u, 0.0) * scv(S, so, c2, k, i));
                Ah[e * PE + k * NSC + i] = u * acc - lo;
            }
        }
    }
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) { /* upwind update, bounds, R+ / R- */
        const int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        const double invA = rc2(S, D(invAreaCell), c, 1, 0);
        for (int k = 0; k < L; k++)
            for (int i = 0; i < NSC; i++) {
                const double s = scv(S, so, c, k, i);
                double hlo = 0.0, pin = 0.0, pout = 0.0, smax = s, smin = s;
                for (int j = 0; j < ne; j++) {
                    const int e = ic2(S, I(edgesOnCell), c, 10, j);
                    const int c1 = ie2(S, I(cellsOnEdge), e, 2, 0), c2 = ie2(S, I(cellsOnEdge), e, 2, 1);
                    const double sg = (c1 == c) ? 1.0 : -1.0;
                    const double u = re(S, ru, e, k), s1 = scv(S, so, c1, k, i), s2 = scv(S, so, c2, k, i);
                    const double lo = re2(S, D(dvEdge), e, 1, 0) * (fmax(u, 0.0) * s1 + fmin(u, 0.0) * s2);
                    hlo = hlo + sg * lo;
                    const double a = -sg * ((e >= 0 && e < nE) ? Ah[(long)e * PE + k * NSC + i] : 0.0);
                    pin = pin + fmax(a, 0.0);
                    pout = pout - fmin(a, 0.0);
                    const double so_ = (c1 == c) ? s2 : s1;
                    smax = fmax(smax, so_);
                    smin = fmin(smin, so_);
                }
                if (k > 0) {
                    smax = fmax(smax, scv(S, so, c, k - 1, i));
                    smin = fmin(smin, scv(S, so, c, k - 1, i));
                }
                if (k < L - 1) {
                    smax = fmax(smax, scv(S, so, c, k + 1, i));
                    smin = fmin(smin, scv(S, so, c, k + 1, i));
                }
                double lob, Ab, lot, At;
                ora_vflux(S, so, ww, c, k, i, &lob, &Ab);
                ora_vflux(S, so, ww, c, k + 1, i, &lot, &At);
                const double r_o = CW(ro, c, k), r_n = CW(rn, c, k);
                const double u_ = (s * r_o - dt * (hlo * invA + (lot - lob) * rdzw[k])) / r_n;
                smax = fmax(smax, u_);
                smin = fmin(smin, u_);
                const double pin_t = dt * (pin * invA + (fmax(Ab, 0.0) - fmin(At, 0.0)) * rdzw[k]);
                const double pout_t = dt * (pout * invA + (fmax(At, 0.0) - fmin(Ab, 0.0)) * rdzw[k]);
                const double qin = (smax - u_) * r_n, qout = (u_ - smin) * r_n;
                const long o = c * PE + k * NSC + i;
                Rp[o] = pin_t > 0.0 ? fmin(1.0, qin / pin_t) : 0.0;
                Rm[o] = pout_t > 0.0 ? fmin(1.0, qout / pout_t) : 0.0;
                su[o] = u_;
            }
    }
#pragma omp parallel for schedule(static)
    for (long c = 0; c < nC; c++) { /* the limited antidiffusive fluxes */
        const int ne = ic2(S, I(nEdgesOnCell), c, 1, 0);
        const double invA = rc2(S, D(invAreaCell), c, 1, 0);
        for (int k = 0; k < L; k++)
            for (int i = 0; i < NSC; i++) {
                double hc = 0.0;
                for (int j = 0; j < ne; j++) {
                    const int e = ic2(S, I(edgesOnCell), c, 10, j);
                    const int c1 = ie2(S, I(cellsOnEdge), e, 2, 0), c2 = ie2(S, I(cellsOnEdge), e, 2, 1);
                    const double sg = (c1 == c) ? 1.0 : -1.0;
                    const double A = (e >= 0 && e < nE) ? Ah[(long)e * PE + k * NSC + i] : 0.0;
                    const double Rp1 = (c1 >= 0 && c1 < nC) ? Rp[(long)c1 * PE + k * NSC + i] : 0.0;
                    const double Rm1 = (c1 >= 0 && c1 < nC) ? Rm[(long)c1 * PE + k * NSC + i] : 0.0;
                    const double Rp2 = (c2 >= 0 && c2 < nC) ? Rp[(long)c2 * PE + k * NSC + i] : 0.0;
                    const double Rm2 = (c2 >= 0 && c2 < nC) ? Rm[(long)c2 * PE + k * NSC + i] : 0.0;
                    const double C = A >= 0.0 ? fmin(Rm1, Rp2) : fmin(Rp1, Rm2);
                    hc = hc + sg * (C * A);
                }
                double fcb = 0.0, fct = 0.0, lo, A;
                if (k > 0) {
                    ora_vflux(S, so, ww, c, k, i, &lo, &A);
                    const long b = c * PE + (k - 1) * NSC + i, t = c * PE + k * NSC + i;
                    fcb = (A >= 0.0 ? fmin(Rm[b], Rp[t]) : fmin(Rp[b], Rm[t])) * A;
                }
                if (k + 1 < L) {
                    ora_vflux(S, so, ww, c, k + 1, i, &lo, &A);
                    const long b = c * PE + k * NSC + i, t = c * PE + (k + 1) * NSC + i;
                    fct = (A >= 0.0 ? fmin(Rm[b], Rp[t]) : fmin(Rp[b], Rm[t])) * A;
                }
                const long o = c * PE + k * NSC + i;
                sn[(c * LV + k) * NSC + i] = su[o] - dt * (hc * invA + (fct - fcb) * rdzw[k]) / CW(rn, c, k);
            }
    }
    free(Ah);
    free(Rp);
    free(Rm);
    free(su);
}

/* ===================== synthetic state (test/bench inputs, not reference semantics) */
static const struct { int kind, width, dist; double lo, hi; } ora_fields[] = {
#define C3 0
#define C3V 1
#define E3 2
#define V3 3
#define C2F 4
#define C2I 5
#define E2F 6
#define E2I 7
#define V2F 8
#define V2I 9
#define C3B 10
#define ZV 11
#define U MPAS_DIST_U
#define M MPAS_DIST_M
#define MPAS_FIELD(name, KIND, W, DIST, LO, HI) {KIND, W, DIST, LO, HI},
#include "mpas_fields.def"
#undef MPAS_FIELD
};

int ora_field_count(void) { return F_COUNT; }

/* Fill every U/Z/B/S field (and, with include_mesh, the fp64 M fields) of the state
 * from the counter-based generator; row n (zero slot) is left untouched.           */
void ora_fill_synthetic(ora_state* S, uint64_t seed, int include_mesh) {
    for (int f = 0; f < F_COUNT; f++) {
        int kind = ora_fields[f].kind, W = ora_fields[f].width, dist = ora_fields[f].dist;
        double lo = ora_fields[f].lo, hi = ora_fields[f].hi;
        if (dist == MPAS_DIST_M) {
            if (!include_mesh) continue;
            if (kind != C2F && kind != E2F && kind != V2F) continue;
            dist = MPAS_DIST_U;
        }
        double* p = (double*)S->f[f];
        long n = 0;
        int levels = 0;
        switch (kind) {
            case C3: n = S->nCells; levels = S->L + 1; break;
            case E3: n = S->nEdges; levels = S->L + 1; break;
            case V3: n = S->nVertices; levels = S->L + 1; break;
            case C3V: n = S->nCells; levels = S->L + 1; break;
            case C2F: n = S->nCells; break;
            case E2F: n = S->nEdges; break;
            case V2F: n = S->nVertices; break;
            case ZV: n = 1; levels = S->L + 1; break;
            default: continue;
        }
        if (kind == C3 || kind == E3 || kind == V3) {
#pragma omp parallel for schedule(static)
            for (long e = 0; e < n; e++)
                for (int k = 0; k < levels; k++)
                    p[e * levels + k] = mpas_synth_value(seed, f, e, k, 0, dist, lo, hi);
        } else if (kind == C3V) {
#pragma omp parallel for schedule(static)
            for (long e = 0; e < n; e++)
                for (int k = 0; k < levels; k++)
                    for (int i = 0; i < W; i++)
                        p[(e * levels + k) * W + i] = mpas_synth_value(seed, f, e, k, i, dist, lo, hi);
        } else if (kind == ZV) {
            for (int k = 0; k < levels; k++) p[k] = mpas_synth_value(seed, f, 0, k, 0, dist, lo, hi);
        } else {
#pragma omp parallel for schedule(static)
            for (long e = 0; e < n; e++)
                for (int i = 0; i < W; i++) p[e * W + i] = mpas_synth_value(seed, f, e, 0, i, dist, lo, hi);
        }
    }
}
