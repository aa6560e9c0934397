// k_solve.hip -- atm_compute_solve_diagnostics (dynamics_tasks.rg:328-454) for gfx950.
//
// Two launches instead of the reference's five loop nests:
//   1. vertices + cells in one grid: vorticity, pv_vertex (vertex columns);
//      divergence (Q9 literal "s + u"), ke (cell columns; ke_edge of each edge of the
//      cell is recomputed from u with the edge loop's exact expression, so no
//      edge->cell barrier is needed)
//   2. edges: h_edge, ke_edge, v (only rk_step in {-1, 2}, Q23 starts at i = 1), pv_edge
// Hollingsworth (never true on the path, rk_timestep.rg:467) adds a ke_vertex pass.
#include "mpas_dev.h"
#include "mpas_halo.h"

#include <type_traits>

namespace mpas {

// MD: the MPAS dynamics (physics = 2, ora_mpas_solve_diagnostics): divergence += s * u (Q9),
// h = rho_zz and rho_edge = h_edge (Q2: MPAS-A passes diag%rho_edge as h_edge), v over
// every edgesOnEdge entry (Q23)
template <int LP, int EPW, bool MD>
__global__ __launch_bounds__(256) void k_solve_vc(DevState S, int nVB, int hollingsworth_part) {
    const int L = S.L;
    const double* u = fd(S, F_u);
    const double *dcEdge = fd(S, F_dcEdge), *dvEdge = fd(S, F_dvEdge);
    ColMapN<LP, EPW> m(S, KV);
    const int k = m.k;
    int bi;
    if (vc_block(S, m.blk, nVB, bi)) {  // EPW vertices: vorticity, pv_vertex (:381-396)
        m.base = col_of<LP>(bi) * EPW + S.lo[KV];
        int ev[EPW][3];
        double sg_[EPW][3], dc_[EPW][3], u_[EPW][3], iat[EPW], fv[EPW];
#pragma unroll
        for (int j = 0; j < EPW; j++) {
            const int v = min(m.base + j, S.nVO - 1);
            row_ld(fi(S, F_edgesOnVertex) + (size_t)v * 3, ev[j]);
            row_ld(fd(S, F_edgesOnVertexSign) + (size_t)v * 3, sg_[j]);
            row_ld(fd(S, X_ve_dc) + (size_t)v * 3, dc_[j]);  // dcEdge(edgesOnVertex)
            iat[j] = fd(S, F_invAreaTriangle)[v];
            fv[j] = fd(S, F_fVertex)[v];
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
            put2<LP>(fw(S, F_vorticity), v, fw(S, F_pv_vertex), v, k, PADW(vort), PADW(fv[j] + vort), k != L, k != L);
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
        ne[j] = fi(S, F_nEdgesOnCell)[c];
        invA[j] = fd(S, F_invAreaCell)[c];
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
        put2<LP>(fw(S, F_divergence), c, fw(S, F_ke), c, k, PADW(div), PADW(ke), k != L, k != L);
    }
}

// hollingsworth second half (:405-417): cells, needs ke_vertex of the whole mesh
template <int LP>
__global__ __launch_bounds__(256) void k_solve_holl(DevState S) {
    ColMap<LP> m(S, KC);
    const int L = S.L, c = m.ent, k = m.k;
    if (c >= S.nCO || k >= L) return;
    const size_t p = (size_t)c * LP + lpos(LP, k);
    double ke_fact = 1.0 - 0.375;
    double ke = colk(fd(S, F_ke), c) * ke_fact;
    double r = fd(S, F_invAreaCell)[c];
    const int ne = fi(S, F_nEdgesOnCell)[c];
    for (int i = 0; i < ne; i++) {
        int iVertex = fi(S, F_verticesOnCell)[(size_t)c * 10 + i];
        int j = fi(S, F_kiteForCell)[(size_t)c * 10 + i];
        double kite = (j >= 0 && j < 3) ? fd(S, F_kiteAreasOnVertex)[(size_t)iVertex * 3 + j] : 0.0;
        ke += (1.0 - ke_fact) * kite * colk(fd(S, F_ke_vertex), iVertex) * r;
    }
    colk(fw(S, F_ke), c) = ke;
}

// EPW consecutive edges per column slot (option "epw"): the loads of all of them are issued
// before the first store; the paired 16-B stores write h_edge with ke_edge and pv_edge with
// v (or alone) -- every lane takes part (put2), level L keeps its value
template <int LP, bool RECON_V, bool MD, int EPW>
__global__ __launch_bounds__(256) void k_solve_e(DevState S) {
    ColMapN<LP, EPW> m(S, KE);
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
        gather2s<LP>(h, coe[0], coe[1], k, h1[j], h2[j]);
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
            uu[j] = colk(u, e);
        }
    }
#pragma unroll
    for (int j = 0; j < EPW; j++) {
        const int e = m.base + j;
        if (e >= S.nEO) break;  // (wave-uniform)
        const double efac = fd(S, F_dcEdge)[e] * fd(S, F_dvEdge)[e];
        const bool w = k != L;  // (padding levels k > L: zeros, PADW)
        put2<LP>(fw(S, F_h_edge), e, fw(S, F_ke_edge), e, k, PADW(0.5 * (h1[j] + h2[j])), PADW(efac * (uu[j] * uu[j])),
                 w, w);
        if (MD && w) colk(fw(S, F_rho_edge), e) = PADW(0.5 * (h1[j] + h2[j]));
        if (RECON_V) put2<LP>(fw(S, F_v), e, fw(S, F_pv_edge), e, k, PADW(vv[j]), PADW(0.5 * (pv1[j] + pv2[j])), w, w);
        else if (w) colk(fw(S, F_pv_edge), e) = PADW(0.5 * (pv1[j] + pv2[j]));
    }
}

template <int LP, bool MD>
static hipError_t solve_lp_md(const DevState& S, hipStream_t st, int hollingsworth, int rk_step) {
    auto kvc = [&](const DevState& X) {  // vertex blocks, then cell blocks
        if (X.epw == 4) {
            const int nv = col_blocks_n<LP, 4>(X, KV), nb = nv + col_blocks_n<LP, 4>(X, KC);
            if (nb) k_solve_vc<LP, 4, MD><<<nb, 256, 0, st>>>(X, nv, hollingsworth);
        } else if (X.epw == 2) {
            const int nv = col_blocks_n<LP, 2>(X, KV), nb = nv + col_blocks_n<LP, 2>(X, KC);
            if (nb) k_solve_vc<LP, 2, MD><<<nb, 256, 0, st>>>(X, nv, hollingsworth);
        } else {
            const int nv = col_blocks_n<LP, 1>(X, KV), nb = nv + col_blocks_n<LP, 1>(X, KC);
            if (nb) k_solve_vc<LP, 1, MD><<<nb, 256, 0, st>>>(X, nv, hollingsworth);
        }
    };
    auto kh = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (nb) k_solve_holl<LP><<<nb, 256, 0, st>>>(X);
    };
    auto ke = [&](const DevState& X) {
        const bool rv = !(rk_step != -1 && rk_step != 2);
        auto go = [&](auto epw) {
            constexpr int E = decltype(epw)::value;
            const int nb = col_blocks_n<LP, E>(X, KE);
            if (!nb) return;
            if (rv) k_solve_e<LP, true, MD, E><<<nb, 256, 0, st>>>(X);
            else k_solve_e<LP, false, MD, E><<<nb, 256, 0, st>>>(X);
        };
        if (X.epw == 4) go(std::integral_constant<int, 4>{});
        else if (X.epw == 2) go(std::integral_constant<int, 2>{});
        else go(std::integral_constant<int, 1>{});
    };
    // ring-1 redundancy (option ring1): the launch that runs after u is fresh on the ghosts
    // also computes the ghost vertices of owned edges (their edges are local, decomp.py),
    // exactly as their owners do; the edge kernels gather vorticity / pv_vertex there only
    const bool r1 = S.halo && S.ring1 && S.nVRing >= S.nVO;
    auto kvc1 = [&](const DevState& X) {
        DevState Y = X;
        if (!X.interior) Y.nVO = S.nVRing;  // the launch after the exchange (whole or boundary)
        kvc(Y);
    };
    if (r1) {
        HALO_RUN(S, st, kvc1, F_u);
        S.halo->wrote_ring1({F_vorticity, F_pv_vertex});
        HALO_WROTE(S, F_ke_vertex, F_divergence, F_ke);
    } else {
        HALO_RUN(S, st, kvc, F_u);
        HALO_WROTE(S, F_vorticity, F_pv_vertex, F_ke_vertex, F_divergence, F_ke);
    }
    if (hollingsworth) {
        HALO_RUN(S, st, kh, F_ke_vertex);
        HALO_WROTE(S, F_ke);
    }
    if (MD) {
        HALO_RUN_R1(S, st, ke, F_pv_vertex, F_rho_zz, F_u, F_pv_vertex);
        HALO_WROTE(S, F_h_edge, F_rho_edge, F_ke_edge, F_v, F_pv_edge);
    } else {
        HALO_RUN_R1(S, st, ke, F_pv_vertex, F_h, F_u, F_pv_vertex);
        HALO_WROTE(S, F_h_edge, F_ke_edge, F_v, F_pv_edge);
    }
    return hipGetLastError();
}
template <int LP>
static hipError_t solve_lp(const DevState& S, hipStream_t st, int hollingsworth, int rk_step) {
    return S.physics == 2 ? solve_lp_md<LP, true>(S, st, hollingsworth, rk_step)
                          : solve_lp_md<LP, false>(S, st, hollingsworth, rk_step);
}
hipError_t launch_solve_diagnostics(const DevState& S, hipStream_t st, int hollingsworth, int rk_step) {
    MPAS_LP_DISPATCH(S.LP, solve_lp, S, st, hollingsworth, rk_step);
}

}  // namespace mpas
