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
#include "k_cols.h"

#include <type_traits>

namespace mpas {

template <int LP, int EPW, bool MD, bool LIVE = false>
__global__ __launch_bounds__(256) void k_solve_vc(DevState S, int nVB, int hollingsworth_part) {
    solve_vc_body<LP, EPW, MD, LIVE>(S, nVB, hollingsworth_part, this_blk());
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

template <int LP, bool RECON_V, bool MD, int EPW, bool LIVE = false>
__global__ __launch_bounds__(256) void k_solve_e(DevState S) {
    solve_e_body<LP, RECON_V, MD, EPW, LIVE>(S, this_blk());
}

template <int LP, bool MD>
static hipError_t solve_lp_md(const DevState& S, hipStream_t st, int hollingsworth, int rk_step, int parts, int no_v) {
    // parts & 4 (atm_srk3 option ntu): the stored diagnostics the step's last stage reads, alone
    const bool live = (parts & 4) && !hollingsworth;
    auto kvc = [&](const DevState& X) {  // vertex blocks, then cell blocks
        auto go = [&](auto epw) {
            constexpr int E = decltype(epw)::value;
            const int nv = col_blocks_n<LP, E>(X, KV), nb = nv + col_blocks_n<LP, E>(X, KC);
            if (!nb) return;
            if (live) k_solve_vc<LP, E, MD, true><<<nb, 256, 0, st>>>(X, nv, hollingsworth);
            else k_solve_vc<LP, E, MD><<<nb, 256, 0, st>>>(X, nv, hollingsworth);
        };
        if (X.epw == 4) go(std::integral_constant<int, 4>{});
        else if (X.epw == 2) go(std::integral_constant<int, 2>{});
        else go(std::integral_constant<int, 1>{});
    };
    auto kh = [&](const DevState& X) {
        const int nb = col_blocks<LP>(X, KC);
        if (nb) k_solve_holl<LP><<<nb, 256, 0, st>>>(X);
    };
    auto ke = [&](const DevState& X) {
        const bool rv = !(rk_step != -1 && rk_step != 2) && !no_v;
        auto go = [&](auto epw) {
            constexpr int E = decltype(epw)::value;
            const int nb = col_blocks_n<LP, E>(X, KE);
            if (!nb) return;
            if (live && !rv) k_solve_e<LP, false, MD, E, true><<<nb, 256, 0, st>>>(X);
            else if (rv) k_solve_e<LP, true, MD, E><<<nb, 256, 0, st>>>(X);
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
    if (!(parts & 1)) {  // (the vertex / cell kernel ran in a combined launch, atm_srk3 hfuse)
    } else if (r1 && live) {
        HALO_RUN(S, st, kvc1, F_u);
        S.halo->wrote_ring1({F_pv_vertex});
        HALO_WROTE(S, F_ke);
    } else if (r1) {
        HALO_RUN(S, st, kvc1, F_u);
        S.halo->wrote_ring1({F_vorticity, F_pv_vertex});
        HALO_WROTE(S, F_ke_vertex, F_divergence, F_ke);
    } else if (live) {
        HALO_RUN(S, st, kvc, F_u);
        HALO_WROTE(S, F_pv_vertex, F_ke);
    } else {
        HALO_RUN(S, st, kvc, F_u);
        HALO_WROTE(S, F_vorticity, F_pv_vertex, F_ke_vertex, F_divergence, F_ke);
    }
    if (hollingsworth && (parts & 1)) {
        HALO_RUN(S, st, kh, F_ke_vertex);
        HALO_WROTE(S, F_ke);
    }
    if (!(parts & 2)) return hipGetLastError();
    if (MD && live && !(rk_step == -1 || rk_step == 2)) {
        HALO_RUN_R1(S, st, ke, F_pv_vertex, F_rho_zz, F_pv_vertex);
        HALO_WROTE(S, F_rho_edge, F_pv_edge);
    } else if (MD) {
        HALO_RUN_R1(S, st, ke, F_pv_vertex, F_rho_zz, F_u, F_pv_vertex);
        HALO_WROTE(S, F_h_edge, F_rho_edge, F_ke_edge, F_v, F_pv_edge);
    } else {
        if (live && !(rk_step == -1 || rk_step == 2)) {
            HALO_RUN_R1(S, st, ke, F_pv_vertex, F_pv_vertex);
            HALO_WROTE(S, F_pv_edge);
            return hipGetLastError();
        }
        HALO_RUN_R1(S, st, ke, F_pv_vertex, F_h, F_u, F_pv_vertex);
        HALO_WROTE(S, F_h_edge, F_ke_edge, F_pv_edge);
        if (!no_v && (rk_step == -1 || rk_step == 2)) HALO_WROTE(S, F_v);
    }
    return hipGetLastError();
}
template <int LP>
static hipError_t solve_lp(const DevState& S, hipStream_t st, int hollingsworth, int rk_step, int parts, int no_v) {
    return S.physics == 2 ? solve_lp_md<LP, true>(S, st, hollingsworth, rk_step, parts, no_v)
                          : solve_lp_md<LP, false>(S, st, hollingsworth, rk_step, parts, no_v);
}
hipError_t launch_solve_diagnostics(const DevState& S, hipStream_t st, int hollingsworth, int rk_step, int parts,
                                    int no_v) {
    MPAS_LP_DISPATCH(S.LP, solve_lp, S, st, hollingsworth, rk_step, parts, no_v);
}

// ---------------------------------------------------------------- combined launches
// Option "hfuse" (atm_srk3, reference semantics, undecomposed): two kernels of the step
// that neither read what the other writes share one grid (blocks [0, nb1) run the first
// body, the rest the second; k_cols.h), saving a dependent launch and overlapping the two
// tails -- the step is launch-bound on small meshes:
//   k_hf_damp_vc   the step's last divergence damping (from the div buffer, fusedamp) beside
//                  stage 2's solve_diagnostics vertex / cell kernel (it reads u only)
//   k_hf_e_finish  stage 2's solve_diagnostics edge kernel beside atm_rk_dynamics_substep_finish
//   k_hf_e_vi      stage 0's solve_diagnostics edge kernel beside stage 1's vert_imp
template <int LP, int EPW, bool TME>
__global__ __launch_bounds__(256) void k_hf_damp_vc(DevState S, double coef, int nb1, int nVB) {
    const int b = (int)blockIdx.x;
    if (b < nb1) divdamp_body<LP, 2, false, true, TME>(S, coef, Blk{b, nb1});
    else solve_vc_body<LP, EPW, false>(S, nVB, 0, Blk{b - nb1, (int)gridDim.x - nb1});
}
template <int EPW, bool RV>
__global__ __launch_bounds__(256) void k_hf_e_finish(DevState S, int nb1, int gx, int substep, int split, double inv,
                                                     Pair64 q, int norz) {
    const int b = (int)blockIdx.x;
    if (b < nb1) {
        solve_e_body<64, RV, false, EPW>(S, Blk{b, nb1});
    } else {
        const int r = b - nb1;
        const bool cells = r >= gx;
        finish64_body(S, substep, split, inv, q, cells, cells ? r - gx : r, gx, norz);
    }
}
template <int LP, int EPW>
__global__ __launch_bounds__(256) void k_hf_e_vi(DevState S, int nb1, double dtseps, double rcv, double c2) {
    const int b = (int)blockIdx.x;
    if (b < nb1) solve_e_body<LP, false, false, EPW>(S, Blk{b, nb1});
    else vert_imp_body<LP, false>(S, dtseps, rcv, c2, Blk{b - nb1, (int)gridDim.x - nb1});
}

static bool hf_ok(const DevState& S) { return !S.halo && S.physics == 0; }
template <int LP, class Fn>
static void epw_go(const DevState& S, Fn&& fn) {
    if (S.epw == 4) fn(std::integral_constant<int, 4>{});
    else if (S.epw == 2) fn(std::integral_constant<int, 2>{});
    else fn(std::integral_constant<int, 1>{});
}

template <int LP>
static hipError_t hf_damp_vc_lp(const DevState& S, hipStream_t st, double dts, int tme) {
    if (!hf_ok(S)) return hipErrorInvalidValue;
    const double coef = divdamp_coef(dts);
    const int nb1 = col_blocks_n<LP, 2>(S, KE);
    epw_go<LP>(S, [&](auto epw) {
        constexpr int E = decltype(epw)::value;
        const int nv = col_blocks_n<LP, E>(S, KV), nb2 = nv + col_blocks_n<LP, E>(S, KC);
        if (nb1 + nb2 == 0) return;
        if (tme) k_hf_damp_vc<LP, E, true><<<nb1 + nb2, 256, 0, st>>>(S, coef, nb1, nv);
        else k_hf_damp_vc<LP, E, false><<<nb1 + nb2, 256, 0, st>>>(S, coef, nb1, nv);
    });
    return hipGetLastError();
}
hipError_t launch_hf_damp_solve_vc(const DevState& S, hipStream_t st, double dts, int tme) {
    MPAS_LP_DISPATCH(S.LP, hf_damp_vc_lp, S, st, dts, tme);
}
hipError_t launch_hf_solve_e_finish(const DevState& S, hipStream_t st, int recon_v, int norz) {
    if (!hf_ok(S) || S.LP != 64) return hipErrorInvalidValue;
    const int gx = (stream_grid_((size_t)S.nEO * 32) + 3) / 4;
    hipError_t e = hipSuccess;
    epw_go<64>(S, [&](auto epw) {
        constexpr int E = decltype(epw)::value;
        const int nb1 = col_blocks_n<64, E>(S, KE);
        if (recon_v) k_hf_e_finish<E, true><<<nb1 + 2 * gx, 256, 0, st>>>(S, nb1, gx, 1, 1, 1.0, Pair64(S.L), norz);
        else k_hf_e_finish<E, false><<<nb1 + 2 * gx, 256, 0, st>>>(S, nb1, gx, 1, 1, 1.0, Pair64(S.L), norz);
    });
    return e == hipSuccess ? hipGetLastError() : e;
}
template <int LP>
static hipError_t hf_e_vi_lp(const DevState& S, hipStream_t st, double dts) {
    if (!hf_ok(S)) return hipErrorInvalidValue;
    const double dtseps = .5 * dts * (1.0 + kEpssm), rcv = kRgas / (kCp - kRgas), c2 = kCp * rcv;
    epw_go<LP>(S, [&](auto epw) {
        constexpr int E = decltype(epw)::value;
        const int nb1 = col_blocks_n<LP, E>(S, KE), nb2 = col_blocks<LP>(S, KC);
        if (nb1 + nb2) k_hf_e_vi<LP, E><<<nb1 + nb2, 256, 0, st>>>(S, nb1, dtseps, rcv, c2);
    });
    return hipGetLastError();
}
hipError_t launch_hf_solve_e_vert_imp(const DevState& S, hipStream_t st, double dts) {
    MPAS_LP_DISPATCH(S.LP, hf_e_vi_lp, S, st, dts);
}

}  // namespace mpas
