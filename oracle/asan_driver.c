/* asan_driver.c -- TEST INFRASTRUCTURE ONLY (race detection / sanitizers).
 *
 * Runs every task of the CPU oracle (mpas_oracle.c, included below so the driver sees its
 * registry) on a small synthetic state under -fsanitize=address,undefined: every field
 * array is its own heap allocation of exactly the reference layout's size, the float
 * fields come from the shared generator, and the connectivity is random ids in the range
 * the Q1 policy defines ([0, n]: n is the zero slot, as mpas_upload clamps) with random
 * list lengths up to the row width.  Any out-of-bounds access, use of uninitialised
 * heap, signed overflow or bad shift in the restatement aborts the run.
 *
 *   make -C oracle asan && oracle/_asan/asan_driver [nCells] [L] [seed]
 */
#include <stdio.h>

#include "mpas_oracle.c"

/* ids of each integer field: target entity kind (0 cell, 1 edge, 2 vertex), or -1 for a
 * count / mask (value range [0, hi]) -- mirrors id_target() of csrc/mpas_ctx.cpp */
static int id_kind(int f, int* hi) {
    switch (f) {
        case F_edgesOnCell: case F_edgesOnEdge: case F_edgesOnEdge_ECP: case F_edgesOnVertex: return 1;
        case F_cellsOnEdge: case F_advCellsForEdge: case F_cellsOnCell: case F_cellsOnVertex: return 0;
        case F_verticesOnEdge: case F_verticesOnCell: return 2;
        case F_nEdgesOnCell: *hi = 10; return -1;
        case F_nEdgesOnEdge: *hi = 20; return -1;
        case F_nAdvCellsForEdge: *hi = 15; return -1;
        case F_kiteForCell: *hi = 2; return -1;
        case F_bdyMaskCell: *hi = 7; return -1;
        default: *hi = 1; return -1;
    }
}

static uint64_t rng_state = 1;
static uint64_t rnd(void) { return rng_state = mpas_splitmix64(rng_state); }

int main(int argc, char** argv) {
    ora_state S;
    int nC = argc > 1 ? atoi(argv[1]) : 162;
    int L = argc > 2 ? atoi(argv[2]) : 7;
    rng_state = argc > 3 ? (uint64_t)atoll(argv[3]) : 20211015ULL;
    S.nCells = nC;
    S.nEdges = 3 * (nC - 2);
    S.nVertices = 2 * (nC - 2);
    S.L = L;
    const long n_of[3] = {S.nCells, S.nEdges, S.nVertices};
    for (int f = 0; f < F_COUNT; f++) {
        int kind = ora_fields[f].kind, W = ora_fields[f].width;
        long rows = 0, per = 0, esz = 8;
        switch (kind) {
            case C3: case C3B: rows = S.nCells + 1; per = L + 1; break;
            case C3V: rows = S.nCells + 1; per = (long)(L + 1) * W; break;
            case E3: rows = S.nEdges + 1; per = L + 1; break;
            case V3: rows = S.nVertices + 1; per = L + 1; break;
            case C2F: case C2I: rows = S.nCells + 1; per = W; break;
            case E2F: case E2I: rows = S.nEdges + 1; per = W; break;
            case V2F: case V2I: rows = S.nVertices + 1; per = W; break;
            case ZV: rows = 1; per = L + 1; break;
        }
        if (kind == C2I || kind == E2I || kind == V2I) esz = 4;
        if (kind == C3B) esz = 1;
        S.f[f] = calloc((size_t)(rows * per), (size_t)esz);
        if (!S.f[f]) return 2;
        if (kind == C2I || kind == E2I || kind == V2I) {
            int hi = 0, tk = id_kind(f, &hi);
            int32_t* p = (int32_t*)S.f[f];
            for (long r = 0; r + 1 < rows; r++)  /* row n: the zero slot stays 0 */
                for (long i = 0; i < per; i++)
                    p[r * per + i] = tk >= 0 ? (int32_t)(rnd() % (uint64_t)(n_of[tk] + 1)) : (int32_t)(rnd() % (uint64_t)(hi + 1));
        } else if (kind == C3B) {
            uint8_t* p = (uint8_t*)S.f[f];
            for (long r = 0; r + 1 < rows; r++)
                for (long i = 0; i < per; i++) p[r * per + i] = (uint8_t)(rnd() & 1);
        }
    }
    ora_fill_synthetic(&S, rng_state, 1);
    double out[31];
    const double dt = 720.0;
    /* every task of the path, both rk_step branches and both small_step branches */
    ora_atm_compute_solve_diagnostics(&S, 0, -1);
    ora_atm_compute_solve_diagnostics(&S, 1, 2);
    ora_atm_rk_integration_setup(&S);
    ora_atm_compute_moist_coefficients(&S);
    ora_atm_compute_vert_imp_coefs(&S, dt / 3);
    for (int hm = 0; hm < 3; hm++) {
        ora_atm_compute_dyn_tend_work(&S, 0, dt, hm, hm == 2 ? 0.5 : 0.0, 0, hm == 1);
        ora_atm_compute_dyn_tend_work(&S, 1, dt, hm, 0.0, 0, 0);
    }
    ora_atm_set_smlstep_pert_variables_work(&S);
    ora_atm_advance_acoustic_step_work(&S, dt / 3, 0);
    ora_atm_advance_acoustic_step_work(&S, dt / 3, 1);
    ora_atm_divergence_damping_3d(&S, dt / 3);
    ora_atm_rk_dynamics_substep_finish(&S, 1, 1);
    ora_atm_recover_large_step_variables_work(&S, 1, 0, dt);
    ora_atm_recover_large_step_variables_work(&S, 2, 2, dt);
    ora_mpas_reconstruct_2d(&S, 0, 1);
    ora_atm_compute_output_diagnostics(&S);
    ora_summarize_timestep(&S, 1, 1, out);
    ora_atm_compute_damping_coefs(&S, 22000.0, 0.2);
    ora_atm_compute_signs(&S);
    ora_atm_adv_coef_compression(&S);
    ora_atm_couple_coef_3rd_order(&S, 0.25);
    ora_atm_compute_mesh_scaling(&S, 1);
    ora_atm_init_coupled_diagnostics(&S);
    ora_mpas_vert_imp_coefs(&S, dt / 2);
    ora_mpas_acoustic_step(&S, dt / 2, 0);
    ora_mpas_acoustic_step(&S, dt / 2, 1);
    ora_mpas_recover(&S, 2, 2, dt);
    ora_mpas_advance_scalars_mono(&S, dt);
    ora_atm_srk3(&S, dt, 0);
    ora_atm_srk3(&S, dt, 1);
    ora_mpas_srk3_ex(&S, dt, 1, 1);
    /* the MPAS dynamics (option physics = 2) */
    ora_mpas_solve_diagnostics(&S, 0, -1);
    ora_mpas_solve_diagnostics(&S, 0, 2);
    ora_mpas_rk_integration_setup(&S);
    ora_mpas_moist_coefficients(&S);
    ora_mpas_dyn_tend(&S, 0, dt, 0, 0.0, 0, 1);
    ora_mpas_dyn_tend(&S, 1, dt, 2, 0.5, 0, 0);
    ora_mpas_set_smlstep(&S);
    ora_mpas2_acoustic_step(&S, dt / 3, 0);
    ora_mpas2_acoustic_step(&S, dt / 3, 1);
    ora_mpas_substep_finish(&S, 1, 1);
    ora_mpas_surface_pressure(&S);
    ora_mpas_srk3_dyn(&S, dt, 1, 1, 2);
    for (int f = 0; f < F_COUNT; f++) free(S.f[f]);
    printf("asan_driver: every oracle task ran clean (nCells %d, L %d)\n", nC, L);
    return 0;
}
