/* mpas_dyn.h -- C-ABI of libmpasdyn, the MI355X (gfx950) drop-in for the RK3 dynamics
 * hot path of alexaiken/mpas-regent (dynamics/rk_timestep.rg:361-519 and the leaf
 * tasks of dynamics/dynamics_tasks.rg).
 *
 * Boundary.  Each Regent leaf task of the path becomes one extern "C" entry point with
 * the task's name (prefixed mpas_) and its scalar parameters in the task's order.  The
 * task's region arguments (cr, cpr, er, vr, vert_r) are the device-resident state owned
 * by an mpas_ctx; fields move across the boundary with mpas_upload / mpas_download,
 * which take a plain host pointer and byte strides, so the Legion SOA layout a Regent
 * binding would hand over (legion_accessor_array_*_raw_rect_ptr: entity stride, level
 * stride; fortran/examples.rg:21-46) is accepted as is.  Field ids are the Regent field
 * names (data_structures.rg), looked up with mpas_field_id.
 *
 * Conventions.  Every function returns 0 on success or a negative MPAS_E* code; the
 * message is in mpas_last_error(ctx).  No C++ exception crosses the ABI.  A context owns
 * one HIP device and its streams and is single-threaded; separate contexts may be
 * driven from separate host threads.  Task calls are stream-ordered (asynchronous);
 * mpas_sync waits.  The host arrays passed to upload/download are borrowed for the call.
 * There is no CPU fallback: without a usable gfx950 device mpas_ctx_create fails.
 */
#ifndef MPAS_DYN_H
#define MPAS_DYN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPAS_OK 0
#define MPAS_EINVAL (-1)
#define MPAS_EHIP (-2)
#define MPAS_ERCCL (-3)
#define MPAS_ENOMEM (-4)
#define MPAS_ENOTSUP (-5)
/* bounds-checked build only (libmpasdyn_bounds.so, `make -C mpas-regent_amd/csrc bounds`):
 * a kernel of the call accessed a field outside its rows; the message names the field.
 * Option "bounds" (read-only) is 1 in that build; "bounds_units" (read-only) packs the
 * translation units whose kernels check (high 32 bits) and those registered (low);
 * "bounds_probe" = n makes it read field u n columns past its end (the check's own test). */
#define MPAS_EBOUNDS (-6)

typedef struct mpas_ctx mpas_ctx;

/* mesh dimensions; constants.rg:18-26 (nCells, nEdges, nVertices, nVertLevels) */
typedef struct {
    int32_t nCells;
    int32_t nEdges;
    int32_t nVertices;
    int32_t nVertLevels; /* L; fields carry L+1 levels (main.rg:21-24), L+1 <= 64 */
} mpas_dims;

/* ---- context and residency ---------------------------------------------------- */
int mpas_ctx_create(mpas_ctx** out, int device, const mpas_dims* dims);
int mpas_ctx_destroy(mpas_ctx* ctx);
const char* mpas_last_error(const mpas_ctx* ctx);
int mpas_sync(mpas_ctx* ctx);
/* the HIP stream (hipStream_t) the tasks run on, for callers that time with events */
int mpas_get_stream(mpas_ctx* ctx, void** stream);
/* options: "exact" = 1 makes the reassociated kernels (Q10 q sum, acoustic scan, set_smlstep's
 * slope-flux sum) evaluate the reference's literal order (bit-identical to the oracle, slower);
 * "xcd" = 0 dispatcher block order, 1 one contiguous eighth of the columns per XCD,
 * G > 1 runs of G blocks per XCD inside windows of 8G (default 64); "epw" = 1, 2 (default)
 * or 4 entities per column slot in div_damping / solve_diagnostics; "cve" = 1, 4 or 8
 * vertices per wavefront in dyn_tend's delsq_vorticity (default 0: 4); "vcmix" = 1 (default)
 * interleaves the vertex and cell blocks of the mixed grids; "overlap" = 1 (default)
 * computes interior entities beside the halo exchange of a decomposed mesh; "self" = 0
 * disables the SELF gathers; "graph" = 1 (default) makes mpas_atm_srk3 capture its step once
 * per (dt, schedule) as a HIP graph and replay it (any option change or mesh upload
 * re-captures; per-task timing runs the launches directly; read-only "graph_captures" /
 * "graph_launches" count them).  "graph_halo" does the same on a decomposed context: 2
 * (default) with the stub transport, 1 with the RCCL transport too (opt-in: its grouped
 * send / recv has been captured on a 1-rank communicator only), 0 never; a step is
 * captured per halo state at its start (a start state met twice; up to 4 kept), and a
 * capture the transport refuses falls back to eager steps (read-only "graph_fallbacks").  "stub_latency_us" (stub transport only) adds a
 * device-side wait of that many microseconds to every exchange (tools/rank_sim.py).  All but
 * "exact" and "physics" change only speed, never results.
 * Cross-task fusion in mpas_atm_srk3 (reference semantics):
 * "fusedamp" = 1 (default) applies each divergence damping inside the next acoustic launch
 * (read-only "fusedamp_active"); "fusesml" = 1 (default, with fusedamp) runs each stage's
 * set_smlstep inside its first acoustic launch; "smlsum" = 1 (default, with fusesml, exact = 0)
 * forms set_smlstep's slope-flux sum once per step (u_tend, zb_cell and zb3_cell are not written
 * within a step) and the stages' fused set_smlstep read it; "fusesetup" = 1 (default) runs setup, moist
 * and stage 0's vert_imp as one launch; "fusecopy" = 1 (default, with fusesetup) makes
 * setup's edge copies in stage 0's dyn_tend edge kernel (decomposed contexts and every
 * "physics" mode too); "defer4" = 1
 * (default) applies rk_step 0's del4 of tend_u_euler (dyn_tend kernel D) in the next stage's
 * rk_step > 0 edge kernel; "vdyn" = 1 (default) has the last stage's dyn_tend edge kernel store
 * solve_diagnostics' v from the u it gathers (when edgesOnEdge_ECP = edgesOnEdge, read-only
 * "eoe_same"); "ntu" = 1 (default; reference semantics, with defer4) leaves out what the stages
 * before the step's last would compute only for values no task reads before the last stage
 * rewrites them: their dyn_tend forms no tend_u and no theta tendencies (tend_theta,
 * tend_rtheta_adv, rthdynten), the last acoustic substep of stages 0 and 1 stores no rho_pp,
 * rtheta_pp, rw_p or wwAvg (the next stage's first substep sets them; the damping reads the div
 * that substep stores), stage 0's solve_diagnostics is not run and stage 1's stores ke and
 * pv_edge alone (its divergence, vorticity, h_edge and ke_edge are dead); every field after a step
 * is bit-identical with it off; 2 = the same with stage 1's solve_diagnostics whole, 3 = with the
 * acoustic state stored (A/Bs);
 * "etile" = 1 (default 0, measured, not kept) forms dyn_tend's theta advection fluxes from tiles
 * of cells in LDS ("etcells", "etclo", "etmode", "etthreads"; read-only "etile_active");
 * "bsplit" (fast path, speed only) puts dyn_tend's per-edge theta flux (and the MPAS dynamics' w
 * flux) in an edge kernel of its own beside the edge kernel B: 1 always, 2 (default) under
 * "physics" = 2 only, where B's registers would otherwise hold it to 3 waves per SIMD, 0 never.
 * "keep_check" = 1 (default 0; debug, slow) compares every field's keep tail -- the value of
 * each column's slot the reference never writes, which the kernels store back so that every
 * column is written as whole lines -- with the field after every task and fails the task
 * (MPAS_EINVAL, naming the task, the field and the first entity) on a mismatch.  "tmedge" = 1 (default 0) has
 * dyn_tend store theta_m(cell1) + theta_m(cell2) per edge for the acoustic substeps;
 * "hfuse" = 1 puts independent neighbouring kernels in one launch, 2 (default) only below
 * 16384 owned cells, undecomposed (read-only "hfuse_active"). "fusedamp_halo" = 1 (default)
 * applies fusedamp and fusesml on decomposed meshes too (with "ring1"): the div is exchanged
 * where rtheta_pp was.  Under "physics" >= 1 "fusesetup" runs setup, moist and stage 0's
 * vert_imp in their MPAS forms as one launch.
 * "physics" = 1 selects the MPAS vertical solver: vert_imp with Q16/Q17
 * fixed, the acoustic step with the ru_p update (Q18), the MPAS statement order (Q19/Q20)
 * and the tridiagonal back substitution (Q21), tend_rt = tend_theta (Q8), recover_large_step
 * with Q24 fixed, and in mpas_atm_srk3 number_sub_steps acoustic substeps (Q5) followed by
 * recover (Q7); every other task as the reference.
 * "physics" = 2 adds the MPAS dynamics (every remaining quirk of the path fixed, so the JW
 * state evolves as a dynamical core): dyn_tend with the w tendency in tend_w computed from
 * the state w (Q8, Q13, Q14), q once (Q10), the MPAS curvature (Q12) and wdtz (Q15);
 * solve_diagnostics with h = rho_zz, rho_edge = h_edge, divergence sign*u (Q9) and v over
 * every edgesOnEdge entry (Q23); set_smlstep on tend_u / tend_w (Q2); setup also saving
 * theta_m_save; moist setting cqu (Q25); mpas_reconstruct_2d after the RK loop; the substep
 * finish keeping rho_zz; atm_compute_output_diagnostics also writing surface_pressure.
 * Default 0: the reference's semantics.
 * "transport" = 1 (needs "physics" >= 1) makes mpas_atm_srk3 copy scalars
 * to scalars_old first and run mpas_atm_advance_scalars_mono(dt) after the last stage's
 * recover, before atm_rk_dynamics_substep_finish.  Default 0.  "trorder" (speed only)
 * orders the transport's column slots: 0 entity-major, 1 pair-major, R >= 2 pair-major
 * within runs of R consecutive entities, one run per XCD (default 64); "trorder_e" the same
 * for the transport's edge kernel alone (0, the default: trorder's).  "trsu" = 1 (speed only; measured
 * slower, default 0): the transport's update forms the upwind update su again instead of
 * storing and reading it.  "trsave" = 1 (default; speed only) folds mpas_atm_srk3's scalars_save
 * copy into the transport (undecomposed, the default transport kernels): they read the old scalars
 * from scalars and the bounds kernel stores scalars_old.  "mdamp" = 1 (default; speed only; the MPAS
 * forms) applies each divergence damping in the kernel that next reads ru_p (the next substep's ru_p
 * kernel, the stage's recover edge kernel); "mru" = 1 (default; the MPAS dynamics, fast path) has
 * the kernel forming a stage's final tend_u store its first acoustic substep's ru_p and ruAvg;
 * "msml" = 1 (default; the MPAS dynamics) applies each stage's set_smlstep in dyn_tend's cell
 * kernel.  "trepw" = 2 (speed only; measured within 2 %, default 1): two
 * edges per wavefront in the transport's edge kernel.  "trtile" = 1
 * (speed only, default 0) runs the transport as two tiled kernels with the scalars of
 * compact cell tiles in LDS and no edge scratch, when every cell has at most 6 edges with
 * at most 9 advCells each (bit-identical; measured slower); "trtcells" and
 * "trtclo" bound a tile's cells (default 16) and LDS columns (default 96); read-only
 * "trtile_active" / "trtile_count" report whether tiles are built and how many.
 * "tredge" = 1 (speed only, default 0) stages each group of 16 consecutive edges' scalars_old
 * columns in LDS for the transport's edge kernel (bit-identical; measured slower, DESIGN.md
 * §7; read-only "tredge_active", "tredge_irregular").  On a decomposed context the tiles are built only with "trtile_ghosts" = 1, which declares that
 * the ghosts close over advCellsForEdge(edgesOnCell) (mpasdyn.decomp.Decomposition(...,
 * tiled_transport=True); lib.setup_subdomain sets it). */
int mpas_set_option(mpas_ctx* ctx, const char* name, int64_t value);
/* reads every option above ("self", default 1: when every cell is
 * among the cellsOnEdge of its own edges -- mpas-mode ids -- the cell kernels gather
 * only the other cell of an edge) and "selfc" (read-only: whether the SELF gathers are
 * in use for the uploaded mesh). */
int mpas_get_option(mpas_ctx* ctx, const char* name, int64_t* value);

/* field registry (include/mpas_fields.def order) */
int mpas_field_count(void);
int mpas_field_id(const char* name);
const char* mpas_field_name(int field_id);
int mpas_field_kind(int field_id);  /* 0 C3,1 C3V,2 E3,3 V3,4 C2F,5 C2I,6 E2F,7 E2I,8 V2F,9 V2I,10 C3B,11 ZV */
int mpas_field_width(int field_id);

/* Host <-> device copy of one field.  Element (entity e, level k, component i) is at
 * byte offset e*stride_entity + k*stride_level + i*stride_comp of host (levels 0..L,
 * entities 0..n-1; components only for array fields).  Element type: double for fp64
 * fields, int32 for integer fields, uint8 for masks.  Entity-id fields are clamped
 * on upload so that any id outside [0, n] resolves to the zero slot n; a list
 * length (nEdgesOnCell, nEdgesOnEdge, nAdvCellsForEdge) past its row width is refused.
 * The view may be device memory (a Legion instance in framebuffer memory, a torch tensor;
 * hipPointerGetAttributes decides): 3-D fields then move device to device with a strided
 * copy kernel, never through the host (non-negative strides); 2-D fields are staged. */
int mpas_upload(mpas_ctx* ctx, int field_id, const void* host, int64_t stride_entity, int64_t stride_level,
                int64_t stride_comp);
int mpas_download(mpas_ctx* ctx, int field_id, void* host, int64_t stride_entity, int64_t stride_level,
                  int64_t stride_comp);
/* Fill every synthetic-distribution field (mpas_fields.def DIST != M) on the device
 * with the counter-based generator of mpas_synth.h (benchmark inputs). */
int mpas_fill_synthetic(mpas_ctx* ctx, uint64_t seed);

/* ---- the hot-path tasks (dynamics_tasks.rg) ------------------------------------ */
/* :747  atm_rk_integration_setup(cr, er) */
int mpas_atm_rk_integration_setup(mpas_ctx* ctx);
/* :460  atm_compute_moist_coefficients(cr, er) */
int mpas_atm_compute_moist_coefficients(mpas_ctx* ctx);
/* :513  atm_compute_vert_imp_coefs(cr, vert_r, dts) */
int mpas_atm_compute_vert_imp_coefs(mpas_ctx* ctx, double dts);
/* :814  atm_compute_dyn_tend_work(cr, er, vr, vert_r, rk_step, dt, config_horiz_mixing,
 *       config_mpas_cam_coef, config_mix_full, config_rayleigh_damp_u);
 *       horiz_mixing: 0 "2d_smagorinsky", 1 "2d_fixed", 2 other */
int mpas_atm_compute_dyn_tend_work(mpas_ctx* ctx, int rk_step, double dt, int config_horiz_mixing,
                                   double config_mpas_cam_coef, int config_mix_full, int config_rayleigh_damp_u);
/* :1503 atm_set_smlstep_pert_variables_work(cpr, er, vert_r); cpr = field cprMask */
int mpas_atm_set_smlstep_pert_variables_work(mpas_ctx* ctx);
/* :1546 atm_advance_acoustic_step_work(cr, er, vert_r, dts, small_step) */
int mpas_atm_advance_acoustic_step_work(mpas_ctx* ctx, double dts, int small_step);
/* :1726 atm_divergence_damping_3d(cpr, er, dts); cpr's isShared = field isShared */
int mpas_atm_divergence_damping_3d(mpas_ctx* ctx, double dts);
/* :328  atm_compute_solve_diagnostics(cr, er, vr, hollingsworth, rk_step) */
int mpas_atm_compute_solve_diagnostics(mpas_ctx* ctx, int hollingsworth, int rk_step);
/* :1951 atm_rk_dynamics_substep_finish(cr, er, dynamics_substep, dynamics_split) */
int mpas_atm_rk_dynamics_substep_finish(mpas_ctx* ctx, int dynamics_substep, int dynamics_split);

/* ---- operators defined beside the RK3 loop but not run inside it ------------------ */
/* :1766 atm_recover_large_step_variables_work(cr, er, vert_r, ns, rk_step, dt); commented
 *       out of atm_srk3 (rk_timestep.rg:460, Q7); Q24 literal */
int mpas_atm_recover_large_step_variables_work(mpas_ctx* ctx, int ns, int rk_step, double dt);
/* :1893 mpas_reconstruct_2d(cr, er, includeHalos, on_a_sphere); atm_core_init
 *       (atm_core.rg:33); commented out of atm_srk3 (rk_timestep.rg:487) */
int mpas_reconstruct_2d(mpas_ctx* ctx, int includeHalos, int on_a_sphere);
/* :729 atm_compute_output_diagnostics(cr), main.rg:70 after the time loop: rho = rho_zz * zz,
 *       pressure = pressure_base + pressure_p on levels 0..nVertLevels-1 (theta is in the
 *       task's write set but its statement is commented out in the reference: unchanged) */
int mpas_atm_compute_output_diagnostics(mpas_ctx* ctx);
/* init_atm_case_jw (vertical_init/init_atm_cases.rg:366-432), host side, no context: the
 * per-column hydrostatic iteration of the JW initial state (10 temperature x 25 pressure
 * passes) for nCells columns of nVertLevels levels, arrays [cell][level] row-major:
 * latCell[nCells]; pb, rb, zz (base pressure, base density, zz) in; dzw, dzu, fzm, fzp the
 * vertical grid (length nVertLevels+1); pressure_p, rho_p, temperature out.  Split over
 * nthreads host threads (<= 0: all).  mpasdyn/jw.py calls it for the large meshes. */
int mpas_jw_hydrostatic(int32_t nCells, int32_t nVertLevels, const double* latCell, const double* pb,
                        const double* rb, const double* zz, const double* dzw, const double* dzu, const double* fzm,
                        const double* fzp, double* pressure_p, double* rho_p, double* temperature, int32_t nthreads);
/* One-time tasks of atm_core_init (atm_core.rg:22-42) that run on the device:
 * :274 atm_compute_damping_coefs(config_zd, config_xnutr, cr) (atm_core.rg:41, defaults
 *       22000.0 and 0.2): dss of the upper damping layer */
int mpas_atm_compute_damping_coefs(mpas_ctx* ctx, double config_zd, double config_xnutr);
/* :651 atm_init_coupled_diagnostics(cr, er, vert_r) (atm_core.rg:31): rho_zz /= zz, ru, rw,
 *       rho_p, rtheta_base, rtheta_p, exner, exner_base, pressure_p, pressure_base */
int mpas_atm_init_coupled_diagnostics(mpas_ctx* ctx);
/* The mesh tasks of atm_core_init (k_mesh.hip; ids compared as uploaded, the bounds the
 * reference leaves undefined as oracle/mpas_oracle.c states them; a decomposed context
 * computes its owned entities, its ghosts keep the uploaded values):
 * :46  atm_compute_signs(cr, er, vr) (atm_core.rg:22): edgesOnVertexSign, edgesOnCellSign,
 *       kiteForCell; zb_cell / zb3_cell (:88-110, the copy of er.zb / zb3 that
 *       init_atm_case_jw writes) stay as uploaded: the state keeps no er.zb, the host that
 *       builds the initial state uploads the copy (mpasdyn/jw.py) */
int mpas_atm_compute_signs(mpas_ctx* ctx);
/* :133 atm_adv_coef_compression(cr, er) (atm_core.rg:24): advCellsForEdge,
 *       nAdvCellsForEdge (the index of the list's last cell, :184), adv_coefs and
 *       adv_coefs_3rd from cellsOnCell, dcEdge, dvEdge and deriv_two (never initialised by
 *       the reference, Q2: upload zeros for its semantics) */
int mpas_atm_adv_coef_compression(mpas_ctx* ctx);
/* :303 atm_couple_coef_3rd_order(config_coef_3rd_order, cr, er) (atm_core.rg:27, 0.25):
 *       adv_coefs_3rd and zb3_cell (level 0) scaled */
int mpas_atm_couple_coef_3rd_order(mpas_ctx* ctx, double config_coef_3rd_order);
/* :595 atm_compute_mesh_scaling(cr, cpr, csr, cgr, er, config_h_ScaleWithMesh)
 *       (atm_core.rg:39, true): meshScalingDel2 / Del4 from meshDensity (the regional
 *       relaxation factors it also writes are read by no task of the path) */
int mpas_atm_compute_mesh_scaling(mpas_ctx* ctx, int config_h_ScaleWithMesh);
/* atm_core.rg:22 atm_core_init: every task in the reference's order -- compute_signs,
 *       adv_coef_compression, couple_coef_3rd_order(0.25), init_coupled_diagnostics,
 *       solve_diagnostics(hollingsworth = false, rk_step = -1), mpas_reconstruct_2d(false,
 *       true), compute_mesh_scaling(true), compute_damping_coefs(config_zd = 22000,
 *       config_xnutr = 0.2; constants.rg:103-104).  physics_init is a stub (OUT OF SCOPE).
 *       Needs the raw mesh uploaded: connectivity (incl. cellsOnCell, cellsOnVertex),
 *       dcEdge, dvEdge, deriv_two, meshDensity. */
int mpas_atm_core_init(mpas_ctx* ctx);
/* Monotonic scalar transport.  Replaces no reference entry point: the
 *       reference has none (Q26 -- scalars:double[8], data_structures.rg:36, is declared and
 *       never used; the north star names the transport).  MPAS-A's atm_advance_scalars_mono
 *       (flux-corrected transport): the 8 scalars of scalars_old are advected over dt by the
 *       mass fluxes ruAvg (edges) and wwAvg (interfaces) from density rho_zz_old_split to
 *       rho_zz with 3rd-order fluxes (adv_coefs, adv_coefs_3rd; flux3 vertically, coef 0.25)
 *       limited so that no new extrema appear; result in scalars (levels 0..nVertLevels-1).
 *       Statement order: oracle/mpas_oracle.c ora_mpas_advance_scalars_mono.  Decomposed
 *       contexts exchange scalars_old and the scratch on their ghosts like every task. */
int mpas_atm_advance_scalars_mono(mpas_ctx* ctx, double dt);
/* rk_timestep.rg:29 summarize_timestep(cr, er, config_print_detailed_minmax_vel,
 *       config_print_global_minmax_vel, config_print_global_minmax_sca): the values the
 *       reference prints, into out[31] (host memory; the call synchronises):
 *       out[0..24] five records {value, index, k, lat_deg, lon_deg}: min w, max w, min u,
 *       max u, max wind speed; out[25], out[26] NaN seen in w, u; out[27..30] the
 *       regentlib min/max folds from 0.0 of w and of u.  Blocks whose flag is 0 stay 0
 *       (the reference calls it with every flag false, rk_timestep.rg:492). */
int mpas_summarize_timestep(mpas_ctx* ctx, int config_print_detailed_minmax_vel, int config_print_global_minmax_vel,
                            int config_print_global_minmax_sca, double* out);

/* ---- the driver (rk_timestep.rg:361-500) ---------------------------------------- */
/* schedule 0: the reference's atm_srk3 (Q4: rk_sub_timestep[rk_step] truncated into
 * dyn_tend's rk_step; Q5: n+1 acoustic substeps); schedule 1: dyn_tend rk_step = 0,1,2
 * (the MPAS schedule used by the benchmark). */
int mpas_atm_srk3(mpas_ctx* ctx, double dt, int schedule);
/* rk_timestep.rg:503 atm_timestep = atm_srk3 with the reference schedule */
int mpas_atm_timestep(mpas_ctx* ctx, double dt);

/* ---- horizontal decomposition (rk_timestep.rg runs on Legion partitions) --
 * A context may hold one subdomain: the local entities are its owned ones first, then
 * its ghosts (everything its owned entities reach through an index array), then the
 * zero slot; mpasdyn/decomp.py builds the local state and the plan.  Every task then
 * computes owned entities only, and before each kernel the fields it gathers that an
 * earlier kernel wrote are exchanged on the ghosts (RCCL send/recv per peer, or the
 * in-process loopback).  Every rank must call the same tasks in the same order. */
/* owned counts (the first entities of each kind); default: all local entities */
int mpas_halo_owned(mpas_ctx* ctx, int32_t nCellsOwned, int32_t nEdgesOwned, int32_t nVerticesOwned);
/* the first n*Interior owned entities of each kind reach no ghost through any index array
 * (mpasdyn/decomp.py numbers them first): a kernel whose gathered fields need an exchange
 * then computes them while the exchange runs on the context's halo stream, and the
 * remaining (boundary) owned entities after it (SURVEY §8.6 overlap; option "overlap") */
int mpas_halo_interior(mpas_ctx* ctx, int32_t nCellsInterior, int32_t nEdgesInterior, int32_t nVerticesInterior);
/* ring-1 ghosts (mpasdyn/decomp.py numbers them first among the ghosts): local edges
 * [0, nEdgesRing1) are the owned edges and the ghost edges of owned cells, local vertices
 * [0, nVerticesRing1) the owned vertices and the ghost vertices of owned edges.  With
 * option "ring1" (default 1) atm_divergence_damping_3d (reference semantics) also updates
 * those edges and atm_compute_solve_diagnostics those vertices, from inputs fresh there,
 * so the acoustic step's ru_p and the edge kernels' vorticity / pv_vertex gathers need no
 * halo exchange.  Every rank must make the same call. */
int mpas_halo_ring1(mpas_ctx* ctx, int32_t nEdgesRing1, int32_t nVerticesRing1);
/* kind 0 cells, 1 edges, 2 vertices: columns this rank sends to / receives from `peer`,
 * as local ids, in the order the peer receives / sends them */
int mpas_halo_plan(mpas_ctx* ctx, int kind, int peer, const int32_t* send_ids, int32_t nsend,
                   const int32_t* recv_ids, int32_t nrecv);
/* global id of every local entity of `kind` (n = local count): mpas_fill_synthetic then
 * generates the same values as on the undecomposed mesh */
int mpas_set_global_ids(mpas_ctx* ctx, int kind, const int32_t* gids, int32_t n);
/* transports: RCCL (one process per GPU; rank 0 makes the 128-byte id, the caller
 * broadcasts it) or loopback (n contexts of one process on one device, rank = index,
 * each driven by its own host thread) */
int mpas_rccl_unique_id(void* id128);
/* (after every mpas_halo_plan call of the context: the transports size their buffers) */
int mpas_halo_rccl(mpas_ctx* ctx, int nranks, int rank, const void* id128);
int mpas_halo_loopback(mpas_ctx** ctxs, int n);
/* host-staged TCP transport: nranks processes (they may share one device -- RCCL refuses
 * two ranks on one GPU), rank r listening on host:base_port + r; each exchange copies the
 * packed regions to the host, swaps them with the peers over the sockets and copies them
 * back (synchronous; never captured in a graph).  The multi-process test of the same
 * plan / pack / unpack code the RCCL transport runs (tests/test_gpu_multiproc.py). */
int mpas_halo_socket(mpas_ctx* ctx, int nranks, int rank, const char* host, int base_port);
/* stub transport (measurement only): every exchange packs the send columns of each peer,
 * stands in for the wire with one device copy of the received bytes out of the send
 * buffer, and unpacks -- one rank's whole launch sequence on one GPU, everything but the
 * wire time; the ghosts do NOT receive their neighbours' values */
int mpas_halo_stub(mpas_ctx* ctx);
/* halo exchanges made so far and fields moved by them */
int mpas_halo_stats(mpas_ctx* ctx, int64_t* exchanges, int64_t* fields);

/* ---- instrumentation ------------------------------------------------------------ */
/* With timing on, every task call is bracketed by HIP events on the task stream and its
 * device time accumulated per task name; mpas_timing_get returns calls and total ms. */
int mpas_timing_enable(mpas_ctx* ctx, int on);
int mpas_timing_reset(mpas_ctx* ctx);
int mpas_timing_count(mpas_ctx* ctx);
int mpas_timing_get(mpas_ctx* ctx, int idx, const char** name, int64_t* calls, double* total_ms);

#ifdef __cplusplus
}
#endif
#endif
