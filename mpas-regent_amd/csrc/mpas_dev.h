// mpas_dev.h -- device-side state layout and kernel launchers of libmpasdyn (gfx950).
//
// Device layout (HBM), chosen for one wavefront per column:
//   C3/E3/V3   f[entity * LP + lpos(k)]            k = 0..L   (LP = pow2 >= L+1, <= 64)
//              (width W > 1, transport scratch only: f[(entity * W + i) * LP + lpos(k)])
//   C3V        f[(entity * W + i) * LP + lpos(k)]  (zb_cell / zb3_cell: coalesced per component)
//   C2*/E2*/V2* f[entity * W + i]                  (2-D mesh data)
//   C3B        uint8 f[entity * LP + lpos(k)]
//   ZV         f[k]                          (vertical_fs, LP entries)
// Every entity array has nEntity+1 rows; row nEntity is the all-zero, never-written
// "zero slot" that raw 1-based MPAS ids equal to nEntity resolve to.
// A column of LP lanes holds one entity's levels: lane k <-> level k, so a gathered
// neighbour column is one contiguous 8*(L+1)-byte read and vertical neighbours are
// register shuffles within the LP-lane segment.
// Level k sits at position lpos(k) of its column: k itself below LP = 64; at LP = 64 the
// levels are interleaved in pairs, position 2j = level j, 2j+1 = level j+32, so that one
// 16-B lane load by a wavefront fetches TWO columns (lanes 0-31 one, lanes 32-63 the
// other) and one permlane32_swap per dword returns both to lane = level (gather2 below):
// the gathers cost per load instruction, not per byte.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpas {

__host__ __device__ constexpr int lpos(int LP, int k) { return LP == 64 ? (((k & 31) << 1) | (k >> 5)) : k; }
__host__ __device__ constexpr int plev(int LP, int p) { return LP == 64 ? ((p >> 1) | ((p & 1) << 5)) : p; }  // inverse

// Element (entity e, component i, level k) of a multi-component 3-D field.  The x8 fields
// (the transport's scalars and its scratch, width kPairW) store an entity's scalars in
// pairs: scalars 2q and 2q+1 at level k are ONE 16-B element of pair column e * 4 + q, at
// position k -- a wavefront loads both scalars of its levels with one 16-B load per lane
// from a wave-uniform base (no lane exchange, no per-lane column select; k_transport.hip).
// Other widths (zb_cell / zb3_cell) keep one column per component in the lpos order.
constexpr int kPairW = 8;
__host__ __device__ constexpr size_t vidx(int W, int LP, size_t e, int i, int k) {
    return W == kPairW ? ((e * (kPairW / 2) + (size_t)(i >> 1)) * LP + (size_t)k) * 2 + (size_t)(i & 1)
                       : (e * W + (size_t)i) * LP + (size_t)lpos(LP, k);
}

enum FieldKind { K_C3, K_C3V, K_E3, K_V3, K_C2F, K_C2I, K_E2F, K_E2I, K_V2F, K_V2I, K_C3B, K_ZV };
enum FieldDist { D_U = 0, D_Z = 1, D_B = 2, D_M = 3, D_S = 4 };

enum FieldId {
#define MPAS_FIELD(name, KIND, W, DIST, LO, HI) F_##name,
#include "mpas_fields.def"
#undef MPAS_FIELD
    F_COUNT,
    // derived mesh arrays (computed at upload time, glibc cos on the host)
    X_cosAngleEdge = F_COUNT,
    X_cosLatEdge,
    X_cosLatCell,
    X_sinLatCell,  // (mpas_reconstruct_2d)
    X_cosLonCell,
    X_sinLonCell,
    // per-cell copies of edge data seen through edgesOnCell (mesh constants computed
    // on the device after upload, k_prepare): one indirection level less per gather
    X_ce_c1,    // cellsOnEdge(edgesOnCell(i,c), 0)      C2I x10
    X_ce_c2,    // cellsOnEdge(edgesOnCell(i,c), 1)      C2I x10
    X_ce_dv,    // dvEdge(edgesOnCell(i,c))              C2F x10
    X_ce_dc,    // dcEdge(edgesOnCell(i,c))              C2F x10
    X_ve_dc,    // dcEdge(edgesOnVertex(i,v))            V2F x3
    X_ce_idc,   // invDcEdge(edgesOnCell(i,c))           C2F x10
    X_ce_msd2,  // meshScalingDel2(edgesOnCell(i,c))     C2F x10
    X_ce_msd4,  // meshScalingDel4(edgesOnCell(i,c))     C2F x10
    X_ce_oth,   // the cell of cellsOnEdge(edgesOnCell(i,c), 0:1) that is not c   C2I x10
    X_ce_s1,    // 1 if cellsOnEdge(edgesOnCell(i,c), 0) == c                     C2I x10
    X_eB,       // per edge, the index lists of dyn_tend's edge kernel in one record:
                // cellsOnEdge(2), edgesOnEdge(10), advCellsForEdge(9), nEdgesOnEdge,
                // nAdvCellsForEdge, 0 -- one scalar round trip instead of three   E2I x24
    X_cR,       // per cell, one record of its first NF edges: edgesOnCell(NF), cell1(NF),
                // cell2(NF) of each, nEdgesOnCell, 0                             C2I x(3NF+2)
    X_cRs,      // the same for the SELF path: edgesOnCell(NF), other cell(NF),
                // "cell is cell1"(NF), nEdgesOnCell, 0                           C2I x(3NF+2)
    X_wfl,      // dyn_tend's w-advection flux_arr over the advCells of the cell's last
                // edge, sum_j (adv_coefs + s adv_coefs_3rd) * 0.0 for s = +1, -1      C2F x2
    // scratch (not reference fields)
    X_wc,       // w after zeroing, horizontal advection and curvature (dyn_tend :1170-1218);
                // the U section still reads the pre-zeroing w (:1013)
    X_F,        // flux_arr of the theta advection (:1333-1340) per edge and level: it
                // depends only on the edge, so it is formed once per edge, not per cell
    X_Fw,       // the same for the w advection of the MPAS dynamics (physics = 2: every
                // edge's flux_arr over the state w, :1174-1205 without Q13)
    // deferred divergence damping (option "fusedamp", k_acoustic.hip MODE 2): the damping
    // of an acoustic substep is applied by the next acoustic substep as it reads ru_p
    X_dvA,      // div = -(rtheta_pp - rtheta_pp_old) of the substep (:1755), per cell    C3
    X_dvB,      //   (two buffers: a fused launch reads one and writes the other)        C3
    X_rupB,     // the second ru_p buffer (a fused launch writes the damped ru_p there)  E3
    X_eown,     // per cell: bit i set when this cell's slot i writes its edge's ru_p    C2I
    X_eowner,   // per edge: the lowest cell * 16 + slot listing it (prepare scratch)    E2I
    X_orph,     // the edges no cell lists (written by the fused launch's extra blocks)  E2I
    X_tme,      // theta_m(cellsOnEdge(1)) + theta_m(cellsOnEdge(0)) per edge and level, formed
                // by dyn_tend's edge kernel (option "tmedge"): theta_m does not change between
                // a stage's dyn_tend and its acoustic substeps, which read it there   E3
    X_smlS,     // set_smlstep's slope flux sum of u_tend per cell and level, formed once per step
                // (atm_srk3 fast path, reference semantics: u_tend, zb_cell, zb3_cell are not
                // written by any task of the step) for the stages' fused set_smlstep      C3
    X_Dd,       // rw_save - rw per cell and level, formed with X_smlS once per step (neither is
                // written within a step in the reference semantics): the acoustic step's only use
                // of the two columns                                                      C3
    // monotonic scalar transport (k_transport.hip), one column per (entity, scalar)
    X_Ah,       // antidiffusive edge flux                                      E3 x 8
    X_Rp,       // R+ (fraction of the incoming antidiffusive flux allowed)     C3V x 8
    X_Rm,       // R- (outgoing)                                                C3V x 8
    X_su,       // the upwind update                                            C3V x 8
    X_COUNT
};

struct FieldInfo {
    const char* name;
    int kind, width, dist;
    double lo, hi;
};
extern const FieldInfo kFields[X_COUNT];

struct Halo;  // mpas_halo.h
struct TrTiles;  // below: the cell tiles of the tiled transport
struct TrEdgeGroups;  // below: the edge groups of the transport's edge kernel

struct DevState {
    int nCells, nEdges, nVertices, L, LP;  // local entity counts (= the zero-slot ids)
    int nCO, nEO, nVO;  // owned entities, the first of the local ones: every kernel's
                        // grid (= the counts above unless the mesh is decomposed)
    int lo[3];          // first cell / edge / vertex of a launch: kernels compute entities
                        // [lo, nXO); 0 except for the boundary launch of a halo overlap
    int n_orph;    // edges in X_orph (k_prepare)
    int interior;  // 1 on the interior launch of a halo overlap (Halo::launch: ghosts not
                   // yet fresh), 0 on a whole-range or boundary launch
    int epw;  // entities per column slot of the few-gather kernels (div_damp, solve): 1, 2 or 4
    int vcmix;  // 1: the vertex and cell blocks of mixed grids interleaved in proportion (vc_block)
    int cve;  // option "cve": vertices per vertex wave of dyn_tend C at LP = 64 (1, 4, 8; 0: 4)
    int bsplit;  // option "bsplit": dyn_tend's per-edge theta / w fluxes in an edge kernel of their own
                 // (fast path): 1 always, 2 under the MPAS dynamics only, 0 never
    int trsu;     // option "trsu": the transport's update forms su again instead of reading X_su
    int trsave;   // (atm_srk3, option "trsave"; set per launch) the transport reads the step's old scalars from
                  // scalars itself and its bounds kernel stores scalars_old: scalars_save folded in
    int trepw;    // option "trepw": transport edge slots per wavefront (1, 2)
    int troe;     // option "trorder_e": the transport edge kernel's slot order (0: trorder's)
    int tro;      // transport slot order (k_transport.hip tr_slot): 0 entity-major, 1 pair-major
    int nERing;   // decomposed mesh: local edges [0, nERing) are owned or ring-1 ghosts (edges of
                  // owned cells, numbered first among the ghost edges); 0 = not set
    int nVRing;   // local vertices [0, nVRing) are owned or ring-1 ghosts (vertices of owned edges)
    int ring1;    // option "ring1": the launchers that can also compute the ring-1 ghosts do
                  // (div_damping: ru_p, reference semantics; solve_diagnostics: vorticity and
                  // pv_vertex), so their gathers need no exchange (speed only, same bits)
    int physics;  // option "physics": 0 the reference's semantics; 1 the MPAS vertical solver
                  // (Q16-Q21, Q24, Q5, Q7); 2 also the MPAS dynamics (dyn_tend, solve_diagnostics,
                  // set_smlstep, setup, moist, finish in MPAS-A's forms: mpas_oracle.c ora_mpas_*)
    int xcd;  // block order: 0 dispatcher, 1 one contiguous eighth per XCD, G > 1 runs of G
              // blocks per XCD in windows of 8G (default 64)
    int eoe_same;  // 1 when edgesOnEdge_ECP equals edgesOnEdge on the owned edges (k_prepare; as
                   // mesh_loading.rg:275 sets it): v's and q's gathers are the same columns
    int selfc;  // 1 when every cell is one of the two cellsOnEdge of each of its first
                // min(nEdgesOnCell, NF) edges (k_prepare): the cell kernels then gather
                // only the other cell of an edge and use their own column for the cell
                // itself (SELF path); 0 (e.g. the literal 1-based "ref" ids) gathers both
    void* f[X_COUNT];
    Halo* halo;  // host-side halo exchanger of a decomposed mesh, nullptr otherwise
    const TrTiles* trt;  // host-side: the tiles of the tiled transport, nullptr = the three-kernel path
    const TrEdgeGroups* tre;  // host-side: the edge groups of k_tr_edge_lds, nullptr = k_tr_edge
    const TrTiles* ett;  // host-side: the cell tiles of dyn_tend's tiled E (k_dyn_Et), nullptr = k_dyn_E
    int etm, etnt;       // options "etmode" (the tiled E's flux form, k_dyn.hip dyn_E_cell ETM) and
                         // "etthreads" (its block size, 256 or 512)
    const int* gid[3];  // device global ids of the local cells/edges/vertices (decomposed
                        // meshes: the synthetic fill hashes them), nullptr = identity
};

// physical constants (constants.rg:27-66), identical to the oracle's
constexpr double kRgas = 287.0;
constexpr double kCp = 7.0 * 287.0 / 2.0;
constexpr double kGravity = 9.80616;
constexpr double kOmega = 7.29212E-5;
constexpr double kEpssm = 0.1;
constexpr double kPrandtl = 1.0;
constexpr int kRelaxZone = 5;
constexpr double kSmdiv = 0.1;
constexpr double kLenDisp = 120000.0;
constexpr double kVisc4_2dsmag = 0.05;
constexpr double kSmagCoef = 0.125;
constexpr double kDel4uDivFactor = 10.0;
constexpr int kRayleighLevels = 6;
constexpr double kRayleighDays = 5.0;
constexpr double kSecondsPerDay = 86400.0;
constexpr double kSphereRadius = 6371229.0;

// dyn_tend configuration (the Regent task's scalar arguments, dynamics_tasks.rg:818-823)
struct DynTendArgs {
    int rk_step;
    double dt;
    int horiz_mixing;  // 0 = 2d_smagorinsky, 1 = 2d_fixed, 2 = none
    double cam_coef;
    int mix_full;
    int rayleigh_damp_u;
    int exact_q;       // 1: Q10 literal (each q term added nVertLevels times), 0: nVertLevels*term
    int tme = 0;       // 1: the edge kernel also stores X_tme (atm_srk3, option "tmedge")
    int hfuse = 0;     // 1: rk_step 0's D and E in one grid (atm_srk3, option "hfuse"; undecomposed)
    int cp = 0;        // 1: the edge kernel also makes setup's ru_save = ru, u_2 = u (atm_srk3 stage 0,
                       // option "fusecopy"; undecomposed)
    int skipA = 0;     // 1: kernel A already ran (launch_hf_solve_e_dyn_A; atm_srk3 hfuse, undecomposed)
    // option "defer4" (atm_srk3, reference semantics): rk_step 0's del4 of tend_u_euler (kernel D)
    // is applied by the next stage's rk_step > 0 edge kernel, which reads tend_u_euler anyway
    int defer_out = 0;  // 1 (rk_step 0): no D; tend_u_euler left without its del4 part, tend_u not stored
    int defer_in = 0;   // 1 (rk_step > 0): apply the deferred del4 to tend_u_euler first, store it
    // option "ntu" (with defer_out): that call's tend_u is dead altogether (the next stage's edge
    // kernel rewrites it, no task in between reads it): the edge kernel forms none of it
    int ntu = 0;
    // option "mru" (atm_srk3, the MPAS dynamics, fast path): the stage's dts -- the kernel forming the final
    // tend_u stores the first acoustic substep's ru_p and ruAvg (k_acoustic_ru FIRST then skipped)
    double rud = 0.0;
    // option "msml" (atm_srk3, the MPAS dynamics): E applies the stage's set_smlstep to the tend_w it forms
    int smlE = 0;
    // option "ntu" (atm_srk3, reference semantics, a stage before the step's last): the call's theta
    // tendencies are dead as well (the last stage rewrites them; the acoustic step reads theta_m as
    // its tend_rt, Q8): E forms none of them, B no per-edge flux for them
    int nth = 0;
    // option "vdyn" (atm_srk3 stage 2, reference semantics): the edge kernel also stores
    // solve_diagnostics' v (:429-437, Q23) from the edgesOnEdge u it gathers (S.eoe_same)
    int store_v = 0;
};

enum EntityKind { KC = 0, KE = 1, KV = 2 };  // DevState::lo index

// blocks of a column-per-wavefront launch over entities [lo, end) of one kind
template <int LP>
inline int col_blocks(const DevState& S, int kind) {
    const int end = kind == KC ? S.nCO : kind == KE ? S.nEO : S.nVO;
    const int n = end - S.lo[kind];
    return n > 0 ? (n + 256 / LP - 1) / (256 / LP) : 0;
}

template <int LP, int EPW>
inline int col_blocks_n(const DevState& S, int kind) {
    const int end = kind == KC ? S.nCO : kind == KE ? S.nEO : S.nVO;
    const int n = end - S.lo[kind], per = (256 / LP) * EPW;
    return n > 0 ? (n + per - 1) / per : 0;
}

// ---- launchers (each returns the hipGetLastError of its launches) ----
hipError_t launch_rk_integration_setup(const DevState& S, hipStream_t st);
hipError_t launch_moist_coefficients(const DevState& S, hipStream_t st);
hipError_t launch_vert_imp_coefs(const DevState& S, hipStream_t st, double dts);
// setup + moist + vert_imp(dts) in one launch (option "fusesetup", reference semantics)
// (nbc, atm_srk3 option ntu: vert_imp's b_tri / c_tri not stored -- stage 1's vert_imp rewrites them)
hipError_t launch_setup_moist_vert_imp(const DevState& S, hipStream_t st, double dts, bool edges = true, int nbc = 0);
// option hfuse (atm_srk3, reference semantics, undecomposed): a stage's last acoustic launch
// (mode 2) beside its solve_diagnostics vertex / cell kernel; the stage's solve_diagnostics
// edge kernel beside the next stage's dyn_tend A (and stage 1's vert_imp after stage 0)
hipError_t launch_hf_acoustic_solve_vc(const DevState& S, hipStream_t st, double dts, int small_step, int exact,
                                       double coef_prev, int wold = 1, int ddx = 0);
hipError_t launch_hf_solve_e_dyn_A(const DevState& S, hipStream_t st, const DynTendArgs& next, int vi, double dts_vi);
// ... and stage 0's setup + moist + vert_imp launch (fusesetup) beside stage 0's dyn_tend A
// flux: also set_smlstep's flux sum of the step (X_smlS; option smlsum)
hipError_t launch_hf_setup_dyn_A(const DevState& S, hipStream_t st, const DynTendArgs& stage0, double dts, int edges,
                                 int flux = 0);
hipError_t launch_dyn_tend(const DevState& S, hipStream_t st, const DynTendArgs& a);
// exact = 0 (reference semantics): the slope-flux terms summed, then subtracted (k_sml_flux's order)
hipError_t launch_set_smlstep(const DevState& S, hipStream_t st, int exact);
// mode (reference semantics, no halo; atm_srk3 with option "fusedamp"): 0 plain, 1 also
// writes div of this substep (X_dvA), 2 also applies the previous substep's damping
// (coefficient coef_prev, its div in X_dvB) to the ru_p it reads and writes the damped
// ru_p to X_rupB; the caller swaps the buffer pairs after the launch
// tme: theta_m at the cells of each edge from X_tme (valid: dyn_tend of this stage wrote it)
// sml: the stage's set_smlstep first (a stage's first substep, mode 1 / 2; option fusesml):
// 1 from its slope fluxes, 2 (exact = 0) from X_smlS, the step's launch_sml_flux
// wold 0 (mode 1 / 2 only): rtheta_pp_old not stored -- atm_srk3's fused damping reads the div
// this launch stores instead, so only the step's last substep leaves rtheta_pp_old
// ddx: rw_save - rw from X_Dd (atm_srk3 with option smlsum: launch_sml_flux formed it this step)
hipError_t launch_acoustic(const DevState& S, hipStream_t st, double dts, int small_step, int exact, int mode = 0,
                           double coef_prev = 0.0, int tme = 0, int sml = 0, int wold = 1, int ddx = 0,
                           int mdamp = 0,   // (mdamp: the MPAS forms, the previous substep's damping folded in)
                           int rudone = 0);  // (rudone: option mru -- this stage's dyn_tend stored ru_p / ruAvg)
// X_smlS = the sum of set_smlstep's slope-flux terms per cell and level (atm_srk3 fast path,
// once per step: u_tend / zb_cell / zb3_cell are not written within a step)
hipError_t launch_sml_flux(const DevState& S, hipStream_t st);
// old_zero: only from srk3, right after a stage's first acoustic substep (k_div_damp OLD0)
hipError_t launch_div_damping(const DevState& S, hipStream_t st, double dts, int old_zero = 0);
// the damping from the div buffer X_dvB (fusedamp: the step's last substep), ru_p in place
hipError_t launch_div_damping_div(const DevState& S, hipStream_t st, double dts, int tme = 0);
// coef_divdamp of atm_divergence_damping_3d (:1736-1738) for dts
double divdamp_coef(double dts);
// combined launches of independent neighbours (option "hfuse", k_solve.hip)
hipError_t launch_hf_damp_solve_vc(const DevState& S, hipStream_t st, double dts, int tme);
hipError_t launch_hf_solve_e_finish(const DevState& S, hipStream_t st, int recon_v = 1, int norz = 0);
hipError_t launch_hf_solve_e_vert_imp(const DevState& S, hipStream_t st, double dts);
// parts: 1 the vertex / cell kernel, 2 the edge kernel, 3 both (the task)
// no_v: v (rk_step -1 / 2) is not reconstructed here (atm_srk3 option "vdyn": stage 2's dyn_tend
// edge kernel has stored it from the same u)
hipError_t launch_solve_diagnostics(const DevState& S, hipStream_t st, int hollingsworth, int rk_step, int parts = 3,
                                    int no_v = 0);
// (norz: atm_srk3, reference semantics, LP = 64 -- rho_zz = rho_zz_old_split is the identity there, not made)
hipError_t launch_substep_finish(const DevState& S, hipStream_t st, int substep, int split, int norz = 0);
hipError_t launch_fill_synthetic(const DevState& S, hipStream_t st, uint64_t seed);
// keep tails (below): set both tails of field f from the field; compare one tail (level 0 or
// L) with the field on the owned entities, *flag = 2 f + lev0 + 1 on a mismatch
hipError_t launch_keep_refresh(const DevState& S, hipStream_t st, int f, int kind);
hipError_t launch_keep_check(const DevState& S, hipStream_t st, int f, int kind, int lev0, int* flag);
hipError_t launch_prepare(DevState& S, hipStream_t st);
// damp (option mdamp, the MPAS forms): 1 the stage's last divergence damping (coefficient of damp_dts)
// applied by the edge kernel, 2 the same with rtheta_pp_old = 0 (the stage's last substep was its first)
hipError_t launch_recover_large_step(const DevState& S, hipStream_t st, int ns, int rk_step, double dt, int navg = 0,
                                     int damp = 0, double damp_dts = 0.0);
hipError_t launch_reconstruct_2d(const DevState& S, hipStream_t st, int on_a_sphere);
hipError_t launch_output_diagnostics(const DevState& S, hipStream_t st);
// fold (atm_srk3, option "trsave"): scalars_save not run before -- scalars still holds the old values,
// and the bounds kernel stores them to scalars_old (undecomposed, default kernels only)
hipError_t launch_advance_scalars_mono(const DevState& S, hipStream_t st, double dt, int fold = 0);
hipError_t launch_damping_coefs(const DevState& S, hipStream_t st, double zd, double xnutr);
hipError_t launch_compute_signs(const DevState& S, hipStream_t st);
// strided device view <-> LP-padded 3-D field (elem 8: fp64, 1: uint8 masks)
hipError_t launch_view_copy(void* dev, void* view, int elem, int n, int W, int L, int LP, int64_t se, int64_t sl,
                            int64_t sc, int to_dev, hipStream_t st);
hipError_t launch_adv_coef_compression(const DevState& S, hipStream_t st);
hipError_t launch_couple_coef_3rd_order(const DevState& S, hipStream_t st, double coef);
hipError_t launch_mesh_scaling(const DevState& S, hipStream_t st, int config_h_ScaleWithMesh);
hipError_t launch_init_coupled_diagnostics(const DevState& S, hipStream_t st);
size_t summarize_scratch_bytes();

// ---- bounds-checked build (MPAS_BOUNDS, below) ----
#ifndef MPAS_BOUNDS
#define MPAS_BOUNDS 0
#endif
constexpr int kBoundsMax = 4096;  // fields of all live contexts
struct BoundsTab {
    unsigned long long lo[kBoundsMax], hi[kBoundsMax];  // sorted field ranges [lo, hi)
    int n;
    unsigned int count;           // accesses outside their field since the last check
    unsigned long long addr;      // the first one: its address,
    unsigned long long field_lo;  // the start of the field it was checked against,
    unsigned long long where;     // blockIdx << 32 | threadIdx
};
// host: every translation unit with kernels registers the address of its table pointer
int bounds_register_tu(void* (*symbol)());
#if MPAS_BOUNDS
// reads `col` columns past the end of field u (tests: the check must catch it)
hipError_t launch_bounds_probe(const DevState& S, hipStream_t st, int col);
#endif
hipError_t launch_summarize(const DevState& S, hipStream_t st, void* scratch, double* out);

// ---- device helpers ----
#if defined(__HIPCC__)
// XCD-aware block order (cdna_hip_programming.md §5.5 T1): the dispatcher deals blocks
// round-robin over the 8 XCDs, so consecutive blocks -- neighbouring columns of the
// Morton-ordered mesh -- would land on 8 different L2s and every neighbour gather would
// miss.  Remap so that the blocks sharing an XCD (b % 8) own one contiguous 1/8 of the
// virtual block range (bijective for any grid size).  Speed only: any placement is correct.
//   on == 1: each XCD owns one contiguous 1/8 of the grid;
//   on == G > 1: within every window of 8G consecutive blocks each XCD owns G contiguous
//   blocks (all XCDs stay inside one Infinity-Cache window, each L2 sees a compact
//   sub-range); blocks past the last whole window keep the dispatcher order.
__device__ __forceinline__ int xcd_block_n(int on, int b, int nb) {
    if (on <= 0) return b;
    if (on == 1) {
        const int q = nb >> 3, r = nb & 7, x = b & 7, pos = b >> 3;
        return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + pos;
    }
    const int W = on << 3;
    if (b >= (nb / W) * W) return b;
    const int w = b / W, r = b - w * W;
    return w * W + (r & 7) * on + (r >> 3);
}
// the remap over the whole grid
__device__ __forceinline__ int xcd_block(int on) { return xcd_block_n(on, (int)blockIdx.x, (int)gridDim.x); }

// The block index and block count a kernel body sees: blockIdx.x / gridDim.x of its own
// launch, or its sub-range of a combined launch (k_hfuse.h: two independent kernels of the
// step in one grid, blocks [0, n1) running the first body and [n1, gridDim.x) the second)
struct Blk {
    int b, n;
};
__device__ __forceinline__ Blk this_blk() { return {(int)blockIdx.x, (int)gridDim.x}; }

// Mixed vertex + cell grids (dyn_tend C, solve_diagnostics): nVB vertex blocks and
// nb - nVB cell blocks.  With S.vcmix they are interleaved in proportion -- block b is a
// vertex block iff floor((b+1) nVB / nb) > floor(b nVB / nb) -- so that the vertex and
// the cell blocks of one region of the Morton-ordered mesh run at the same time and the
// edge columns both gather are fetched into L2 once; otherwise all vertex blocks come
// first.  Returns true for a vertex block; idx = its vertex (or cell) block index.
__device__ __forceinline__ bool vc_block(const DevState& S, int blk, int nVB, int& idx, int nblocks = -1) {
    if (!S.vcmix) {
        idx = blk < nVB ? blk : blk - nVB;
        return blk < nVB;
    }
    const long long nb = nblocks >= 0 ? (long long)nblocks : (long long)gridDim.x;
    const int a = (int)((long long)blk * nVB / nb), a1 = (int)((long long)(blk + 1) * nVB / nb);
    idx = a1 > a ? a : blk - a;
    return a1 > a;
}

// entity of this lane's column in virtual block blk; at LP == 64 one column per
// wavefront, made explicit so connectivity and mesh constants of the column come
// through the scalar unit (s_load) and gathers are SGPR base + lane offset
template <int LP>
__device__ __forceinline__ int col_of(int blk) {
    int e = blk * (256 / LP) + (int)(threadIdx.x / LP);
    if constexpr (LP == 64) e = __builtin_amdgcn_readfirstlane(e);
    return e;
}

template <int LP>
struct ColMap {
    static constexpr int COLS = 256 / LP;
    int blk, ent, k;
    __device__ __forceinline__ ColMap(const DevState& S, int kind, Blk bk = this_blk()) {
        blk = xcd_block_n(S.xcd, bk.b, bk.n);
        ent = col_of<LP>(blk) + S.lo[kind];
        k = (int)(threadIdx.x % LP);
    }
};

// EPW consecutive entities per column slot: the kernels with only a few gathers per
// entity issue the loads of EPW entities together (more memory requests in flight per
// wavefront; a one-entity wave of such a kernel is latency-bound)
template <int LP, int EPW>
struct ColMapN {
    static constexpr int COLS = 256 / LP;
    int blk, base, k;
    __device__ __forceinline__ ColMapN(const DevState& S, int kind, Blk bk = this_blk()) {
        blk = xcd_block_n(S.xcd, bk.b, bk.n);
        base = col_of<LP>(blk) * EPW + S.lo[kind];
        k = (int)(threadIdx.x % LP);
    }
};

// Fast-path unroll widths: x1 meshes have 5-6 edges per cell and <= 10 edgesOnEdge;
// loads for these many entries are issued unconditionally (padding ids are valid
// entity ids, clamped on upload) ahead of the in-order accumulation; any entries
// beyond them are handled by a generic tail loop.
constexpr int NF = 6;   // edgesOnCell

constexpr int QF = 10;  // edgesOnEdge
constexpr int AF = 9;   // advCellsForEdge (the reference's list holds at most 9, :175)
static_assert(NF % 2 == 0 && QF % 2 == 0, "the gathers go in pairs (gather2)");

// Tiled transport (k_transport.hip, option "trtile"): the owned cells grouped into compact
// tiles of at most TRT_CELLS cells (breadth-first growth on the host, mpas_ctx.cpp
// trt_build); a tile's CLOSURE is every cell its kernels read scalars_old at -- the cells
// themselves, both cells of each of their edges and the advCellsForEdge of those edges --
// loaded into LDS once per (tile, scalar).  Per tile cell one row of TRT_ROW LDS slots:
// the cell, then per edge slot i < NF: cellsOnEdge(0), cellsOnEdge(1), advCells(0..AF-1).
constexpr int TRT_CELLS = 16;
constexpr int TRT_ROW = 1 + NF * (2 + AF);
struct TrTiles {
    int ntiles = 0, nt_int = 0;  // tiles; the first nt_int hold interior cells only
    int nco = 0, nint = 0;       // the owned / interior cell counts the tiles were built for
    int maxclo = 0;              // largest closure (LDS columns per block)
    int nclo = 0;                // closure columns of all tiles (the staging loads)
    int* tptr = nullptr;         // ntiles + 1: first cell of each tile in tcell
    int* tcell = nullptr;        // the tiles' cells
    int* cptr = nullptr;         // ntiles + 1: first closure cell of each tile in ccell
    int* ccell = nullptr;        // closure cells, in LDS column order
    int* slot = nullptr;          // TRT_ROW LDS columns per tile cell (tcell order)
    // dyn_tend's tiled E (k_dyn_Et): the tile's edges, and per tile cell one ETT_REC-byte record
    int* teptr = nullptr;         // ntiles + 1: first edge of each tile in tedge
    int* tedge = nullptr;         // the edges of the tile's cells, in first-use order
    unsigned* erow = nullptr;     // per tile cell (tcell order), per edge slot i < NF, ETT_EB bytes: the
                                  // edge's index among the tile's edges, then its AF advCells' closure
                                  // columns (the zero column, index = closure size, past nAdvCellsForEdge
                                  // and for slots past nEdgesOnCell)
    unsigned* terec = nullptr;    // per tile edge (tedge order) ETT_ER bytes: its AF advCells' closure columns
    int maxte = 0;                // most edges of a tile
};
constexpr int ETT_EB = 12;            // record bytes per edge slot (1 + AF, padded)
constexpr int ETT_REC = NF * ETT_EB;  // 72: 18 dwords per tile cell
constexpr int ETT_ER = 12;            // record bytes per tile edge (AF, padded)

// The transport's edge kernel with its scalars_old columns staged in LDS (k_tr_edge_lds,
// option "tredge"): the owned edges in groups of TRE_GE consecutive ids (Morton-adjacent);
// a group's UNION is the distinct cells its edges read scalars_old at (advCellsForEdge
// and cellsOnEdge), at most TRE_U; a group with a larger union or an edge with more than AF
// advCells is irregular (ucnt = -1) and gathers directly.  Built on the host (tre_build).
constexpr int TRE_GE = 16;  // edges per group
constexpr int TRE_U = 52;   // LDS columns per group (52 KB at LP = 64 with a scalar pair
                            // each: three blocks per CU)
constexpr int TRE_ROW = 12;  // slot bytes per edge: AF advCells, cellsOnEdge(0), (1), pad
struct TrEdgeGroups {
    int ngroups = 0, neo = 0;  // groups; the owned edge count they were built for
    int nirr = 0;              // irregular groups (reported by option "tredge_irregular")
    int* ucell = nullptr;      // ngroups * TRE_U: the union's cells (padding: its first cell)
    int* ucnt = nullptr;       // ngroups: union size, -1 = irregular
    unsigned* eslot = nullptr; // neo * TRE_ROW / 4: each edge's LDS columns, one byte each
};

// value of x held by level k-1 of the same column (0.0 at k == 0: level -1 reads 0)
template <int LP>
__device__ __forceinline__ double lvl_dn(double x, int k) {
    double y = __shfl_up(x, 1, LP);
    return k == 0 ? 0.0 : y;
}
template <int LP>
__device__ __forceinline__ double lvl_dn2(double x, int k) {
    double y = __shfl_up(x, 2, LP);
    return k < 2 ? 0.0 : y;
}
// value held by level k+1 (0.0 above the column's last lane)
template <int LP>
__device__ __forceinline__ double lvl_up(double x, int k) {
    double y = __shfl_down(x, 1, LP);
    return k == LP - 1 ? 0.0 : y;
}

// A wave-uniform pointer held in SGPRs.  Loads through it at a lane offset compile to
// the saddr + 32-bit voffset form: no per-load 64-bit VALU address add (the compiler
// otherwise folds the lane offset into a VGPR base and adds the row offset per gather).
#define MPAS_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ MPAS_GLOBAL T* sgpr_ptr(T* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (MPAS_GLOBAL T*)(((uint64_t)hi << 32) | lo);
}

// A wave-uniform double made visibly uniform (readfirstlane of both halves; only for values
// the whole wavefront shares: one column per wave, LP = 64).  The lane
// reads are convergent, so the compiler cannot sink the load feeding them into a
// lane-divergent block, where it would be waited for with a full s_waitcnt vmcnt(0)
__device__ __forceinline__ double uniform_d(double x) {
    const uint64_t v = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

#if MPAS_BOUNDS
// Bounds-checked build (-DMPAS_BOUNDS=1, `make -C csrc bounds` -> libmpasdyn_bounds.so,
// selected with env MPAS_LIB).  Every column access (colk, gather2, gather2s,
// col_rd) is checked against the field its base pointer starts, every mesh-row load
// (row_ld) against the field it falls in, through a sorted table of the [begin, end) of
// every field of every live context (mpas_ctx.cpp bounds_publish).  An access outside
// reads / writes a sink instead and is recorded; the C-ABI call that ran the kernel then
// fails with MPAS_EBOUNDS, naming the field.  Each translation unit has its own copy of
// the table pointer, registered with the host at load time.
static __device__ BoundsTab* g_bounds;
static __device__ double g_bounds_sink[64];  // (covers the widest row_ld)
static void* bounds_symbol_() {
    void* p = nullptr;
    return hipGetSymbolAddress(&p, HIP_SYMBOL(g_bounds)) == hipSuccess ? p : nullptr;
}
static const int g_bounds_registered_ = bounds_register_tu(&bounds_symbol_);
__device__ __noinline__ static inline void* bounds_chk(const void* base, const void* p, unsigned bytes) {
    BoundsTab* t = g_bounds;
    if (!t) return (void*)p;
    const unsigned long long b = (unsigned long long)base, a = (unsigned long long)p;
    int lo = 0, hi = t->n - 1, hit = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (t->lo[mid] <= b) hit = mid, lo = mid + 1;
        else hi = mid - 1;
    }
    if (hit < 0 || b >= t->hi[hit]) return (void*)p;  // not inside a field: not checked
    if (a >= t->lo[hit] && a + bytes <= t->hi[hit]) return (void*)p;
    if (atomicAdd(&t->count, 1u) == 0u) {
        t->addr = a;
        t->field_lo = t->lo[hit];
        t->where = ((unsigned long long)blockIdx.x << 32) | threadIdx.x;
    }
    return g_bounds_sink;
}
#define MPAS_CHK(base, p, bytes) bounds_chk((base), (p), (bytes))
#else
#define MPAS_CHK(base, p, bytes) (p)
#endif

// Level k of column ent of field f, addressed as the field's base (wave-uniform, SGPRs)
// plus a 32-bit byte offset in a VGPR: loads compile to the saddr + voffset form, every
// field gathered at the same neighbour shares one offset register, and only one SGPR
// pair per field is live (per-row SGPR pointers run the scalar file out of registers,
// and the compiler then serialises the connectivity loads).  Every field is < 4 GiB.
template <int LP>
__device__ __forceinline__ uint32_t col_off(int ent, int k) {
    return ((uint32_t)ent * (uint32_t)LP + (uint32_t)lpos(LP, k)) * (uint32_t)sizeof(double);
}
template <class T>
__device__ __forceinline__ T& at_off(T* f, uint32_t off) {
#if MPAS_BOUNDS
    return *(T*)bounds_chk(f, (const char*)f + off, sizeof(T));
#else
    return *(T*)((MPAS_GLOBAL char*)(f) + off);
#endif
}
// level k of column ent of field pointer f (needs LP and k in scope)
#define colk(f, ent) at_off((f), col_off<LP>((ent), k))


// Two gathered columns, a = level k of column ia of field fa, b = level k of column ib
// of field fb (any fields, any entities).  At LP = 64 one 16-B load per lane (lanes 0-31
// read level pair j = k & 31 of column a, lanes 32-63 that of column b; see lpos) and one
// permlane32_swap per dword (lanes 32-63 of x <-> lanes 0-31 of y) give both columns back
// in lane = level order: half the load instructions of two 8-B gathers, which is what
// the gather kernels are bound by.  Two plain loads below LP 64.
__device__ __forceinline__ void swap_halves(double& x, double& y) {
    int2 xi = __builtin_bit_cast(int2, x), yi = __builtin_bit_cast(int2, y);
    const auto r0 = __builtin_amdgcn_permlane32_swap(xi.x, yi.x, false, false);
    const auto r1 = __builtin_amdgcn_permlane32_swap(xi.y, yi.y, false, false);
    xi.x = (int)r0[0];
    yi.x = (int)r0[1];
    xi.y = (int)r1[0];
    yi.y = (int)r1[1];
    x = __builtin_bit_cast(double, xi);
    y = __builtin_bit_cast(double, yi);
}
template <int LP>
__device__ __forceinline__ void gather2(const double* fa, int ia, const double* fb, int ib, int k, double& a,
                                        double& b) {
    if constexpr (LP == 64) {
        const bool hi = k >= 32;
        const char* base = hi ? (const char*)fb + (size_t)(uint32_t)ib * 512 : (const char*)fa + (size_t)(uint32_t)ia * 512;
        const double2 t = *(const double2*)MPAS_CHK(hi ? fb : fa, base + (k & 31) * 16, 16);
        double x = t.x, y = t.y;
        swap_halves(x, y);
        a = x;
        b = y;
    } else {
        a = colk(fa, ia);
        b = colk(fb, ib);
    }
}

// gather2 / gather2s in two halves, for a kernel that issues every load of a section before
// the first swap (the loads, __builtin_amdgcn_sched_barrier, then g2_fin): the compiler
// otherwise interleaves the first swaps with the loads and waits on each (dyn_tend B)
template <int LP>
__device__ __forceinline__ double2 gather2_ld(const double* fa, int ia, const double* fb, int ib, int k) {
    if constexpr (LP == 64) {
        const bool hi = k >= 32;
        const char* base = hi ? (const char*)fb + (size_t)(uint32_t)ib * 512 : (const char*)fa + (size_t)(uint32_t)ia * 512;
        return *(const double2*)MPAS_CHK(hi ? fb : fa, base + (k & 31) * 16, 16);
    } else {
        return make_double2(colk(fa, ia), colk(fb, ib));
    }
}
template <int LP>
__device__ __forceinline__ double2 gather2s_ld(const double* f, int ia, int ib, int k) {
    if constexpr (LP == 64) {
        const uint32_t off = (uint32_t)(k >= 32 ? ib : ia) * 512u + (uint32_t)(k & 31) * 16u;
        return at_off((const double2*)f, off);
    } else {
        return make_double2(colk(f, ia), colk(f, ib));
    }
}
template <int LP>
__device__ __forceinline__ void g2_fin(double2 t, double& a, double& b) {
    double x = t.x, y = t.y;
    if constexpr (LP == 64) swap_halves(x, y);
    a = x;
    b = y;
}

// f at the two cellsOnEdge (x1, x2) of edge slot i of a cell.  SELF (S.selfc): the cell
// is one of them, so only the other cell `oth` is gathered and `own`, f at the cell
// itself, stands in for the other (s1: the cell is cellsOnEdge(0)).  Same values either way.
template <int LP, bool SELF>
__device__ __forceinline__ void cell_pair(const double* f, int c1, int c2, int oth, int s1, double own, int k,
                                          double& x1, double& x2) {
    if constexpr (SELF) {
        const double xo = colk(f, oth);
        x1 = s1 ? own : xo;
        x2 = s1 ? xo : own;
    } else {
        x1 = colk(f, c1);
        x2 = colk(f, c2);
    }
}

// gather2 of one field at two entities: the field base stays in SGPRs and only the
// 32-bit offset is selected per lane (the saddr + voffset form of col_off)
// The inverse of gather2: lane k holds level k of column ia of fa (value a) and of column
// ib of fb (value b); at LP = 64 one 16-B store per lane writes both (lanes 0-31 the level
// pair of ia, lanes 32-63 that of ib, after the same permlane32 swap), so every lane of the
// wavefront must take part.  oka / okb: whether level k of each column is written (a level
// the reference never writes -- level L, or level 0 of some fields -- keeps its value);
// the caller applies PADW to the padding levels.
template <int LP>
__device__ __forceinline__ void put2(double* fa, int ia, double* fb, int ib, int k, double a, double b, bool oka,
                                     bool okb) {
    if constexpr (LP == 64) {
        double x = a, y = b;
        swap_halves(x, y);
        const auto f = __builtin_amdgcn_permlane32_swap((unsigned)oka, (unsigned)okb, false, false);
        const bool sx = f[0] != 0, sy = f[1] != 0;  // this lane's two elements (levels k & 31, +32)
        const bool hi = k >= 32;
        char* base = hi ? (char*)fb + (size_t)(uint32_t)ib * 512 : (char*)fa + (size_t)(uint32_t)ia * 512;
        double* q = (double*)MPAS_CHK(hi ? fb : fa, base + (k & 31) * 16, 16);
        if (sx && sy) *(double2*)q = make_double2(x, y);
        else if (sx) q[0] = x;
        else if (sy) q[1] = y;
    } else {
        if (oka) colk(fa, ia) = a;
        if (okb) colk(fb, ib) = b;
    }
}

// put2 of two whole columns (every level stored: the keep-tail stores, KEEPW): one 16-B store
// per lane with no mask exchange -- put2's masks, even when all true, cost a permlane of the
// flags and three divergent store branches (the compiler cannot fold them through the swap)
template <int LP>
__device__ __forceinline__ void put2f(double* fa, int ia, double* fb, int ib, int k, double a, double b) {
    if constexpr (LP == 64) {
        double x = a, y = b;
        swap_halves(x, y);
        const bool hi = k >= 32;
        char* base = hi ? (char*)fb + (size_t)(uint32_t)ib * 512 : (char*)fa + (size_t)(uint32_t)ia * 512;
        *(double2*)MPAS_CHK(hi ? fb : fa, base + (k & 31) * 16, 16) = make_double2(x, y);
    } else {
        colk(fa, ia) = a;
        colk(fb, ib) = b;
    }
}

template <int LP>
__device__ __forceinline__ void gather2s(const double* f, int ia, int ib, int k, double& a, double& b) {
    if constexpr (LP == 64) {
        const uint32_t off = (uint32_t)(k >= 32 ? ib : ia) * 512u + (uint32_t)(k & 31) * 16u;
        const double2 t = at_off((const double2*)f, off);
        double x = t.x, y = t.y;
        swap_halves(x, y);
        a = x;
        b = y;
    } else {
        a = colk(f, ia);
        b = colk(f, ib);
    }
}

// cell_pair for edge slots i and i+1 of one field: two gather2 (SELF: one)
template <int LP, bool SELF>
__device__ __forceinline__ void cell_pair2(const double* f, const int* c1, const int* c2, const int* oth, const int* s1,
                                           double own, int i, int k, double& x1, double& x2, double& y1, double& y2) {
    if constexpr (SELF) {
        double xo, yo;
        gather2s<LP>(f, oth[i], oth[i + 1], k, xo, yo);
        x1 = s1[i] ? own : xo;
        x2 = s1[i] ? xo : own;
        y1 = s1[i + 1] ? own : yo;
        y2 = s1[i + 1] ? yo : own;
    } else {
        gather2s<LP>(f, c1[i], c2[i], k, x1, x2);
        gather2s<LP>(f, c1[i + 1], c2[i + 1], k, y1, y2);
    }
}
// cell_pair of two fields at edge slot i: (SELF: one gather2 of both fields)
template <int LP, bool SELF>
__device__ __forceinline__ void cell_pair_ff(const double* f, const double* g, const int* c1, const int* c2,
                                             const int* oth, const int* s1, double fown, double gown, int i, int k,
                                             double& f1, double& f2, double& g1, double& g2) {
    if constexpr (SELF) {
        double fo, go;
        gather2<LP>(f, oth[i], g, oth[i], k, fo, go);
        f1 = s1[i] ? fown : fo;
        f2 = s1[i] ? fo : fown;
        g1 = s1[i] ? gown : go;
        g2 = s1[i] ? go : gown;
    } else {
        gather2s<LP>(f, c1[i], c2[i], k, f1, f2);
        gather2s<LP>(g, c1[i], c2[i], k, g1, g2);
    }
}

__device__ __forceinline__ const double* fd(const DevState& S, int id) { return (const double*)S.f[id]; }
__device__ __forceinline__ double* fw(const DevState& S, int id) { return (double*)S.f[id]; }
__device__ __forceinline__ const int* fi(const DevState& S, int id) { return (const int*)S.f[id]; }

// Masked column values.  Every lane of a column row (LP doubles) is allocated, so the
// load is issued unconditionally and masked afterwards with a select: a load under a
// lane condition compiles to a branch around it, which serialises the gathers
// (s_waitcnt vmcnt(0) at every join) and costs the memory-level parallelism.
__device__ __forceinline__ double ldz(bool keep, double v) { return keep ? v : 0.0; }

// acc + t where c holds, acc elsewhere.  A select, not a branch: the operands, loaded
// ahead, are then not sunk by the compiler into a conditional block (one memory round
// trip, and one full s_waitcnt vmcnt(0), per list entry).  Bit-identical to `if (c) acc += t`.
__device__ __forceinline__ double add_if(bool c, double acc, double t) { return c ? acc + t : acc; }
__device__ __forceinline__ double sub_if(bool c, double acc, double t) { return c ? acc - t : acc; }

// A load the compiler may take through the scalar unit: the constant address space
// declares the data read-only for the kernel's lifetime (mesh rows and the tile tables,
// which only the one-time preparation kernels write).  With a wave-uniform address it is an s_load; through a
// generic pointer the kernels' stores between cells would make every row entry a vector
// load of its own (the compiler cannot prove they do not alias).
#define MPAS_CONST __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ T ldc(const T* p) {
    return *(const MPAS_CONST T*)(uintptr_t)p;
}

// the first N entries of a padded mesh-data row, loaded unconditionally (every row is
// allocated at its full width, so the entries past the list's length are in bounds).
// Through ldc: every row_ld source is mesh data or a precomputed mesh table, so a
// wave-uniform row is scalar loads even in a kernel that also stores (a mixed vertex /
// cell grid, a damping path)
template <int N, class T>
__device__ __forceinline__ void row_ld(const T* p, T (&r)[N]) {
#if MPAS_BOUNDS
    p = (const T*)(MPAS_CHK(p, p, N * sizeof(T)) == (const void*)p ? p : (const T*)g_bounds_sink);
#endif
#pragma unroll
    for (int i = 0; i < N; i++) r[i] = ldc(p + i);
}

// a cell's first NF edges and their cells from its record (X_cR / X_cRs): one scalar
// round trip; a_/b_ = cell1/cell2 of each edge, or (SELF) the other cell / "cell is cell1"
constexpr int CREC = 3 * NF + 2;
template <bool SELF>
__device__ __forceinline__ int cell_rec(const DevState& S, int c, int (&e_)[NF], int (&a_)[NF], int (&b_)[NF]) {
    int r[CREC];
    row_ld(fi(S, SELF ? X_cRs : X_cR) + (size_t)c * CREC, r);
#pragma unroll
    for (int i = 0; i < NF; i++) {
        e_[i] = r[i];
        a_[i] = r[NF + i];
        b_[i] = r[2 * NF + i];
    }
    return r[3 * NF];
}

// A store masked to the levels below L leaves level L and the padding levels L+1..LP-1
// unwritten; with the level-pair layout (lpos) those sit at odd positions spread over the
// last two 64-B sectors of the column, and every partially written sector costs HBM time.
// Kernels therefore also write the padding levels, with 0.0 (their content everywhere):
// `if (k < L || k > L) f = PADW(v)`.
#define PADW(v) (k > L ? 0.0 : (v))

// Keep tails (round 5).  Level L of the fields the reference never writes there (and level
// 0 of vert_imp's tridiagonal coefficients) used to stay unwritten: one 8-B hole per column,
// so the column's last 128-B line was written partially -- measured +9 to +24 % on a write
// stream (tools/ubench/pitch.py, profiles/r05/pitch_ubench_holes.json) and -4 % over the
// step when filled (timing-only build, profiles/r05/nohole_ab).  Every width-1 C3 / E3 / V3
// field's allocation now ends with two tails of n + 1 doubles: the value of level L
// (keepL) and of level 0 (keep0) of each column.  A kernel that leaves one of those slots
// writes the tail's value there instead (the value the slot holds: the same bits), so every
// line of the column is written whole.  The tails are set from the field by
// mpas_ctx.cpp keep_refresh after every write from outside the step kernels (upload, the
// synthetic fill, the init tasks, ...), and a kernel that writes level L of a keep field
// (set_smlstep's w) writes its tail too; option "keep_check" (tests) compares every tail
// with its field after each task.
template <int LP>
__device__ __forceinline__ const double* keep_tail(const DevState& S, int f, int kind, bool lev0) {
    const int n = kind == KC ? S.nCells : kind == KE ? S.nEdges : S.nVertices;
    return fd(S, f) + (size_t)(n + 1) * LP + (lev0 ? (size_t)(n + 1) : 0);
}
// the kept level-L (lev0: level-0) value of column ent of field f: a scalar load when ent is
// wave-uniform (the tails change only between launches)
template <int LP>
__device__ __forceinline__ double keepv(const DevState& S, int f, int kind, int ent, bool lev0 = false) {
    return ldc(keep_tail<LP>(S, f, kind, lev0) + ent);
}
// a kernel that changes the level-L value of a keep field updates its tail with it
template <int LP>
__device__ __forceinline__ void keep_put(const DevState& S, int f, int kind, int ent, double v) {
    const_cast<double*>(keep_tail<LP>(S, f, kind, false))[ent] = v;
}
template <int LP>
__device__ __forceinline__ void keep_put0(const DevState& S, int f, int kind, int ent, double v) {
    const_cast<double*>(keep_tail<LP>(S, f, kind, true))[ent] = v;
}
// the value a store of level k writes: v where the kernel computes the level, the kept
// value at level L (and, hold0, at level 0), 0.0 on the padding levels
#define KEEPW(v, kl_) (k == L ? (kl_) : PADW(v))
#define KEEPW0(v, k0_, kl_) (k == 0 ? (k0_) : KEEPW(v, kl_))

// column read with the level policy: levels outside 0..L read 0.0
template <int LP>
__device__ __forceinline__ double col_rd(const double* f, int ent, int k, int L) {
    return ldz(k <= L, at_off(f, col_off<LP>(ent, k)));
}
// col_rd of two fields of one column (gather2)
template <int LP>
__device__ __forceinline__ void col_rd2(const double* f, const double* g, int ent, int k, int L, double& a, double& b) {
    gather2<LP>(f, ent, g, ent, k, a, b);
    a = ldz(k <= L, a);
    b = ldz(k <= L, b);
}
#endif

}  // namespace mpas

#define MPAS_LP_DISPATCH(LPVAL, FN, ...)                              \
    do {                                                              \
        switch (LPVAL) {                                              \
            case 8: return FN<8>(__VA_ARGS__);                        \
            case 16: return FN<16>(__VA_ARGS__);                      \
            case 32: return FN<32>(__VA_ARGS__);                      \
            case 64: return FN<64>(__VA_ARGS__);                      \
            default: return hipErrorInvalidValue;                     \
        }                                                             \
    } while (0)
