// k_mesh.hip -- the mesh tasks of atm_core_init (atm_core.rg:22-39) on the device:
// atm_compute_signs (dynamics_tasks.rg:46-130), atm_adv_coef_compression (:133-269),
// atm_couple_coef_3rd_order (:303-325) and atm_compute_mesh_scaling (:595-646).
//
// One-time integer / list work over the mesh: one thread per entity, the reference's
// loops serial inside it (a hexagon's lists are 6-10 long; HBM-light, run once).  Ids
// are compared as the arrays hold them (uploaded with the Q1 clamp to [0, n]) and read
// through them as the hot path does (row n is the zero slot).  The bounds the reference
// leaves undefined follow the oracle (oracle/mpas_oracle.c ora_atm_adv_coef_compression):
// the cell list is capped at maxEdges - 1 in both loops, deriv_two past its 30 entries
// reads 0.0.  Every task computes the owned entities of a decomposed mesh; ghosts keep
// their uploaded values.
#include "mpas_dev.h"
#include "mpas_halo.h"

namespace mpas {

constexpr int kMaxEdges = 10, kVertexDegree = 3, kFifteen = 15;

__device__ __forceinline__ int ent_of(const DevState& S, int kind) {
    return (int)(blockIdx.x * 256 + threadIdx.x) + S.lo[kind];
}

// ---------------------------------------------------------------- atm_compute_signs
__global__ __launch_bounds__(256) void k_signs_vertices(DevState S) {
    const int v = ent_of(S, KV);
    if (v >= S.nVO) return;
    const int *eov = fi(S, F_edgesOnVertex), *voe = fi(S, F_verticesOnEdge);
    double* sgn = fw(S, F_edgesOnVertexSign);
    for (int i = 0; i < kVertexDegree; i++) {  // :61-73
        const int e = eov[(size_t)v * kVertexDegree + i];
        sgn[(size_t)v * kVertexDegree + i] = e <= S.nEdges ? (v == voe[(size_t)e * 2 + 1] ? 1.0 : -1.0) : 0.0;
    }
}

template <int LP>
__global__ __launch_bounds__(256) void k_signs_cells(DevState S) {
    const int c = ent_of(S, KC);
    if (c >= S.nCO) return;
    const int *eoc = fi(S, F_edgesOnCell), *coe = fi(S, F_cellsOnEdge), *voc = fi(S, F_verticesOnCell),
              *cov = fi(S, F_cellsOnVertex);
    double* sgn = fw(S, F_edgesOnCellSign);
    int* kite = (int*)S.f[F_kiteForCell];
    int ne = fi(S, F_nEdgesOnCell)[c];
    if (ne > kMaxEdges) ne = kMaxEdges;
    const size_t r = (size_t)c * kMaxEdges;
    for (int i = 0; i < ne; i++) {  // :75-87
        const int e = eoc[r + i];
        sgn[r + i] = e <= S.nEdges ? (c == coe[(size_t)e * 2] ? 1.0 : -1.0) : 0.0;
    }
    // :88-110: zb_cell / zb3_cell = er.zb / er.zb3 of the cell's edge (component 0 or 1 by
    // the cell's side), written by init_atm_case_jw (init_atm_cases.rg:657-660).  The port
    // keeps no er.zb: the host that builds the initial state does that copy when it
    // uploads zb_cell / zb3_cell (mpasdyn/jw.py), so the device task leaves them as uploaded
    for (int i = 0; i < ne; i++) {  // :115-128 (no match: the value stays)
        const int iVtx = voc[r + i];
        if (iVtx <= S.nVertices) {
            for (int j = 1; j < kVertexDegree; j++)
                if (c == cov[(size_t)iVtx * kVertexDegree + j]) {
                    kite[r + i] = j;
                    break;
                }
        } else {
            kite[r + i] = 1;
        }
    }
}

template <int LP>
static hipError_t signs_lp(const DevState& S, hipStream_t st) {
    const int nv = S.nVO - S.lo[KV], nc = S.nCO - S.lo[KC];
    if (nv > 0) k_signs_vertices<<<(nv + 255) / 256, 256, 0, st>>>(S);
    if (nc > 0) k_signs_cells<LP><<<(nc + 255) / 256, 256, 0, st>>>(S);
    return hipGetLastError();
}
hipError_t launch_compute_signs(const DevState& S, hipStream_t st) { MPAS_LP_DISPATCH(S.LP, signs_lp, S, st); }

// ---------------------------------------------------------------- atm_adv_coef_compression
__global__ __launch_bounds__(256) void k_adv_coef_compression(DevState S) {
    const int e = ent_of(S, KE);
    if (e >= S.nEO) return;
    const int nC = S.nCells;
    const int *coe = fi(S, F_cellsOnEdge), *coc = fi(S, F_cellsOnCell), *nEoC = fi(S, F_nEdgesOnCell);
    int* nadv = (int*)S.f[F_nAdvCellsForEdge];
    int* advc = (int*)S.f[F_advCellsForEdge] + (size_t)e * kFifteen;
    double* a = fw(S, F_adv_coefs) + (size_t)e * kFifteen;
    double* a3 = fw(S, F_adv_coefs_3rd) + (size_t)e * kFifteen;
    const double* d2 = fd(S, F_deriv_two) + (size_t)e * 30;
    nadv[e] = 0;  // :147
    const int cell1 = coe[(size_t)e * 2], cell2 = coe[(size_t)e * 2 + 1];
    if (!(cell1 <= nC || cell2 <= nC)) return;  // :153
    int cl[kMaxEdges];
    cl[0] = cell1;
    cl[1] = cell2;
    int n = 1;
    const int ne1 = nEoC[cell1], ne2 = nEoC[cell2];
    for (int i = 0; i < ne1; i++) {  // :159-165
        const int cc = coc[(size_t)cell1 * kMaxEdges + i];
        if (cc != cell2 && n < kMaxEdges - 1) cl[++n] = cc;
    }
    for (int ic = 0; ic < ne2; ic++) {  // :168-179
        const int cc = coc[(size_t)cell2 * kMaxEdges + ic];
        bool add = true;
        for (int i = 0; i < n; i++)
            if (cl[i] == cc) add = false;
        if (add && n < kMaxEdges - 1) cl[++n] = cc;
    }
    nadv[e] = n;  // :181-184
    for (int i = 0; i < n; i++) advc[i] = cl[i];
    for (int j = 0; j < kFifteen; j++) a[j] = a3[j] = 0.0;
    auto D2 = [&](int idx) { return idx < 30 ? d2[idx] : 0.0; };
    auto slot = [&](int cell) {  // the LAST j < n holding `cell` (0 if none)
        int j_in = 0;
        for (int j = 0; j < n; j++)
            if (cl[j] == cell) j_in = j;
        return j_in;
    };
    int j_in = slot(cell1);  // :193-213
    a[j_in] += d2[0];
    a3[j_in] += d2[0];
    for (int ic = 0; ic < ne1; ic++) {
        j_in = slot(coc[(size_t)cell1 * kMaxEdges + ic]);
        a[j_in] += D2(ic * kFifteen + 0);
        a3[j_in] += D2(ic * kFifteen + 0);
    }
    j_in = slot(cell2);  // :215-235
    a[j_in] += d2[1];
    a3[j_in] += d2[1];
    for (int ic = 0; ic < ne2; ic++) {
        j_in = slot(coc[(size_t)cell2 * kMaxEdges + ic]);
        a[j_in] += D2(ic * kFifteen + 1);
        a3[j_in] += D2(ic * kFifteen + 1);
    }
    const double dc = fd(S, F_dcEdge)[e], dv = fd(S, F_dvEdge)[e];
    for (int j = 0; j < n; j++) {  // :237-240, pow(dcEdge, 2) as dc * dc
        a[j] = -1.0 * (dc * dc) * a[j] / 12;
        a3[j] = -1.0 * (dc * dc) * a3[j] / 12;
    }
    a[slot(cell1)] += 0.5;  // :244-258
    a[slot(cell2)] += 0.5;
    for (int j = 0; j < n; j++) {  // :262-265
        a[j] *= dv;
        a3[j] *= dv;
    }
}

hipError_t launch_adv_coef_compression(const DevState& S, hipStream_t st) {
    const int ne = S.nEO - S.lo[KE];
    if (ne > 0) k_adv_coef_compression<<<(ne + 255) / 256, 256, 0, st>>>(S);
    return hipGetLastError();
}

// ---------------------------------------------------------------- atm_couple_coef_3rd_order
template <int LP>
__global__ __launch_bounds__(256) void k_couple_coef(DevState S, double coef) {
    const int t = (int)(blockIdx.x * 256 + threadIdx.x);
    const int ne = S.nEO - S.lo[KE], nc = S.nCO - S.lo[KC];
    if (t < ne) {  // :313-317
        double* a3 = fw(S, F_adv_coefs_3rd) + (size_t)(t + S.lo[KE]) * kFifteen;
        for (int i = 0; i < kFifteen; i++) a3[i] *= coef;
    } else if (t - ne < nc) {  // :319-323: zb3_cell at level 0
        const size_t c = (size_t)(t - ne + S.lo[KC]);
        double* zb3 = fw(S, F_zb3_cell);
        for (int j = 0; j < kMaxEdges; j++) zb3[(c * kMaxEdges + j) * LP + lpos(LP, 0)] *= coef;
    }
}
template <int LP>
static hipError_t couple_lp(const DevState& S, hipStream_t st, double coef) {
    const int n = (S.nEO - S.lo[KE]) + (S.nCO - S.lo[KC]);
    if (n > 0) k_couple_coef<LP><<<(n + 255) / 256, 256, 0, st>>>(S, coef);
    HALO_WROTE(S, F_zb3_cell);
    return hipGetLastError();
}
hipError_t launch_couple_coef_3rd_order(const DevState& S, hipStream_t st, double coef) {
    MPAS_LP_DISPATCH(S.LP, couple_lp, S, st, coef);
}

// ---------------------------------------------------------------- atm_compute_mesh_scaling
// del2 / del4 scaling per edge from the meshDensity of cellOne / cellTwo (the cells of
// cellsOnEdge(0/1), data_structures.rg:486-487); the regional-relaxation factors the task
// also writes are read by no task of the path
__global__ __launch_bounds__(256) void k_mesh_scaling(DevState S, int scale) {
    const int e = ent_of(S, KE);
    if (e >= S.nEO) return;
    double d2 = 1.0, d4 = 1.0;  // :609-612
    if (scale) {  // :614-621
        const int c1 = fi(S, F_cellsOnEdge)[(size_t)e * 2], c2 = fi(S, F_cellsOnEdge)[(size_t)e * 2 + 1];
        const double avg = (fd(S, F_meshDensity)[c1] + fd(S, F_meshDensity)[c2]) / 2.0;
        d2 = 1.0 / pow(avg, 0.25);
        d4 = 1.0 / pow(avg, 0.75);
    }
    fw(S, F_meshScalingDel2)[e] = d2;
    fw(S, F_meshScalingDel4)[e] = d4;
}
hipError_t launch_mesh_scaling(const DevState& S, hipStream_t st, int config_h_ScaleWithMesh) {
    const int ne = S.nEO - S.lo[KE];
    if (ne > 0) k_mesh_scaling<<<(ne + 255) / 256, 256, 0, st>>>(S, config_h_ScaleWithMesh ? 1 : 0);
    return hipGetLastError();
}

}  // namespace mpas
