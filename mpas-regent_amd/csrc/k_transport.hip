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
// Column slot = (entity, scalar pair): the 8 scalars of an entity are stored as 4 pair
// columns (scalars 2q, 2q+1 of a level in one 16-B element: vidx in mpas_dev.h); a
// wavefront computes one pair (one 16-B lane load per gathered entity, from a wave-uniform
// address: the gathers cost per load instruction), and the 4 wavefronts of an
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
// trorder R >= 2: pair-major within runs of R consecutive entities (the run's entities for
// pair 0, then pair 1, ...), each run on one XCD: the waves in flight on an XCD share a
// quarter of the per-entity footprint and the run's mesh data stays in its L2 across the
// four pairs
// entity and pair of column slot `slot` (of (nXO - lo) * 4 slots) in the order option
// "trorder" selects
// (the edge kernel's order: option "trorder_e" when set, else "trorder")
__device__ __forceinline__ int tro_of(const DevState& S, int kind) { return kind == KE && S.troe ? S.troe : S.tro; }
__device__ __forceinline__ void tr_map(const DevState& S, int kind, int slot, int& ent, int& p) {
    const int n = (kind == KC ? S.nCO : S.nEO) - S.lo[kind];
    const int tro = tro_of(S, kind);
    if (tro >= 2) {
        const int R = tro, per = (NSC / 2) * R;  // slots per run
        const int run = slot / per, m = min(R, n - run * R);
        if (m <= 0) {
            ent = 0x7fffffff;  // past the last run (caller returns)
            p = 0;
            return;
        }
        const int within = slot - run * per, q = within / m;
        ent = run * R + (within - q * m) + S.lo[kind];
        p = q * 2;
        if (q >= NSC / 2) ent = 0x7fffffff;
    } else if (tro) {
        const int q = slot / n;
        ent = slot - q * n + S.lo[kind];
        p = q * 2;
        if (q >= NSC / 2) ent = 0x7fffffff;  // past the grid's last slot (caller returns)
    } else {
        ent = (slot >> 2) + S.lo[kind];
        p = (slot & 3) * 2;
    }
}
// the first of this wavefront's EPW consecutive column slots (a block holds 256 / LP * EPW
// slots; with trorder R >= 2 one XCD takes each run's blocks)
template <int LP, int EPW = 1>
__device__ __forceinline__ int tr_slot0(const DevState& S, int kind) {
    constexpr int SPB = 256 / LP * EPW;  // slots per block
    const int tro = tro_of(S, kind);
    const int on = tro >= 2 ? ((NSC / 2) * tro + SPB - 1) / SPB : S.xcd;
    return col_of<LP>(xcd_block(on)) * EPW;
}
template <int LP>
__device__ __forceinline__ void tr_slot(const DevState& S, int kind, int& ent, int& p) {
    tr_map(S, kind, tr_slot0<LP>(S, kind), ent, p);
}

// The x8 fields in their pair layout (vidx in mpas_dev.h): scalars p and p + 1 (p even)
// of entity ent at level k are one 16-B element.  A wavefront (lane = level) loads or
// stores both with one 16-B access per lane; the column's address is wave-uniform (ent
// and p are: SGPRs) and the lane's level is the offset -- no permlane exchange, no per-lane
// column select (64-bit: the edge scratch exceeds 4 GiB on the largest meshes).
// Only levels 0..L-1 are read or written (the transport never uses level L or the
// padding): the lanes k >= L neither load (their values are 0) nor store, so the scratch
// (A, R+, R-, su; never uploaded) packs its pair columns at pitch L instead of LP
// (undecomposed contexts) -- at 56 levels 7/8 of the bytes of every column access.
struct Px {
    int pitch, L;  // pair-column pitch (elements) and live lanes (levels 0..L-1)
};
template <int LP>
__device__ __forceinline__ Px px_pub(int L) { return Px{LP, L}; }          // scalars_old, scalars
template <int LP>
__device__ __forceinline__ Px px_scr(const DevState& S) {  // X_Ah, X_Rp, X_Rm, X_su
    // (a decomposed mesh keeps pitch LP: the halo moves an x8 entity as its 8 x LP block)
    return Px{LP == 64 && !S.halo ? S.L : LP, S.L};
}
template <int LP>
__device__ __forceinline__ double2* pcol(Px x, const double* f, int ent, int p) {
    return (double2*)f + ((size_t)(uint32_t)ent * (NSC / 2) + (size_t)(p >> 1)) * (size_t)x.pitch;
}
// The lane mask costs no branch: the column is a raw buffer of L 16-B elements (the
// descriptor's range is the column, built in SGPRs), so a lane k >= L is out of range --
// its load returns 0 and fetches nothing, its store is dropped.  (Bounds-checked build:
// the same through a branch and MPAS_CHK.)
template <int LP>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t prsrc(Px x, const double* f, int ent, int p) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)pcol<LP>(x, f, ent, p), 0, x.L * 16, 0x00020000);
}
template <int LP>
__device__ __forceinline__ void ld2(Px x, const double* f, int ent, int p, int k, double& a, double& b) {
#if MPAS_BOUNDS
    double2 t = make_double2(0.0, 0.0);
    if (k < x.L) t = *(const double2*)MPAS_CHK(f, pcol<LP>(x, f, ent, p) + k, 16);
#else
    const double2 t = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(prsrc<LP>(x, f, ent, p), k * 16, 0, 0));
#endif
    a = t.x;
    b = t.y;
}
template <int LP>
__device__ __forceinline__ void st2(Px x, double* f, int ent, int p, int k, double a, double b) {
#if MPAS_BOUNDS
    if (k < x.L) *(double2*)MPAS_CHK(f, pcol<LP>(x, f, ent, p) + k, 16) = make_double2(a, b);
#else
    using u4 = __attribute__((ext_vector_type(4))) unsigned;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, make_double2(a, b)), prsrc<LP>(x, f, ent, p), k * 16, 0, 0);
#endif
}
// scalar i of entity ent at level k < L (one 8-B element of the pair layout; the tiled
// kernels)
template <int LP>
__device__ __forceinline__ double& sat(Px x, const double* f, int ent, int i, int k) {
    return *(double*)MPAS_CHK(f, (double*)(pcol<LP>(x, f, ent, i) + k) + (i & 1), 8);
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

// EPW consecutive slots per wavefront (option "trepw" = 2: two edges of one pair, every
// load of both issued before either is computed -- twice the gathers in flight per wave and
// the record round trip paid once per two edges; the same expressions)
template <int LP, int EPW>
__global__ __launch_bounds__(256) void k_tr_edge_n(DevState S) {
    const int L = S.L, k = (int)(threadIdx.x % LP);
    const Px XP = px_pub<LP>(L), XS = px_scr<LP>(S);
    const int s0 = tr_slot0<LP, EPW>(S, KE);
    int e_[EPW], p_[EPW];
#pragma unroll
    for (int i = 0; i < EPW; i++) tr_map(S, KE, s0 + i, e_[i], p_[i]);
    if (e_[0] >= S.nEO) return;
    const double* so = fd(S, S.trsave ? F_scalars : F_scalars_old);  // (trsave: scalars holds the old values)
    int na_[EPW], c1_[EPW], c2_[EPW], adv[EPW][AF];
    double ac[EPW][AF], ac3[EPW][AF], dv_[EPW], u_[EPW], xa[EPW][AF], xb[EPW][AF];
#pragma unroll
    for (int i = 0; i < EPW; i++) {
        const int e = e_[i] < S.nEO ? e_[i] : e_[0];  // (a slot past the end: loads edge e_[0], stores nothing)
        const int* rec = fi(S, X_eB) + (size_t)e * 24;
        c1_[i] = rec[0], c2_[i] = rec[1], na_[i] = rec[22];
#pragma unroll
        for (int j = 0; j < AF; j++) adv[i][j] = rec[12 + j];
        row_ld(fd(S, F_adv_coefs) + (size_t)e * 15, ac[i]);
        row_ld(fd(S, F_adv_coefs_3rd) + (size_t)e * 15, ac3[i]);
        dv_[i] = fd(S, F_dvEdge)[e];
        u_[i] = colk(fd(S, F_ruAvg), e);
#pragma unroll
        for (int j = 0; j < AF; j++) ld2<LP>(XP, so, adv[i][j], p_[i], k, xa[i][j], xb[i][j]);
    }
#pragma unroll
    for (int i = 0; i < EPW; i++) {
        if (e_[i] >= S.nEO) break;
        const int e = e_[i], p = p_[i], na = na_[i], c1 = c1_[i], c2 = c2_[i];
        const double u = u_[i], dv = dv_[i];
        double s1a, s1b, s2a, s2b;
        if (na >= 2 && adv[i][0] == c1 && adv[i][1] == c2) {
            s1a = xa[i][0], s1b = xb[i][0], s2a = xa[i][1], s2b = xb[i][1];
        } else {
            ld2<LP>(XP, so, c1, p, k, s1a, s1b);
            ld2<LP>(XP, so, c2, p, k, s2a, s2b);
        }
        const double sgn = copysign(1.0, u);
        double acca = 0.0, accb = 0.0;
#pragma unroll
        for (int j = 0; j < AF; j++) {
            const double wgt = ac[i][j] + sgn * ac3[i][j];
            acca = add_if(j < na, acca, wgt * xa[i][j]);
            accb = add_if(j < na, accb, wgt * xb[i][j]);
        }
        for (int j = AF; j < na; j++) {
            const int cj = fi(S, F_advCellsForEdge)[(size_t)e * 15 + j];
            const double wgt = fd(S, F_adv_coefs)[(size_t)e * 15 + j] + sgn * fd(S, F_adv_coefs_3rd)[(size_t)e * 15 + j];
            double ya, yb;
            ld2<LP>(XP, so, cj, p, k, ya, yb);
            acca = acca + wgt * ya;
            accb = accb + wgt * yb;
        }
        const double loa = dv * (fmax(u, 0.0) * s1a + fmin(u, 0.0) * s2a);
        const double lob = dv * (fmax(u, 0.0) * s1b + fmin(u, 0.0) * s2b);
        st2<LP>(XS, fw(S, X_Ah), e, p, k, PADW(u * acca - loa), PADW(u * accb - lob));
    }
}

template <int LP>
__global__ __launch_bounds__(256) void k_tr_edge(DevState S) {
    int e, p;
    tr_slot<LP>(S, KE, e, p);
    const int L = S.L, k = (int)(threadIdx.x % LP);
    const Px XP = px_pub<LP>(L), XS = px_scr<LP>(S);
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
    const double* so = fd(S, S.trsave ? F_scalars : F_scalars_old);  // (trsave: scalars holds the old values)
    const double u = colk(fd(S, F_ruAvg), e);
    double xa[AF], xb[AF], s1a, s1b, s2a, s2b;
#pragma unroll
    for (int j = 0; j < AF; j++) ld2<LP>(XP, so, adv[j], p, k, xa[j], xb[j]);
    // the upwind flux's two cells are normally advCellsForEdge(0) and (1) (MPAS's list
    // construction): take their columns from the list; gather them only where they are not
    // (wave-uniform branch, the same column either way)
    if (na >= 2 && adv[0] == c1 && adv[1] == c2) {
        s1a = xa[0], s1b = xb[0], s2a = xa[1], s2b = xb[1];
    } else {
        ld2<LP>(XP, so, c1, p, k, s1a, s1b);
        ld2<LP>(XP, so, c2, p, k, s2a, s2b);
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
        ld2<LP>(XP, so, cj, p, k, ya, yb);
        acca = acca + wgt * ya;
        accb = accb + wgt * yb;
    }
    const double loa = dv * (fmax(u, 0.0) * s1a + fmin(u, 0.0) * s2a);
    const double lob = dv * (fmax(u, 0.0) * s1b + fmin(u, 0.0) * s2b);
    st2<LP>(XS, fw(S, X_Ah), e, p, k, PADW(u * acca - loa), PADW(u * accb - lob));
}

// k_tr_edge with the scalars_old columns staged in LDS (option "tredge", opt-in: measured
// 2-9 % slower over the transport than the direct gathers at 8-16 edges per group, DESIGN.md
// §7; LP = 64,
// undecomposed; TrEdgeGroups in mpas_dev.h).  A block is one (group of TRE_GE consecutive
// edges, scalar pair): its 4 wavefronts first copy the union's column pairs into LDS (one
// 16-B lane load per cell: ~36 loads for the group's 144 advCell gathers), then each
// computes every fourth edge of the group from LDS with k_tr_edge's expressions in its
// order (the same bits).  The gathers were what bounded k_tr_edge (one 1-KB request per
// advCell and scalar pair, served by the L2); LDS reads cost no memory requests.  An
// irregular group (union > TRE_U, or an edge with more than AF advCells) gathers directly.
struct TreK {
    const int* ucell;
    const int* ucnt;
    const unsigned* eslot;
    int ngroups;
};
__global__ __launch_bounds__(256) void k_tr_edge_lds(DevState S, TreK T) {
    constexpr int LP = 64, NW = 4, NL = (TRE_U + NW - 1) / NW, EW = TRE_GE / NW;
    static_assert(TRE_GE % NW == 0, "edges per wavefront");
    __shared__ double2 lds[TRE_U * LP];
    const int b = xcd_block_n(S.xcd, (int)blockIdx.x, (int)gridDim.x);
    const int g = b >> 2, p = (b & 3) * 2;
    if (g >= T.ngroups) return;
    const int L = S.L, k = (int)(threadIdx.x % LP), w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / LP));
    const Px XP = px_pub<LP>(L), XS = px_scr<LP>(S);
    const int nu = T.ucnt[g];
    const double* so = fd(S, F_scalars_old);
    const int e0 = g * TRE_GE, ne = min(TRE_GE, S.nEO - e0);
    // this wavefront's edges e0 + w, + NW, ...: their mass flux columns first, so that the
    // loads overlap the staging (edges past the owned range load edge e0's and store nothing)
    double u_[EW];
#pragma unroll
    for (int i = 0; i < EW; i++) {
        const int q = w + i * NW;
        u_[i] = colk(fd(S, F_ruAvg), e0 + (q < ne ? q : 0));
    }
    if (nu >= 0) {  // (block-uniform) stage the union: every load first, then the LDS stores
        const int* uc = T.ucell + (size_t)g * TRE_U;
        double a_[NL], b_[NL];
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int s = w + i * NW;
            const int cell = uc[s < TRE_U ? s : 0];
            ld2<LP>(XP, so, cell, p, k, a_[i], b_[i]);
        }
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int s = w + i * NW;
            if (s < nu) lds[s * LP + k] = make_double2(a_[i], b_[i]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < EW; i++) {
        const int q = w + i * NW;
        if (q >= ne) break;
        const int e = e0 + q;
        const int* rec = fi(S, X_eB) + (size_t)e * 24;  // cellsOnEdge(2) .. advCellsForEdge(9) @12, nAdv @22
        const int c1 = rec[0], c2 = rec[1], na = rec[22];
        double ac[AF], ac3[AF];
        row_ld(fd(S, F_adv_coefs) + (size_t)e * 15, ac);
        row_ld(fd(S, F_adv_coefs_3rd) + (size_t)e * 15, ac3);
        const double dv = fd(S, F_dvEdge)[e];
        const double u = u_[i];
        double xa[AF], xb[AF], s1a, s1b, s2a, s2b;
        if (nu >= 0) {
            unsigned sl[TRE_ROW / 4];
#pragma unroll
            for (int j = 0; j < TRE_ROW / 4; j++) sl[j] = T.eslot[(size_t)e * (TRE_ROW / 4) + j];
            auto slot = [&](int j) { return (int)((sl[j >> 2] >> ((j & 3) * 8)) & 0xffu); };
#pragma unroll
            for (int j = 0; j < AF; j++) {
                const double2 v = lds[slot(j) * LP + k];
                xa[j] = v.x, xb[j] = v.y;
            }
            const double2 v1 = lds[slot(AF) * LP + k], v2 = lds[slot(AF + 1) * LP + k];
            s1a = v1.x, s1b = v1.y, s2a = v2.x, s2b = v2.y;
        } else {
            int adv[AF];
#pragma unroll
            for (int j = 0; j < AF; j++) adv[j] = rec[12 + j];
#pragma unroll
            for (int j = 0; j < AF; j++) ld2<LP>(XP, so, adv[j], p, k, xa[j], xb[j]);
            ld2<LP>(XP, so, c1, p, k, s1a, s1b);
            ld2<LP>(XP, so, c2, p, k, s2a, s2b);
        }
        const double sgn = copysign(1.0, u);
        double acca = 0.0, accb = 0.0;
#pragma unroll
        for (int j = 0; j < AF; j++) {
            const double wgt = ac[j] + sgn * ac3[j];
            acca = add_if(j < na, acca, wgt * xa[j]);
            accb = add_if(j < na, accb, wgt * xb[j]);
        }
        for (int j = AF; j < na; j++) {  // (irregular groups only)
            const int cj = fi(S, F_advCellsForEdge)[(size_t)e * 15 + j];
            const double wgt = fd(S, F_adv_coefs)[(size_t)e * 15 + j] + sgn * fd(S, F_adv_coefs_3rd)[(size_t)e * 15 + j];
            double ya, yb;
            ld2<LP>(XP, so, cj, p, k, ya, yb);
            acca = acca + wgt * ya;
            accb = accb + wgt * yb;
        }
        const double loa = dv * (fmax(u, 0.0) * s1a + fmin(u, 0.0) * s2a);
        const double lob = dv * (fmax(u, 0.0) * s1b + fmin(u, 0.0) * s2b);
        st2<LP>(XS, fw(S, X_Ah), e, p, k, PADW(u * acca - loa), PADW(u * accb - lob));
    }
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

// SU (option "trsu"): su is not stored; k_tr_update forms it again from the same values
template <int LP, bool SELF, bool SU>
__global__ __launch_bounds__(256) void k_tr_bounds(DevState S, double dt) {
    int c, p;
    tr_slot<LP>(S, KC, c, p);
    const int L = S.L, k = (int)(threadIdx.x % LP);
    const Px XP = px_pub<LP>(L), XS = px_scr<LP>(S);
    if (c >= S.nCO) return;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    TrSlots t;
    tr_slots(S, c, t);
    const double invA = fd(S, F_invAreaCell)[c];
    const double rdzw = fd(S, F_rdzw)[k], fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    // (trsave, wave-uniform: scalars holds the old values; the cell's whole pair column, every level and
    // the padding, is stored to scalars_old at the end -- scalars_save's copy of it)
    const bool save = S.trsave != 0;
    const double *so = fd(S, save ? F_scalars : F_scalars_old), *ru = fd(S, F_ruAvg);
    const double* Ah = fd(S, X_Ah);
    const Px XF{LP, LP};
    double sa, sb, fa = 0.0, fb = 0.0;
    if (save) {
        ld2<LP>(XF, so, c, p, k, fa, fb);
        sa = k < L ? fa : 0.0;
        sb = k < L ? fb : 0.0;
    } else {
        ld2<LP>(XP, so, c, p, k, sa, sb);
    }
    const double w = colk(fd(S, F_wwAvg), c), r_o = colk(fd(S, F_rho_zz_old_split), c), r_n = colk(fd(S, F_rho_zz), c);
    double u_[NF], x1a[NF], x2a[NF], x1b[NF], x2b[NF], Aa[NF], Ab[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        u_[i] = colk(ru, t.e[i]);
        ld2<LP>(XS, Ah, t.e[i], p, k, Aa[i], Ab[i]);
        if constexpr (SELF) {
            double xa, xb;
            ld2<LP>(XP, so, t.oth[i], p, k, xa, xb);
            x1a[i] = t.s1[i] ? sa : xa;
            x2a[i] = t.s1[i] ? xa : sa;
            x1b[i] = t.s1[i] ? sb : xb;
            x2b[i] = t.s1[i] ? xb : sb;
        } else {
            ld2<LP>(XP, so, t.c1[i], p, k, x1a[i], x1b[i]);
            ld2<LP>(XP, so, t.c2[i], p, k, x2a[i], x2b[i]);
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
        ld2<LP>(XP, so, c1, p, k, y1a, y1b);
        ld2<LP>(XP, so, c2, p, k, y2a, y2b);
        ld2<LP>(XS, Ah, e, p, k, Ba, Bb);
        tr_bound_slot(true, s1f, dv, u, y1a, y2a, Ba, ra);
        tr_bound_slot(true, s1f, dv, u, y1b, y2b, Bb, rb);
    }
    double Rpa, Rma, sua, Rpb, Rmb, sub;
    tr_bound_fin<LP>(ra, sa, w, r_o, r_n, invA, rdzw, fzm, fzp, dt, k, L, Rpa, Rma, sua);
    tr_bound_fin<LP>(rb, sb, w, r_o, r_n, invA, rdzw, fzm, fzp, dt, k, L, Rpb, Rmb, sub);
    // level L and the padding levels of the scratch are never read
    st2<LP>(XS, fw(S, X_Rp), c, p, k, Rpa, Rpb);
    st2<LP>(XS, fw(S, X_Rm), c, p, k, Rma, Rmb);
    if constexpr (!SU) st2<LP>(XS, fw(S, X_su), c, p, k, sua, sub);
    if (save) {
        st2<LP>(XF, fw(S, F_scalars_old), c, p, k, fa, fb);
        if (c == S.nCells - 1) {  // (and the zero slot's column, as the copy of the whole array)
            double za, zb;
            ld2<LP>(XF, so, S.nCells, p, k, za, zb);
            st2<LP>(XF, fw(S, F_scalars_old), S.nCells, p, k, za, zb);
        }
    }
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

// SU (option "trsu"): su formed here as k_tr_bounds forms it -- the upwind sum over the
// cell's edges (tr_bound_slot's order) and tr_bound_fin's expression -- instead of read
// from X_su: the same values, one scratch array fewer (written once, read once)
template <int LP, bool SELF, bool SU>
__global__ __launch_bounds__(256) void k_tr_update(DevState S, double dt) {
    int c, p;
    tr_slot<LP>(S, KC, c, p);
    const int L = S.L, k = (int)(threadIdx.x % LP);
    const Px XP = px_pub<LP>(L), XS = px_scr<LP>(S);
    if (c >= S.nCO) return;
    const int ne = fi(S, F_nEdgesOnCell)[c];
    TrSlots t;
    tr_slots(S, c, t);
    const double invA = fd(S, F_invAreaCell)[c];
    const double rdzw = fd(S, F_rdzw)[k], fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double *Ah = fd(S, X_Ah), *Rp = fd(S, X_Rp), *Rm = fd(S, X_Rm);
    const double* so = fd(S, F_scalars_old);
    double sa, sb, sua = 0.0, sub = 0.0, rpa, rpb, rma, rmb;
    ld2<LP>(XP, so, c, p, k, sa, sb);
    if constexpr (!SU) ld2<LP>(XS, fd(S, X_su), c, p, k, sua, sub);
    ld2<LP>(XS, Rp, c, p, k, rpa, rpb);
    ld2<LP>(XS, Rm, c, p, k, rma, rmb);
    const double w = colk(fd(S, F_wwAvg), c), r_n = colk(fd(S, F_rho_zz), c);
    if constexpr (SU) {  // su (k_tr_bounds: tr_bound_slot's upwind sum, tr_bound_fin)
        const double* ru = fd(S, F_ruAvg);
        const double r_o = colk(fd(S, F_rho_zz_old_split), c);
        double u_[NF], x1a[NF], x2a[NF], x1b[NF], x2b[NF];
#pragma unroll
        for (int i = 0; i < NF; i++) {
            u_[i] = colk(ru, t.e[i]);
            if constexpr (SELF) {
                double xa, xb;
                ld2<LP>(XP, so, t.oth[i], p, k, xa, xb);
                x1a[i] = t.s1[i] ? sa : xa;
                x2a[i] = t.s1[i] ? xa : sa;
                x1b[i] = t.s1[i] ? sb : xb;
                x2b[i] = t.s1[i] ? xb : sb;
            } else {
                ld2<LP>(XP, so, t.c1[i], p, k, x1a[i], x1b[i]);
                ld2<LP>(XP, so, t.c2[i], p, k, x2a[i], x2b[i]);
            }
        }
        double hla = 0.0, hlb = 0.0;
        auto up = [](bool on, int s1f, double dv, double u, double x1, double x2, double& hlo) {
            const double sg = s1f ? 1.0 : -1.0;
            const double lo = dv * (fmax(u, 0.0) * x1 + fmin(u, 0.0) * x2);
            hlo = add_if(on, hlo, sg * lo);
        };
#pragma unroll
        for (int i = 0; i < NF; i++) {
            up(i < ne, t.s1[i], t.dv[i], u_[i], x1a[i], x2a[i], hla);
            up(i < ne, t.s1[i], t.dv[i], u_[i], x1b[i], x2b[i], hlb);
        }
        for (int i = NF; i < ne; i++) {
            const size_t r = (size_t)c * 10 + i;
            const int e = fi(S, F_edgesOnCell)[r], c1 = fi(S, X_ce_c1)[r], c2 = fi(S, X_ce_c2)[r];
            const int s1f = fi(S, X_ce_s1)[r];
            const double dv = fd(S, X_ce_dv)[r], u = colk(ru, e);
            double y1a, y1b, y2a, y2b;
            ld2<LP>(XP, so, c1, p, k, y1a, y1b);
            ld2<LP>(XP, so, c2, p, k, y2a, y2b);
            up(true, s1f, dv, u, y1a, y2a, hla);
            up(true, s1f, dv, u, y1b, y2b, hlb);
        }
        double loa, Aa_, lob, Ab_;
        tr_vflux<LP>(sa, w, k, L, fzm, fzp, loa, Aa_);
        tr_vflux<LP>(sb, w, k, L, fzm, fzp, lob, Ab_);
        const double lota = lvl_up<LP>(loa, k), lotb = lvl_up<LP>(lob, k);
        sua = (sa * r_o - dt * (hla * invA + (lota - loa) * rdzw)) / r_n;
        sub = (sb * r_o - dt * (hlb * invA + (lotb - lob) * rdzw)) / r_n;
    }
    double Aa[NF], Ab[NF], p1a[NF], p1b[NF], m1a[NF], m1b[NF], p2a[NF], p2b[NF], m2a[NF], m2b[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        ld2<LP>(XS, Ah, t.e[i], p, k, Aa[i], Ab[i]);
        if constexpr (SELF) {  // the cell is one of the two: gather only the other
            double qa, qb, na, nb;
            ld2<LP>(XS, Rp, t.oth[i], p, k, qa, qb);
            ld2<LP>(XS, Rm, t.oth[i], p, k, na, nb);
            const bool f = t.s1[i];
            p1a[i] = f ? rpa : qa, p1b[i] = f ? rpb : qb, m1a[i] = f ? rma : na, m1b[i] = f ? rmb : nb;
            p2a[i] = f ? qa : rpa, p2b[i] = f ? qb : rpb, m2a[i] = f ? na : rma, m2b[i] = f ? nb : rmb;
        } else {
            ld2<LP>(XS, Rp, t.c1[i], p, k, p1a[i], p1b[i]);
            ld2<LP>(XS, Rm, t.c1[i], p, k, m1a[i], m1b[i]);
            ld2<LP>(XS, Rp, t.c2[i], p, k, p2a[i], p2b[i]);
            ld2<LP>(XS, Rm, t.c2[i], p, k, m2a[i], m2b[i]);
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
        ld2<LP>(XS, Ah, e, p, k, Ba, Bb);
        ld2<LP>(XS, Rp, c1, p, k, q1a, q1b);
        ld2<LP>(XS, Rm, c1, p, k, n1a, n1b);
        ld2<LP>(XS, Rp, c2, p, k, q2a, q2b);
        ld2<LP>(XS, Rm, c2, p, k, n2a, n2b);
        hca = hca + sg * tr_limited(Ba, n1a, q2a, q1a, n2a);
        hcb = hcb + sg * tr_limited(Bb, n1b, q2b, q1b, n2b);
    }
    const double na = tr_update_fin<LP>(hca, sa, w, sua, rpa, rma, r_n, invA, rdzw, fzm, fzp, dt, k, L);
    const double nb = tr_update_fin<LP>(hcb, sb, w, sub, rpb, rmb, r_n, invA, rdzw, fzm, fzp, dt, k, L);
    if (k < L) st2<LP>(XP, fw(S, F_scalars), c, p, k, na, nb);  // level L keeps its value (the oracle writes 0..L-1)
}

// ---------------------------------------------------------------- tiled transport
// Opt-in (option "trtile"; measured 2x slower than the three kernels above at x1.163842:
// the traffic halves but A is computed four times per edge).
// Two kernels and no edge scratch: a block is one (tile,
// scalar) pair (TrTiles, mpas_dev.h).  It loads the scalars_old columns of its tile's
// closure into LDS, then each cell of the tile forms the antidiffusive flux A of each of
// its edges from LDS with k_tr_edge's expression -- the edge's A is computed by both of its
// cells instead of stored once and gathered twice --, and
//   k_trt_bounds  su, the bounds and R+ / R- (k_tr_bounds' expressions; R+ / R- stored)
//   k_trt_update  su again, each A limited with R+ / R- of the edge's cells (gathered),
//                 the new scalars (k_tr_update's expressions)
// The same operations on the same values as the three kernels above: bit-identical.  Used
// when every owned cell has at most NF edges and each of them at most AF advCells.
struct TrtK {
    const int *tptr, *tcell, *cptr, *ccell;
    const int* slot;
    int t0;
};
constexpr int TRT_THREADS = 1024;
constexpr int TRT_WAVES = 8;  // min waves per SIMD (VGPR cap 64): two 16-wave blocks per CU, one tile cell per wave

// this lane's column slot of the block (wave-uniform at LP = 64: SGPR)
template <int LP>
__device__ __forceinline__ int trt_slot() {
    int s = (int)(threadIdx.x / LP);
    if constexpr (LP == 64) s = __builtin_amdgcn_readfirstlane(s);
    return s;
}

// (ldc, the constant-address-space load of the mesh rows and the tile tables: mpas_dev.h)

// The mesh data of one tile cell (LP = 64: every index is wave-uniform, so all of it
// comes through the scalar unit).
template <int LP>
struct TrtCell {
    int c, ne;
    const int* row;
    size_t r;
    const DevState* S;

    __device__ __forceinline__ void load(const DevState& S_, const TrtK& T, int qi, int k) {
        (void)k;
        S = &S_;
        if constexpr (LP == 64) qi = __builtin_amdgcn_readfirstlane(qi);
        c = ldc(T.tcell + qi);
        ne = ldc(fi(*S, F_nEdgesOnCell) + c);
        row = T.slot + (size_t)qi * TRT_ROW;
        r = (size_t)c * 10;
    }
    __device__ __forceinline__ int slot(int idx) const { return ldc(row + idx); }
    __device__ __forceinline__ int e(int i) const { return ldc(fi(*S, F_edgesOnCell) + r + i); }
    __device__ __forceinline__ int s1(int i) const { return ldc(fi(*S, X_ce_s1) + r + i); }
    __device__ __forceinline__ int oth(int i) const { return ldc(fi(*S, X_ce_oth) + r + i); }
    __device__ __forceinline__ int c1(int i) const { return ldc(fi(*S, X_ce_c1) + r + i); }
    __device__ __forceinline__ int c2(int i) const { return ldc(fi(*S, X_ce_c2) + r + i); }
    __device__ __forceinline__ double dv(int i) const { return ldc(fd(*S, X_ce_dv) + r + i); }
    __device__ __forceinline__ int na(int i) const { return ldc(fi(*S, F_nAdvCellsForEdge) + e(i)); }
    __device__ __forceinline__ double ac(int i, int j) const { return ldc(fd(*S, F_adv_coefs) + (size_t)e(i) * 15 + j); }
    __device__ __forceinline__ double ac3(int i, int j) const {
        return ldc(fd(*S, F_adv_coefs_3rd) + (size_t)e(i) * 15 + j);
    }
};

// the closure columns of scalar sc of the tile into LDS (column i at lds[i * LP], level
// order); two columns per 16-B lane load at LP = 64 (ld2)
template <int LP>
__device__ __forceinline__ void trt_load(const DevState& S, const TrtK& T, int tile, int sc, double* lds) {
    constexpr int NS = TRT_THREADS / LP, U = 4;
    const int k = (int)(threadIdx.x % LP), slot = trt_slot<LP>();
    const Px XP = px_pub<LP>(S.L);
    const int cb = T.cptr[tile], n = T.cptr[tile + 1] - cb;
    const double* so = fd(S, F_scalars_old);
    for (int i0 = 2 * slot; i0 < n; i0 += 2 * U * NS) {
        double a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + 2 * u * NS;
            const int ca = T.ccell[cb + (i < n ? i : 0)], cbb = T.ccell[cb + (i + 1 < n ? i + 1 : 0)];
            a[u] = sat<LP>(XP, so, ca, sc, k), b[u] = sat<LP>(XP, so, cbb, sc, k);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + 2 * u * NS;
            if (i < n) lds[i * LP + k] = a[u];
            if (i + 1 < n) lds[(i + 1) * LP + k] = b[u];
        }
    }
    __syncthreads();
}

// edge slot i of one tile cell: the mass flux u, the scalar at cellsOnEdge(0/1) (x1, x2)
// and the antidiffusive flux A (k_tr_edge: high-order - upwind, PADW as stored in X_Ah)
template <int LP>
__device__ __forceinline__ double trt_flux(const double* lds, const TrtCell<LP>& t, int i, double u, int k, int L,
                                           double& x1, double& x2) {
    const int b = 1 + i * (2 + AF), na = t.na(i);
    x1 = lds[t.slot(b) * LP + k];
    x2 = lds[t.slot(b + 1) * LP + k];
    const double sgn = copysign(1.0, u);
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < AF; j++) {
        const double wgt = t.ac(i, j) + sgn * t.ac3(i, j);
        acc = add_if(j < na, acc, wgt * lds[t.slot(b + 2 + j) * LP + k]);
    }
    const double lo = t.dv(i) * (fmax(u, 0.0) * x1 + fmin(u, 0.0) * x2);
    return PADW(u * acc - lo);
}

// The edge slots of a cell run as a loop (not unrolled: the scalar registers of one slot's
// coefficients and LDS columns, ~40, would otherwise be live for all six at once and
// spill); the global loads of slot i + 1 are issued before slot i is computed.
template <int LP>
__global__ __launch_bounds__(TRT_THREADS, TRT_WAVES) void k_trt_bounds(DevState S, TrtK T, double dt) {
    extern __shared__ double lds[];
    const int v = xcd_block(S.xcd), tile = T.t0 + v / NSC, sc = v % NSC;
    trt_load<LP>(S, T, tile, sc, lds);
    constexpr int NS = TRT_THREADS / LP;
    const int L = S.L, k = (int)(threadIdx.x % LP), slot = trt_slot<LP>();
    const Px XP = px_pub<LP>(L), XS = px_scr<LP>(S);
    const double rdzw = fd(S, F_rdzw)[k], fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double* ru = fd(S, F_ruAvg);
    const int tb = T.tptr[tile], nt = T.tptr[tile + 1] - tb;
    for (int q = slot; q < nt; q += NS) {
        TrtCell<LP> t;
        t.load(S, T, tb + q, k);
        const int c = t.c;
        const double invA = fd(S, F_invAreaCell)[c];
        const double w = colk(fd(S, F_wwAvg), c), r_o = colk(fd(S, F_rho_zz_old_split), c),
                     r_n = colk(fd(S, F_rho_zz), c);
        const double s = lds[t.slot(0) * LP + k];
        TrAcc r;
        r.smax = r.smin = s;
        // slots past nEdgesOnCell change nothing in k_tr_bounds (every update is masked)
        const int ne = t.ne < NF ? t.ne : NF;
        double un = colk(ru, t.e(0));
#pragma unroll 1
        for (int i = 0; i < ne; i++) {
            const double u = un;
            if (i + 1 < ne) un = colk(ru, t.e(i + 1));
            double x1, x2;
            const double A = trt_flux<LP>(lds, t, i, u, k, L, x1, x2);
            tr_bound_slot(true, t.s1(i), t.dv(i), u, x1, x2, A, r);
        }
        double Rp, Rm, su;
        tr_bound_fin<LP>(r, s, w, r_o, r_n, invA, rdzw, fzm, fzp, dt, k, L, Rp, Rm, su);
        if (k < L) {  // (the scratch holds levels 0..L-1 only: px_scr)
            sat<LP>(XS, fw(S, X_Rp), c, sc, k) = Rp;
            sat<LP>(XS, fw(S, X_Rm), c, sc, k) = Rm;
        }
    }
}

// R+ and R- of the two cells of edge slot i: p1/m1 at cellsOnEdge(0), p2/m2 at (1)
template <int LP, bool SELF>
__device__ __forceinline__ void trt_r(Px XS, const double* Rp, const double* Rm, const TrtCell<LP>& t, int i, int sc,
                                      double rp, double rm, int k, double& p1, double& m1, double& p2, double& m2) {
    if constexpr (SELF) {  // the cell is one of the two: gather only the other
        const int co = t.oth(i);
        const double qo = sat<LP>(XS, Rp, co, sc, k), no = sat<LP>(XS, Rm, co, sc, k);
        const bool f = t.s1(i);
        p1 = f ? rp : qo, m1 = f ? rm : no, p2 = f ? qo : rp, m2 = f ? no : rm;
    } else {
        const int c1 = t.c1(i), c2 = t.c2(i);
        p1 = sat<LP>(XS, Rp, c1, sc, k), m1 = sat<LP>(XS, Rm, c1, sc, k);
        p2 = sat<LP>(XS, Rp, c2, sc, k), m2 = sat<LP>(XS, Rm, c2, sc, k);
    }
}

template <int LP, bool SELF>
__global__ __launch_bounds__(TRT_THREADS, TRT_WAVES) void k_trt_update(DevState S, TrtK T, double dt) {
    extern __shared__ double lds[];
    const int v = xcd_block(S.xcd), tile = T.t0 + v / NSC, sc = v % NSC;
    trt_load<LP>(S, T, tile, sc, lds);
    constexpr int NS = TRT_THREADS / LP;
    const int L = S.L, k = (int)(threadIdx.x % LP), slot = trt_slot<LP>();
    const Px XP = px_pub<LP>(L), XS = px_scr<LP>(S);
    const double rdzw = fd(S, F_rdzw)[k], fzm = fd(S, F_fzm)[k], fzp = fd(S, F_fzp)[k];
    const double *Rp = fd(S, X_Rp), *Rm = fd(S, X_Rm), *ru = fd(S, F_ruAvg);
    const int tb = T.tptr[tile], nt = T.tptr[tile + 1] - tb;
    for (int q = slot; q < nt; q += NS) {
        TrtCell<LP> t;
        t.load(S, T, tb + q, k);
        const int c = t.c;
        const double invA = fd(S, F_invAreaCell)[c];
        const double w = colk(fd(S, F_wwAvg), c), r_o = colk(fd(S, F_rho_zz_old_split), c),
                     r_n = colk(fd(S, F_rho_zz), c);
        const double rp = sat<LP>(XS, Rp, c, sc, k), rm = sat<LP>(XS, Rm, c, sc, k);
        const double s = lds[t.slot(0) * LP + k];
        // su as k_tr_bounds forms it (tr_bound_slot's upwind sum, tr_bound_fin's update),
        // and the limited antidiffusive sum of k_tr_update (masked slots add nothing)
        const int ne = t.ne < NF ? t.ne : NF;
        double hlo = 0.0, hc = 0.0;
        double un = colk(ru, t.e(0)), p1n, m1n, p2n, m2n;
        trt_r<LP, SELF>(XS, Rp, Rm, t, 0, sc, rp, rm, k, p1n, m1n, p2n, m2n);
#pragma unroll 1
        for (int i = 0; i < ne; i++) {
            const double u = un, p1 = p1n, m1 = m1n, p2 = p2n, m2 = m2n;
            if (i + 1 < ne) {
                un = colk(ru, t.e(i + 1));
                trt_r<LP, SELF>(XS, Rp, Rm, t, i + 1, sc, rp, rm, k, p1n, m1n, p2n, m2n);
            }
            double x1, x2;
            const double A = trt_flux<LP>(lds, t, i, u, k, L, x1, x2);
            const double sg = t.s1(i) ? 1.0 : -1.0;
            const double lo = t.dv(i) * (fmax(u, 0.0) * x1 + fmin(u, 0.0) * x2);
            hlo = hlo + sg * lo;
            hc = hc + sg * tr_limited(A, m1, p2, p1, m2);
        }
        double lob, Ab;
        tr_vflux<LP>(s, w, k, L, fzm, fzp, lob, Ab);
        const double lot = lvl_up<LP>(lob, k);
        const double su = (s * r_o - dt * (hlo * invA + (lot - lob) * rdzw)) / r_n;
        const double sn = tr_update_fin<LP>(hc, s, w, su, rp, rm, r_n, invA, rdzw, fzm, fzp, dt, k, L);
        if (k < L) sat<LP>(XP, fw(S, F_scalars), c, sc, k) = sn;
    }
}

template <int LP>
static hipError_t transport_tiled(const DevState& S, hipStream_t st, double dt) {
    const TrTiles& TT = *S.trt;
    // the tiles of a launch range: all owned cells, or (halo overlap) those of the interior
    // launch (interior cells reading owned columns only) or of the boundary launch (the
    // rest) -- trt_build's launch classes; every owned cell is in exactly one tile
    auto range = [&](const DevState& X, int& t0, int& t1) {
        const int lo = X.lo[KC], hi = X.nCO;
        t0 = t1 = 0;
        if (lo >= hi) return true;
        if (lo == 0 && hi == TT.nco) t1 = TT.ntiles;
        else if (lo == 0 && hi == TT.nint) t1 = TT.nt_int;
        else if (lo == TT.nint && hi == TT.nco) t0 = TT.nt_int, t1 = TT.ntiles;
        else return false;
        return true;
    };
    auto args = [&](int t0) { return TrtK{TT.tptr, TT.tcell, TT.cptr, TT.ccell, TT.slot, t0}; };
    const size_t shm = (size_t)TT.maxclo * LP * sizeof(double);
    hipError_t bad = hipSuccess;
    auto k1 = [&](const DevState& X) {
        int t0, t1;
        if (!range(X, t0, t1)) bad = hipErrorInvalidValue;
        else if (t1 > t0) k_trt_bounds<LP><<<(t1 - t0) * NSC, TRT_THREADS, shm, st>>>(X, args(t0), dt);
    };
    HALO_RUN(S, st, k1, F_scalars_old, F_ruAvg);
    HALO_WROTE(S, X_Rp, X_Rm);
    auto k2 = [&](const DevState& X) {
        int t0, t1;
        if (!range(X, t0, t1)) bad = hipErrorInvalidValue;
        else if (t1 > t0 && X.selfc) k_trt_update<LP, true><<<(t1 - t0) * NSC, TRT_THREADS, shm, st>>>(X, args(t0), dt);
        else if (t1 > t0) k_trt_update<LP, false><<<(t1 - t0) * NSC, TRT_THREADS, shm, st>>>(X, args(t0), dt);
    };
    HALO_RUN(S, st, k2, F_scalars_old, F_ruAvg, X_Rp, X_Rm);
    HALO_WROTE(S, F_scalars);
    return bad != hipSuccess ? bad : hipGetLastError();
}

template <int LP>
static hipError_t transport_lp(const DevState& S0, hipStream_t st, double dt, int fold) {
    DevState S = S0;
    S.trsave = fold;
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
        if constexpr (LP == 64) {
            if (X.tre && !X.halo && X.lo[KE] == 0 && X.tre->neo == X.nEO) {  // (option "tredge")
                const TrEdgeGroups& G = *X.tre;
                if (G.ngroups) k_tr_edge_lds<<<G.ngroups * (NSC / 2), 256, 0, st>>>(X, TreK{G.ucell, G.ucnt, G.eslot, G.ngroups});
                return;
            }
        }
        if (X.trepw == 2) {  // (option "trepw" = 2)
            const long n = (long)(X.nEO - X.lo[KE]) * (NSC / 2);
            const int nb = n > 0 ? (int)((n + 2 * COLS - 1) / (2 * COLS)) : 0;
            if (nb) k_tr_edge_n<LP, 2><<<nb, 256, 0, st>>>(X);
            return;
        }
        const int nb = blocks(X, KE);
        if (nb) k_tr_edge<LP><<<nb, 256, 0, st>>>(X);
    };
    HALO_RUN(S, st, ke, F_scalars_old, F_ruAvg);
    HALO_WROTE(S, X_Ah);
    auto kb = [&](const DevState& X) {
        const int nb = blocks(X, KC);
        if (!nb) return;
        if (X.trsu) {
            if (X.selfc) k_tr_bounds<LP, true, true><<<nb, 256, 0, st>>>(X, dt);
            else k_tr_bounds<LP, false, true><<<nb, 256, 0, st>>>(X, dt);
        } else {
            if (X.selfc) k_tr_bounds<LP, true, false><<<nb, 256, 0, st>>>(X, dt);
            else k_tr_bounds<LP, false, false><<<nb, 256, 0, st>>>(X, dt);
        }
    };
    HALO_RUN(S, st, kb, F_scalars_old, F_ruAvg, X_Ah);
    if (S.trsu) HALO_WROTE(S, X_Rp, X_Rm);
    else HALO_WROTE(S, X_Rp, X_Rm, X_su);
    auto ku = [&](const DevState& X) {
        const int nb = blocks(X, KC);
        if (!nb) return;
        if (X.trsu) {
            if (X.selfc) k_tr_update<LP, true, true><<<nb, 256, 0, st>>>(X, dt);
            else k_tr_update<LP, false, true><<<nb, 256, 0, st>>>(X, dt);
        } else {
            if (X.selfc) k_tr_update<LP, true, false><<<nb, 256, 0, st>>>(X, dt);
            else k_tr_update<LP, false, false><<<nb, 256, 0, st>>>(X, dt);
        }
    };
    if (S.trsu) HALO_RUN(S, st, ku, F_scalars_old, F_ruAvg, X_Ah, X_Rp, X_Rm);
    else HALO_RUN(S, st, ku, X_Ah, X_Rp, X_Rm);
    HALO_WROTE(S, F_scalars);
    return hipGetLastError();
}
hipError_t launch_advance_scalars_mono(const DevState& S, hipStream_t st, double dt, int fold) {
    // (fold: only the default kernels -- undecomposed, no tiles, no LDS edge groups, su stored)
    if (fold && (S.halo || S.trt || S.tre || S.trsu)) return hipErrorInvalidValue;
    if (S.trt) MPAS_LP_DISPATCH(S.LP, transport_tiled, S, st, dt);
    MPAS_LP_DISPATCH(S.LP, transport_lp, S, st, dt, fold);
}

}  // namespace mpas
