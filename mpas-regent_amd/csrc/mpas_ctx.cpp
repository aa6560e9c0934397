// mpas_ctx.cpp -- libmpasdyn host runtime: context, device residency, the C-ABI task
// entry points of include/mpas_dyn.h, and the atm_srk3 driver (rk_timestep.rg:361-500).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <memory>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "mpas_dev.h"
#include "mpas_halo.h"
#include "mpas_dyn.h"

namespace mpas {
const FieldInfo kFields[X_COUNT] = {
#define MPAS_FIELD(name, KIND, W, DIST, LO, HI) {#name, K_##KIND, W, D_##DIST, LO, HI},
#include "mpas_fields.def"
#undef MPAS_FIELD
    {"cosAngleEdge", K_E2F, 1, D_M, 0, 0},
    {"cosLatEdge", K_E2F, 1, D_M, 0, 0},
    {"cosLatCell", K_C2F, 1, D_M, 0, 0},
    {"sinLatCell", K_C2F, 1, D_M, 0, 0},
    {"cosLonCell", K_C2F, 1, D_M, 0, 0},
    {"sinLonCell", K_C2F, 1, D_M, 0, 0},
    {"ce_c1", K_C2I, 10, D_M, 0, 0},
    {"ce_c2", K_C2I, 10, D_M, 0, 0},
    {"ce_dv", K_C2F, 10, D_M, 0, 0},
    {"ce_dc", K_C2F, 10, D_M, 0, 0},
    {"ve_dc", K_V2F, 3, D_M, 0, 0},
    {"ce_idc", K_C2F, 10, D_M, 0, 0},
    {"ce_msd2", K_C2F, 10, D_M, 0, 0},
    {"ce_msd4", K_C2F, 10, D_M, 0, 0},
    {"ce_oth", K_C2I, 10, D_M, 0, 0},
    {"ce_s1", K_C2I, 10, D_M, 0, 0},
    {"eB", K_E2I, 24, D_M, 0, 0},
    {"cR", K_C2I, CREC, D_M, 0, 0},
    {"cRs", K_C2I, CREC, D_M, 0, 0},
    {"wfl", K_C2F, 2, D_M, 0, 0},
    {"wc", K_C3, 1, D_M, 0, 0},
    {"F", K_E3, 1, D_M, 0, 0},
    {"Fw", K_E3, 1, D_M, 0, 0},
    {"dvA", K_C3, 1, D_M, 0, 0},
    {"dvB", K_C3, 1, D_M, 0, 0},
    {"rupB", K_E3, 1, D_M, 0, 0},
    {"eown", K_C2I, 1, D_M, 0, 0},
    {"eowner", K_E2I, 1, D_M, 0, 0},
    {"orph", K_E2I, 1, D_M, 0, 0},
    {"tme", K_E3, 1, D_M, 0, 0},
    {"smlS", K_C3, 1, D_M, 0, 0},
    {"Dd", K_C3, 1, D_M, 0, 0},
    {"Ah", K_E3, 8, D_M, 0, 0},
    {"Rp", K_C3V, 8, D_M, 0, 0},
    {"Rm", K_C3V, 8, D_M, 0, 0},
    {"su", K_C3V, 8, D_M, 0, 0},
};
// translation units with kernels, registered at load time (mpas_dev.h, bounds-checked build)
static std::vector<void* (*)()>& bounds_tus() {
    static std::vector<void* (*)()> v;
    return v;
}
int bounds_register_tu(void* (*symbol)()) {
    bounds_tus().push_back(symbol);
    return 0;
}
}  // namespace mpas

using namespace mpas;

struct TimedCall {
    int task;
    hipEvent_t e0, e1;
};

struct mpas_ctx {
    int device = 0;
    mpas_dims dims{};
    DevState S{};
    hipStream_t stream = nullptr;
    std::string err;
    int exact = 0;
    int transport = 0;  // option "transport": atm_srk3 runs the monotonic scalar transport (physics = 1)
    int self_on = 1;   // option "self": allow the SELF gathers when the mesh permits
    int self_ok = 0;   // k_prepare's verdict on the uploaded mesh
    int overlap = 1;   // option "overlap": halo exchanges beside interior compute
    // option "hfuse": independent neighbouring kernels share a launch (same values); 2 = on
    // where the grids do not fill the chip (hfuse_auto_cells), the case it pays in
    // (x1.2562: -3 %; x1.163842: +0.8 %, the pair runs at the lower occupancy of the two)
    int hfuse = 2;
    int fusesml = 1;    // option "fusesml": each stage's set_smlstep inside its first acoustic launch (with fusedamp)
    int smlsum = 1;     // option "smlsum": its slope-flux sum once per step (fast path, with fusesml)
    int fusedamp_halo = 1;  // option "fusedamp_halo": fusedamp / fusesml on decomposed meshes too
    int tmedge = 0;     // option "tmedge": theta_m edge sums from dyn_tend for the acoustic substeps (same values;
                        // measured slower at both sizes)
    int fusecopy = 1;   // option "fusecopy" (with fusesetup): setup's edge copies made by stage 0's dyn_tend
                        // edge kernel from the columns it loads anyway (same values)
    int fusesetup = 1;  // option "fusesetup": stage 0's setup, moist and vert_imp in one launch (same values)
    int vdyn = 1;      // option "vdyn": atm_srk3's stage 2 dyn_tend edge kernel stores solve_diagnostics' v
                       // (reference semantics, edgesOnEdge_ECP = edgesOnEdge; same values)
    int defer4 = 1;    // option "defer4": atm_srk3 applies rk_step 0's del4 of tend_u_euler (dyn_tend D) in the
                       // next stage's rk_step > 0 edge kernel (reference semantics; same values)
    int msml = 1;      // option "msml" (the MPAS dynamics): each stage's set_smlstep applied by dyn_tend's E to
                       // the tend_w it forms (no task reads tend_w in between)
    int mru = 1;       // option "mru" (the MPAS dynamics, fast path): the kernel forming a stage's final tend_u
                       // stores its first acoustic substep's ru_p / ruAvg (k_acoustic_ru FIRST skipped)
    int mdamp = 1;     // option "mdamp" (the MPAS forms): each divergence damping applied by the kernel that next
                       // reads ru_p -- the next substep's k_acoustic_ru, or the stage's recover edge kernel
    int ntu = 1;       // option "ntu" (with defer4): that rk_step 0 call's whole tend_u is dead (the next stage's
                       // edge kernel rewrites it, no task in between reads it): its edge kernel forms none of
                       // it and skips its gathers (k_dyn_B NTU; the same values of everything read later)
    int fusedamp = 1;  // option "fusedamp": atm_srk3 applies each divergence damping inside the next
                       // acoustic launch (reference semantics, undecomposed; same bits)
    void* raw[X_COUNT] = {};  // the allocations behind S.f (S.f[f] = raw[f] + stagger)
    bool timing = false;
    bool dirty = true;  // derived mesh arrays need k_prepare
    std::vector<std::string> task_names;
    std::vector<int64_t> task_calls;
    std::vector<double> task_ms;
    std::vector<TimedCall> pending;
    std::vector<hipEvent_t> event_pool;
    std::unique_ptr<Halo> halo;           // decomposed mesh only
    std::shared_ptr<LoopGroup> loopgrp;   // in-process loopback transport
    int* gid_dev[3] = {nullptr, nullptr, nullptr};
    void* sum_scratch = nullptr;  // summarize_timestep partials (allocated on first use)
    double* sum_out = nullptr;
    // option "graph": mpas_atm_srk3 captured once per (dt, schedule) as a HIP graph and
    // replayed (one hipGraphLaunch per step instead of ~60 kernel launches); invalidated
    // by any option change or mesh upload; not used while per-task timing is on or on a
    // decomposed context (the halo bookkeeping is host-side per launch)
    int graph_on = 1;
    // decomposed contexts (option "graph_halo"; RCCL and stub transports -- the loopback's
    // host barriers cannot be captured): the halo bookkeeping is host-side and evolves
    // identically every step from a given state at the step's start, so that state is part
    // of a captured step's key (stale0), and a replay sets the host state to the one the
    // captured step ended in (stale1).  A few steps are kept, one per start state seen twice
    // (a standalone task or an upload between steps gives a second one)
    struct GraphEntry {
        double dt = 0.0;
        int schedule = -1;
        std::vector<uint8_t> stale0, stale1;
        int64_t exch = 0, fields = 0;
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        uint64_t used = 0;
    };
    static constexpr size_t kGraphCache = 4;
    std::vector<GraphEntry> graphs;
    uint64_t graph_clock = 0;
    int64_t graph_captures = 0, graph_launches = 0;
    // 2 (default): the stub transport only; 1: RCCL too (its grouped send / recv captured --
    // exercised on a 1-rank communicator only, which moves nothing); 0: off.  A capture that
    // fails on a transport falls back to eager steps (graph_fallbacks)
    int graph_halo = 2;
    int64_t graph_fallbacks = 0;
    // option "keep_check" (tests): after every task, every keep tail is compared with its
    // field on the owned entities (mpas_dev.h keep tails); a mismatch fails the task
    int keep_check = 0;
    int* keep_flag = nullptr;
    // set when a transport refused a capture: eager steps from then on (the user's graph_halo
    // stays as set; a new halo plan or a graph_halo option change clears it)
    bool graph_refused = false;
    std::vector<std::vector<uint8_t>> seen_stale0;  // start states stepped eagerly once
    // option "trtile": the tiled transport (k_transport.hip) when the mesh allows it; the
    // tiles are rebuilt after a mesh upload or a change of the owned / interior cells.
    // Off by default: measured 2x slower than the three kernels
    int trtile = 0;
    int trt_cells = TRT_CELLS, trt_clo = 96;  // options "trtcells", "trtclo": tile size limits (speed only)
    int trt_ghosts = 0;  // option "trtile_ghosts": a decomposed mesh's ghosts close over
                         // advCellsForEdge(edgesOnCell) (decomp.Decomposition(tiled_transport))
    bool trt_dirty = true;
    TrTiles trt;
    // option "tredge" (default 0: measured slower): the transport's edge kernel
    // with scalars_old staged in LDS per group of consecutive edges (undecomposed contexts;
    // rebuilt with the tiles)
    int tredge = 0;
    // option "trsave" (default 1; atm_srk3 with the transport, undecomposed, the default transport
    // kernels): scalars_save's copy folded into the transport -- its edge and bounds kernels read the old
    // scalars from scalars itself (nothing writes scalars before the transport's update) and the bounds
    // kernel stores them to scalars_old
    int trsave = 1;
    TrEdgeGroups tre;
    // option "etile" (default 1): dyn_tend's cell kernel E over compact tiles of cells, the tile's
    // theta_m closure staged in LDS, each edge's advCells flux formed there (k_dyn_Et) -- the edge
    // kernel then forms no flux and the per-edge scratch X_F goes (reference semantics, LP = 64,
    // undecomposed; the same bits either way).  Options "etcells" / "etclo": tile size limits
    int etile = 0;
    int ett_cells = 8, ett_clo = 56;
    bool ett_dirty = true;
    TrTiles ett;
};

namespace {

void ett_ensure(mpas_ctx* c);

struct Fail {
    int code;
    std::string msg;
};

void hipcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Fail{MPAS_EHIP, std::string(what) + ": " + hipGetErrorString(e)};
}

int entity_count(const mpas_ctx* c, int kind) {
    switch (kind) {
        case K_C3: case K_C3V: case K_C2F: case K_C2I: case K_C3B: return c->dims.nCells;
        case K_E3: case K_E2F: case K_E2I: return c->dims.nEdges;
        case K_V3: case K_V2F: case K_V2I: return c->dims.nVertices;
        default: return 1;
    }
}
size_t elem_size(int kind) {
    if (kind == K_C2I || kind == K_E2I || kind == K_V2I) return 4;
    if (kind == K_C3B) return 1;
    return 8;
}
// bytes of one device array (entity rows include the zero slot)
size_t dev_bytes(const mpas_ctx* c, int f) {
    const FieldInfo& fi = kFields[f];
    const size_t LP = c->S.LP;
    size_t rows = (size_t)entity_count(c, fi.kind) + 1;
    switch (fi.kind) {
        // (width-1 fields: + the two keep tails of rows doubles each, mpas_dev.h keep_tail)
        case K_C3: case K_E3: case K_V3: return rows * fi.width * LP * 8 + (fi.width == 1 ? 2 * rows * 8 : 0);
        case K_C3V: return rows * fi.width * LP * 8;
        case K_C3B: return rows * LP;
        case K_ZV: return LP * 8;
        default: return rows * fi.width * elem_size(fi.kind);
    }
}
// Keep tails (mpas_dev.h): the fields a step kernel writes with the kept value of level L
// (kKeepL) or of level 0 (kKeep0) -- the slots the reference never writes there.  Their
// tails are set from the field after every write from outside the step kernels
// (keep_refresh); option "keep_check" compares them with the field after every task.
const int kKeepL[] = {
    // dyn_tend (A, D, E; B and C keep the reference's unwritten slots)
    F_kdiff, F_h_divergence, F_tend_rho, F_dpdz, F_v, F_ru_save, F_u_2, F_tend_u_euler, F_tend_u,
    F_tend_w_euler, F_tend_theta_euler, F_tend_rtheta_adv, F_w, F_rthdynten, F_tend_theta,
    // vert_imp
    F_coftz, F_cofwt, F_cofwr, F_cofwz, F_a_tri, F_b_tri, F_c_tri, F_alpha_tri, F_gamma_tri,
    // solve_diagnostics (its edge kernel)
    F_h_edge, F_ke_edge, F_rho_edge, F_pv_edge,
    // setup + moist
    F_cqu, F_rw_save, F_rtheta_p_save, F_rho_p_save, F_w_2, F_theta_m_2, F_rho_zz_2, F_rho_zz_old_split,
    F_theta_m_save, F_qtot, F_cqw,
    // acoustic
    F_rtheta_pp_old, F_rho_pp, F_rtheta_pp,
    // recover (the MPAS forms)
    F_rho_p, F_rho_zz, F_rtheta_p, F_theta_m, F_exner, F_pressure_p, F_rw, F_ru, F_u,
    // substep_finish
    F_wwAvg_split, F_ruAvg_split,
    // mpas_reconstruct_2d
    F_uReconstructX, F_uReconstructY, F_uReconstructZ, F_uReconstructZonal, F_uReconstructMeridional};
const int kKeep0[] = {F_cofwr, F_cofwz, F_a_tri, F_b_tri, F_c_tri, F_alpha_tri, F_cqw, F_rw};
int keep_kind(int f) { return kFields[f].kind == K_C3 ? 0 : kFields[f].kind == K_E3 ? 1 : 2; }  // KC / KE / KV

void keep_refresh_all(mpas_ctx* c) {
    for (int f : kKeepL) hipcheck(launch_keep_refresh(c->S, c->stream, f, keep_kind(f)), "keep_refresh");
    for (int f : kKeep0) hipcheck(launch_keep_refresh(c->S, c->stream, f, keep_kind(f)), "keep_refresh");
}
void keep_verify(mpas_ctx* c, const char* task) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipcheck(hipStreamIsCapturing(c->stream, &cs), "hipStreamIsCapturing");
    if (cs != hipStreamCaptureStatusNone) return;  // (a captured step is checked when it runs eagerly)
    if (!c->keep_flag) hipcheck(hipMalloc(&c->keep_flag, 8 * sizeof(int)), "hipMalloc");
    hipcheck(hipMemsetAsync(c->keep_flag, 0, 7 * sizeof(int), c->stream), "hipMemsetAsync");
    hipcheck(hipMemsetAsync(c->keep_flag + 7, 0x7f, sizeof(int), c->stream), "hipMemsetAsync");
    for (int f : kKeepL) hipcheck(launch_keep_check(c->S, c->stream, f, keep_kind(f), 0, c->keep_flag), "keep_check");
    for (int f : kKeep0) hipcheck(launch_keep_check(c->S, c->stream, f, keep_kind(f), 1, c->keep_flag), "keep_check");
    int fl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    hipcheck(hipMemcpyAsync(fl, c->keep_flag, sizeof(fl), hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync");
    hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    if (fl[0]) {
        double v[2];
        std::memcpy(v, fl + 2, sizeof v);
        throw Fail{MPAS_EINVAL, std::string(task) + ": keep tail of " + kFields[(fl[0] - 1) / 2].name + " (level " +
                                    ((fl[0] - 1) % 2 ? "0" : "L") + ") differs from the field at entity " +
                                    std::to_string(fl[1]) + ": field " + std::to_string(v[0]) + ", tail " +
                                    std::to_string(v[1]) + "; " + std::to_string(fl[6]) +
                                    " mismatches, the first at entity " + std::to_string(fl[7]) + " (keep_check)"};
    }
}

// entity kind an integer field refers to (for the Q1 clamp), -1 if it is not an id
int id_target(int f) {
    switch (f) {
        case F_edgesOnCell: case F_edgesOnEdge: case F_edgesOnEdge_ECP: case F_edgesOnVertex: return K_E3;
        case F_cellsOnEdge: case F_advCellsForEdge: case F_cellsOnCell: case F_cellsOnVertex: return K_C3;
        case F_verticesOnEdge: case F_verticesOnCell: return K_V3;
        default: return -1;
    }
}

// true when p is device memory (a device-resident view: Legion framebuffer instance,
// torch tensor); host, pinned-host and unregistered pointers are host views
bool is_device_ptr(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // unregistered host memory reports an error: clear it
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}
// bytes a strided view of n entities x W components x levels 0..Lv spans (non-negative strides)
size_t view_span(int n, int W, int Lv, int64_t se, int64_t sl, int64_t sc, size_t elem) {
    if (n <= 0) return 0;
    if (se < 0 || sl < 0 || sc < 0) throw Fail{MPAS_EINVAL, "device views need non-negative strides"};
    return (size_t)((int64_t)(n - 1) * se + (int64_t)Lv * sl + (int64_t)(W - 1) * sc) + elem;
}
bool is_3d(int kind) { return kind == K_C3 || kind == K_E3 || kind == K_V3 || kind == K_C3V || kind == K_C3B; }

// width of the id rows a count field gives the length of (0: not a count)
int count_width(int f) {
    switch (f) {
        case F_nEdgesOnCell: return 10;      // edgesOnCell, verticesOnCell, cellsOnCell, edgesOnCell_sign, ...
        case F_nEdgesOnEdge: return 20;      // edgesOnEdge, weightsOnEdge
        case F_nAdvCellsForEdge: return 15;  // advCellsForEdge, adv_coefs(_3rd)
        default: return 0;
    }
}

int task_index(mpas_ctx* c, const char* name) {
    for (size_t i = 0; i < c->task_names.size(); i++)
        if (c->task_names[i] == name) return (int)i;
    c->task_names.push_back(name);
    c->task_calls.push_back(0);
    c->task_ms.push_back(0.0);
    return (int)c->task_names.size() - 1;
}

hipEvent_t get_event(mpas_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipcheck(hipEventCreate(&e), "hipEventCreate");
    return e;
}

void harvest(mpas_ctx* c) {
    for (auto& t : c->pending) {
        hipcheck(hipEventSynchronize(t.e1), "hipEventSynchronize");
        float ms = 0.f;
        hipcheck(hipEventElapsedTime(&ms, t.e0, t.e1), "hipEventElapsedTime");
        c->task_calls[t.task] += 1;
        c->task_ms[t.task] += ms;
        c->event_pool.push_back(t.e0);
        c->event_pool.push_back(t.e1);
    }
    c->pending.clear();
}

// run a task launcher, bracketed by events when timing is on
// roctx ranges per task (SURVEY §5 tracing): env MPAS_ROCTX=1 loads libroctx64 at the
// first task and brackets every task launch, so rocprofv3 --marker-trace shows the
// Regent task names over their kernels.  Off: no library, no cost.
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    Roctx() {
        const char* v = std::getenv("MPAS_ROCTX");
        if (!v || !*v || *v == '0') return;
        void* h = dlopen("libroctx64.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
        pop = (int (*)())dlsym(h, "roctxRangePop");
        if (!push || !pop) push = nullptr, pop = nullptr;
    }
};
const Roctx& roctx() {
    static Roctx r;
    return r;
}

template <class Fn>
void run_task(mpas_ctx* c, const char* name, Fn&& fn) {
    const Roctx& rx = roctx();
    if (rx.push) rx.push(name);
    struct Pop {
        const Roctx& r;
        ~Pop() {
            if (r.pop) r.pop();
        }
    } pop_at_exit{rx};
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int ti = -1;
    if (c->timing) {
        ti = task_index(c, name);
        e0 = get_event(c);
        e1 = get_event(c);
        hipcheck(hipEventRecord(e0, c->stream), "hipEventRecord");
    }
    if (c->dirty) {
        hipcheck(launch_prepare(c->S, c->stream), "prepare");
        c->self_ok = c->S.selfc;
        c->S.selfc = c->self_ok && c->self_on;
        c->dirty = false;
    }
    ett_ensure(c);  // (built before a capture by prepare_now)
    hipError_t e = fn();
    if (e != hipSuccess) {
        if (c->halo && !c->halo->err.empty())
            throw Fail{MPAS_ERCCL, std::string(name) + ": halo exchange: " + c->halo->err};
        throw Fail{MPAS_EHIP, std::string(name) + ": " + hipGetErrorString(e)};
    }
    if (c->halo && !c->halo->race.empty()) throw Fail{MPAS_EINVAL, std::string(name) + ": " + c->halo->race};
    if (c->keep_check) keep_verify(c, name);
    if (c->timing) {
        hipcheck(hipEventRecord(e1, c->stream), "hipEventRecord");
        c->pending.push_back({ti, e0, e1});
        if (c->pending.size() > 4096) harvest(c);
    }
}

// ---- bounds-checked build (mpas_dev.h MPAS_BOUNDS): the field table the kernels check
// against, and the check after every C-ABI call (which then synchronises the context)
#if MPAS_BOUNDS
struct BoundsReg {
    std::mutex mu;
    std::map<unsigned long long, std::pair<unsigned long long, std::string>> fields;  // lo -> (hi, name)
    BoundsTab* dev = nullptr;
};
BoundsReg& bounds_reg() {
    static BoundsReg r;
    return r;
}
// upload the sorted field ranges (every live context) and point each unit's table at them
void bounds_publish() {
    BoundsReg& r = bounds_reg();
    std::lock_guard<std::mutex> lk(r.mu);
    if (r.fields.size() > (size_t)kBoundsMax) throw Fail{MPAS_ENOMEM, "bounds table full"};
    hipcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
    if (!r.dev) {
        hipcheck(hipMalloc(&r.dev, sizeof(BoundsTab)), "hipMalloc");
        hipcheck(hipMemset(r.dev, 0, sizeof(BoundsTab)), "hipMemset");
        for (auto sym : bounds_tus()) {
            void* p = sym();
            if (!p) throw Fail{MPAS_EHIP, "bounds table symbol not found"};
            hipcheck(hipMemcpy(p, &r.dev, sizeof(r.dev), hipMemcpyHostToDevice), "hipMemcpy bounds");
        }
    }
    std::vector<unsigned long long> lo, hi;
    for (auto& kv : r.fields) lo.push_back(kv.first), hi.push_back(kv.second.first);
    const int n = (int)lo.size();
    if (n) {
        hipcheck(hipMemcpy(r.dev->lo, lo.data(), n * sizeof(lo[0]), hipMemcpyHostToDevice), "hipMemcpy bounds");
        hipcheck(hipMemcpy(r.dev->hi, hi.data(), n * sizeof(hi[0]), hipMemcpyHostToDevice), "hipMemcpy bounds");
    }
    hipcheck(hipMemcpy(&r.dev->n, &n, sizeof(n), hipMemcpyHostToDevice), "hipMemcpy bounds");
}
void bounds_add(mpas_ctx* c) {
    {
        BoundsReg& r = bounds_reg();
        std::lock_guard<std::mutex> lk(r.mu);
        for (int f = 0; f < X_COUNT; f++) {
            const unsigned long long lo = (unsigned long long)c->S.f[f];
            // (the columns only: the keep tails behind them are reached by keepv / keep_put alone)
            const FieldInfo& fi = kFields[f];
            const bool tails = (fi.kind == K_C3 || fi.kind == K_E3 || fi.kind == K_V3) && fi.width == 1;
            const size_t cols = dev_bytes(c, f) - (tails ? 2 * ((size_t)entity_count(c, fi.kind) + 1) * 8 : 0);
            r.fields[lo] = {lo + cols, kFields[f].name};
        }
    }
    bounds_publish();
}
void bounds_remove(mpas_ctx* c) {
    {
        BoundsReg& r = bounds_reg();
        std::lock_guard<std::mutex> lk(r.mu);
        for (int f = 0; f < X_COUNT; f++)
            if (c->S.f[f]) r.fields.erase((unsigned long long)c->S.f[f]);
    }
    try {
        bounds_publish();
    } catch (const Fail&) {
    }
}
// translation units whose table pointer is set (read back from each unit's symbol)
int bounds_units() {
    BoundsReg& r = bounds_reg();
    int n = 0;
    for (auto sym : bounds_tus()) {
        void* p = sym();
        BoundsTab* t = nullptr;
        if (p && hipMemcpy(&t, p, sizeof(t), hipMemcpyDeviceToHost) == hipSuccess && t && t == r.dev) n++;
    }
    return n;
}
void bounds_check(mpas_ctx* c) {
    BoundsReg& r = bounds_reg();
    if (!r.dev || !c->stream) return;
    hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    unsigned int count = 0;
    hipcheck(hipMemcpy(&count, &r.dev->count, sizeof(count), hipMemcpyDeviceToHost), "hipMemcpy bounds");
    if (!count) return;
    unsigned long long addr = 0, flo = 0, where = 0;
    hipcheck(hipMemcpy(&addr, &r.dev->addr, sizeof(addr), hipMemcpyDeviceToHost), "hipMemcpy bounds");
    hipcheck(hipMemcpy(&flo, &r.dev->field_lo, sizeof(flo), hipMemcpyDeviceToHost), "hipMemcpy bounds");
    hipcheck(hipMemcpy(&where, &r.dev->where, sizeof(where), hipMemcpyDeviceToHost), "hipMemcpy bounds");
    const unsigned int zero = 0;
    hipcheck(hipMemcpy(&r.dev->count, &zero, sizeof(zero), hipMemcpyHostToDevice), "hipMemcpy bounds");
    std::string name = "?";
    unsigned long long fhi = 0;
    {
        std::lock_guard<std::mutex> lk(r.mu);
        auto it = r.fields.find(flo);
        if (it != r.fields.end()) name = it->second.second, fhi = it->second.first;
    }
    char msg[256];
    snprintf(msg, sizeof msg, "%u access(es) outside their field; first: field %s, byte %lld of %llu (block %llu thread %llu)",
             count, name.c_str(), (long long)(addr - flo), fhi - flo, where >> 32, where & 0xffffffffull);
    throw Fail{MPAS_EBOUNDS, msg};
}
#else
void bounds_add(mpas_ctx*) {}
void bounds_remove(mpas_ctx*) {}
void bounds_check(mpas_ctx*) {}
#endif

template <class Fn>
int guarded(mpas_ctx* c, Fn&& fn) {
    if (!c) return MPAS_EINVAL;
    try {
        fn();
        if (MPAS_BOUNDS) bounds_check(c);
        return MPAS_OK;
    } catch (const Fail& f) {
        c->err = f.msg;
        return f.code;
    } catch (const std::bad_alloc&) {
        c->err = "out of host memory";
        return MPAS_ENOMEM;
    } catch (const std::exception& ex) {
        c->err = ex.what();
        return MPAS_EINVAL;
    } catch (...) {
        c->err = "unknown error";
        return MPAS_EINVAL;
    }
}

// ---- tiled transport: the cell tiles (TrTiles, mpas_dev.h) ----
void tiles_free(TrTiles& T);
void trt_free(mpas_ctx* c) {
    tiles_free(c->trt);
    c->S.trt = nullptr;
}
template <class V>
V* dev_copy(const std::vector<V>& h) {
    V* d = nullptr;
    hipcheck(hipMalloc(&d, sizeof(V) * (h.empty() ? 1 : h.size())), "hipMalloc");
    if (!h.empty()) hipcheck(hipMemcpy(d, h.data(), sizeof(V) * h.size(), hipMemcpyHostToDevice), "hipMemcpy H2D");
    return d;
}
template <class V>
std::vector<V> dev_read(const void* d, size_t n) {
    std::vector<V> h(n);
    hipcheck(hipMemcpy(h.data(), d, sizeof(V) * n, hipMemcpyDeviceToHost), "hipMemcpy D2H");
    return h;
}

// Compact tiles of at most TRT_CELLS owned cells, grown breadth-first over the cells'
// edge neighbours from the lowest unassigned cell id, within one launch class of a
// decomposed mesh (below), and closed
// before the closure -- the cells whose scalars_old the tile's kernels read, as the ids
// on the device resolve -- would exceed trt_clo LDS columns (default 96: 48 KB at LP = 64,
// three blocks per CU).  Not built (the three-kernel path runs) when an owned cell has more
// than NF edges or one of its edges more than AF advCells.
// The edge groups of k_tr_edge_lds (TrEdgeGroups, mpas_dev.h): TRE_GE consecutive owned
// edges per group; LDS columns in first-use order over the group's edges (advCells, then
// the two cells of the edge).
void tre_free(mpas_ctx* c) {
    TrEdgeGroups& G = c->tre;
    for (void* p : {(void*)G.ucell, (void*)G.ucnt, (void*)G.eslot})
        if (p) (void)hipFree(p);
    G = TrEdgeGroups{};
    c->S.tre = nullptr;
}
void tre_build(mpas_ctx* c) {
    tre_free(c);
    if (!c->tredge || c->halo || c->S.LP != 64) return;
    const DevState& S = c->S;
    const int nE = S.nEdges, nEO = S.nEO;
    if (nEO <= 0) return;
    const auto coe = dev_read<int>(S.f[F_cellsOnEdge], ((size_t)nE + 1) * 2);
    const auto adv = dev_read<int>(S.f[F_advCellsForEdge], ((size_t)nE + 1) * 15);
    const auto nadv = dev_read<int>(S.f[F_nAdvCellsForEdge], (size_t)nE + 1);
    const int ng = (nEO + TRE_GE - 1) / TRE_GE;
    std::vector<int> ucell((size_t)ng * TRE_U, 0), ucnt(ng, 0);
    std::vector<unsigned char> eslot((size_t)nEO * TRE_ROW, 0);
    int nirr = 0;
    for (int g = 0; g < ng; g++) {
        std::vector<int> u;
        bool ok = true;
        auto slot_of = [&](int cell) {
            for (size_t i = 0; i < u.size(); i++)
                if (u[i] == cell) return (int)i;
            u.push_back(cell);
            return (int)u.size() - 1;
        };
        for (int e = g * TRE_GE; e < std::min(nEO, (g + 1) * TRE_GE) && ok; e++) {
            const int na = nadv[e];
            if (na > AF) ok = false;
            unsigned char* r = &eslot[(size_t)e * TRE_ROW];
            for (int j = 0; j < AF && ok; j++) r[j] = (unsigned char)slot_of(adv[(size_t)e * 15 + j]);
            r[AF] = (unsigned char)slot_of(coe[(size_t)e * 2]);
            r[AF + 1] = (unsigned char)slot_of(coe[(size_t)e * 2 + 1]);
            if ((int)u.size() > TRE_U) ok = false;
        }
        if (!ok) {
            ucnt[g] = -1;
            nirr++;
            continue;
        }
        ucnt[g] = (int)u.size();
        for (int i = 0; i < TRE_U; i++) ucell[(size_t)g * TRE_U + i] = i < (int)u.size() ? u[i] : u[0];
    }
    TrEdgeGroups& G = c->tre;
    G.ngroups = ng;
    G.neo = nEO;
    G.nirr = nirr;
    G.ucell = dev_copy(ucell);
    G.ucnt = dev_copy(ucnt);
    std::vector<unsigned> packed(eslot.size() / 4);
    std::memcpy(packed.data(), eslot.data(), eslot.size());
    G.eslot = dev_copy(packed);
    c->S.tre = &c->tre;
}

void tiles_free(TrTiles& T) {
    for (void* p : {(void*)T.tptr, (void*)T.tcell, (void*)T.cptr, (void*)T.ccell, (void*)T.slot, (void*)T.teptr,
                    (void*)T.tedge, (void*)T.erow, (void*)T.terec})
        if (p) (void)hipFree(p);
    T = TrTiles{};
}
// the tiles (into T) of at most `cells` owned cells whose closure fits `clo_max` LDS columns;
// false (T empty) when the mesh does not allow them
bool tiles_build(mpas_ctx* c, TrTiles& T, int max_cells, int clo_max, int te_max = 1 << 30);

void trt_build(mpas_ctx* c) {
    trt_free(c);
    tre_free(c);
    c->trt_dirty = false;
    tre_build(c);
    if (!c->trtile) return;
    if (c->halo && !c->trt_ghosts) return;  // the tiles would read ghosts the local mesh lacks
    if (tiles_build(c, c->trt, c->trt_cells, c->trt_clo)) c->S.trt = &c->trt;
}

// option "etile": dyn_tend's cell kernel E over tiles of cells with the tile's theta_m closure
// in LDS (k_dyn_Et, k_dyn.hip); reference semantics, LP = 64, undecomposed
void ett_free(mpas_ctx* c) {
    tiles_free(c->ett);
    c->S.ett = nullptr;
}
void ett_build(mpas_ctx* c) {
    ett_free(c);
    c->ett_dirty = false;
    if (!c->etile || c->halo || c->S.LP != 64 || c->S.physics == 2) return;
    // (at most 96 edges per tile: the LDS of a block, (closure + 1 + edges) columns, stays < 160 KiB)
    if (tiles_build(c, c->ett, c->ett_cells, c->ett_clo, 96)) c->S.ett = &c->ett;
}
void ett_ensure(mpas_ctx* c) {
    if (c->ett_dirty) ett_build(c);
}

bool tiles_build(mpas_ctx* c, TrTiles& T, int max_cells, int clo_max, int te_max) {
    hipcheck(hipSetDevice(c->device), "hipSetDevice");
    const DevState& S = c->S;
    const int nC = S.nCells, nE = S.nEdges, nCO = S.nCO;
    const int nint = (c->halo && c->halo->interior) ? c->halo->nint[0] : nCO;
    const auto nEoC = dev_read<int>(S.f[F_nEdgesOnCell], (size_t)nC + 1);
    const auto eoc = dev_read<int>(S.f[F_edgesOnCell], ((size_t)nC + 1) * 10);
    const auto coe = dev_read<int>(S.f[F_cellsOnEdge], ((size_t)nE + 1) * 2);
    const auto adv = dev_read<int>(S.f[F_advCellsForEdge], ((size_t)nE + 1) * 15);
    const auto nadv = dev_read<int>(S.f[F_nAdvCellsForEdge], (size_t)nE + 1);
    auto nedges = [&](int x) { return nEoC[x] > 0 ? nEoC[x] : 0; };
    for (int x = 0; x < nCO; x++) {
        if (nEoC[x] > NF) return false;
        for (int i = 0; i < nedges(x); i++)
            if (nadv[eoc[(size_t)x * 10 + i]] > AF) return false;
    }
    // the columns cell x's kernels read: x, both cells of each edge, the edge's advCells
    auto need = [&](int x, auto&& f) {
        f(x);
        for (int i = 0; i < nedges(x); i++) {
            const size_t e = (size_t)eoc[(size_t)x * 10 + i];
            f(coe[e * 2]);
            f(coe[e * 2 + 1]);
            for (int j = 0; j < nadv[e]; j++) f(adv[e * 15 + j]);
        }
    };
    std::vector<int> mark((size_t)nC + 1, -1), seen((size_t)nC + 1, -1), inq((size_t)nC + 1, -1);
    std::vector<char> assigned((size_t)nC + 1, 0);
    std::vector<int> tptr{0}, tcell, cptr{0}, ccell, queue, cells, clo;
    std::vector<int> slot;
    int stamp = 0, maxclo = 0, nt_int = 0;
    std::vector<int> emark((size_t)nE + 1, -1), tmark((size_t)nE + 1, -1), tedge, teptr{0};
    std::vector<unsigned> erow, terec;
    int tebase = 0, maxte = 0;
    // launch classes: 0 = interior cells whose every column is owned (or the zero slot),
    // run beside a halo exchange; 1 = the rest (boundary cells, and interior cells that
    // reach a ghost through advCellsForEdge(edgesOnCell), which the halo's interior
    // classification does not follow), run after it
    std::vector<char> cls_of((size_t)nC + 1, 1);
    for (int x = 0; x < nint; x++) {
        bool own = true;
        need(x, [&](int y) { own = own && (y < nCO || y == nC); });
        cls_of[x] = own ? 0 : 1;
    }
    for (int cls = 0; cls < 2; cls++) {
        const int lo = 0, hi = nCO;
        for (int seed = lo; seed < hi; seed++) {
            if (assigned[seed] || cls_of[seed] != cls) continue;
            const int tid = (int)tptr.size();
            cells.clear();
            clo.clear();
            queue.assign(1, seed);
            inq[seed] = tid;
            int nte = 0;  // the tile's edges so far (tmark: the tile id of an edge's last use)
            for (size_t qh = 0; qh < queue.size() && (int)cells.size() < max_cells; qh++) {
                const int x = queue[qh];
                int add = 0, adde = 0;
                stamp++;
                need(x, [&](int y) {
                    if (mark[y] < 0 && seen[y] != stamp) seen[y] = stamp, add++;
                });
                for (int i = 0; i < nedges(x); i++) adde += tmark[eoc[(size_t)x * 10 + i]] != tid;
                if (!cells.empty() && ((int)clo.size() + add > clo_max || nte + adde > te_max)) continue;
                for (int i = 0; i < nedges(x); i++) {
                    const int e = eoc[(size_t)x * 10 + i];
                    if (tmark[e] != tid) tmark[e] = tid, nte++;
                }
                cells.push_back(x);
                assigned[x] = 1;
                need(x, [&](int y) {
                    if (mark[y] < 0) mark[y] = (int)clo.size(), clo.push_back(y);
                });
                for (int i = 0; i < nedges(x); i++) {
                    const size_t e = (size_t)eoc[(size_t)x * 10 + i];
                    for (int side = 0; side < 2; side++) {
                        const int y = coe[e * 2 + side];
                        if (y >= lo && y < hi && cls_of[y] == cls && !assigned[y] && inq[y] != tid)
                            inq[y] = tid, queue.push_back(y);
                    }
                }
            }
            for (int x : cells) {  // the tile's edges (first use) and each cell's record of them (ETT_REC)
                unsigned char r[ETT_REC] = {};
                const int zero = (int)clo.size();  // (the zero column after the closure's)
                for (int i = 0; i < NF; i++) {
                    unsigned char* ri = r + i * ETT_EB;
                    for (int j = 0; j < AF; j++) ri[1 + j] = (unsigned char)zero;
                    if (i >= nedges(x)) continue;
                    const int e = eoc[(size_t)x * 10 + i];
                    if (emark[e] < 0) {
                        emark[e] = (int)tedge.size() - tebase;
                        tedge.push_back(e);
                        unsigned char er[ETT_ER] = {};  // the edge's advCells' closure columns (zero column past nAdv)
                        for (int j = 0; j < AF; j++) er[j] = (unsigned char)(j < nadv[e] ? mark[adv[(size_t)e * 15 + j]] : zero);
                        const unsigned* ew = (const unsigned*)er;
                        terec.insert(terec.end(), ew, ew + ETT_ER / 4);
                    }
                    ri[0] = (unsigned char)emark[e];
                    for (int j = 0; j < nadv[e]; j++) ri[1 + j] = (unsigned char)mark[adv[(size_t)e * 15 + j]];
                }
                const unsigned* rw = (const unsigned*)r;
                erow.insert(erow.end(), rw, rw + ETT_REC / 4);
            }
            for (int x : cells) {  // the LDS rows
                int row[TRT_ROW] = {};
                row[0] = mark[x];
                for (int i = 0; i < nedges(x); i++) {
                    const size_t e = (size_t)eoc[(size_t)x * 10 + i];
                    int* ri = row + 1 + i * (2 + AF);
                    ri[0] = mark[coe[e * 2]];
                    ri[1] = mark[coe[e * 2 + 1]];
                    for (int j = 0; j < nadv[e]; j++) ri[2 + j] = mark[adv[e * 15 + j]];
                }
                slot.insert(slot.end(), row, row + TRT_ROW);
                tcell.push_back(x);
            }
            for (int y : clo) mark[y] = -1, ccell.push_back(y);
            for (size_t q = tebase; q < tedge.size(); q++) emark[tedge[q]] = -1;
            maxte = std::max(maxte, (int)tedge.size() - tebase);
            tebase = (int)tedge.size();
            teptr.push_back(tebase);
            maxclo = std::max(maxclo, (int)clo.size());
            tptr.push_back((int)tcell.size());
            cptr.push_back((int)ccell.size());
        }
        if (cls == 0) nt_int = (int)tptr.size() - 1;
    }
    T.ntiles = (int)tptr.size() - 1;
    T.nt_int = nt_int;
    T.nco = nCO;
    T.nint = nint;
    T.maxclo = maxclo;
    T.tptr = dev_copy(tptr);
    T.tcell = dev_copy(tcell);
    T.cptr = dev_copy(cptr);
    T.ccell = dev_copy(ccell);
    T.slot = dev_copy(slot);
    T.nclo = (int)ccell.size();
    T.teptr = dev_copy(teptr);
    T.tedge = dev_copy(tedge);
    T.erow = dev_copy(erow);
    T.terec = dev_copy(terec);
    T.maxte = maxte;
    return true;
}
void trt_ensure(mpas_ctx* c) {
    if (c->trt_dirty) trt_build(c);
}

// option hfuse (reference semantics, undecomposed); 2: only below this many owned cells
// (a cell kernel then has fewer than ~16 wavefronts per SIMD: the launches do not fill the
// chip and their fixed cost dominates)
constexpr int hfuse_auto_cells = 16384;
bool hfuse_active(const mpas_ctx* c) {
    if (c->S.physics != 0 || c->halo) return false;
    return c->hfuse == 1 || (c->hfuse == 2 && c->S.nCO < hfuse_auto_cells);
}

// timing keys: one Regent task, split where its read/write set (B_alg) differs by argument
// (bench.py aggregates the variants per task)
// (nold: a fused launch that does not store rtheta_pp_old -- every one but the step's last --
// tagged "-old" so that bench.py credits it no rtheta_pp_old write)
// (sml 2: set_smlstep from the step's flux sum X_smlS, "+smlS")
const char* acoustic_name(int small_step, bool damp = false, int sml = 0, bool nold = false) {
    if (sml == 2)
        return damp ? (nold ? "atm_advance_acoustic_step_work[ss0+smlS+damp-old]" : "atm_advance_acoustic_step_work[ss0+smlS+damp]")
                    : (nold ? "atm_advance_acoustic_step_work[ss0+smlS-old]" : "atm_advance_acoustic_step_work[ss0+smlS]");
    if (sml)  // (option fusesml: the stage's set_smlstep run by this launch first)
        return damp ? (nold ? "atm_advance_acoustic_step_work[ss0+sml+damp-old]" : "atm_advance_acoustic_step_work[ss0+sml+damp]")
                    : (nold ? "atm_advance_acoustic_step_work[ss0+sml-old]" : "atm_advance_acoustic_step_work[ss0+sml]");
    if (damp)  // (option fusedamp: the previous substep's damping applied by this launch)
        return small_step == 0
                   ? (nold ? "atm_advance_acoustic_step_work[ss0+damp-old]" : "atm_advance_acoustic_step_work[ss0+damp]")
                   : (nold ? "atm_advance_acoustic_step_work[ss>0+damp-old]" : "atm_advance_acoustic_step_work[ss>0+damp]");
    if (nold) return small_step == 0 ? "atm_advance_acoustic_step_work[ss0-old]" : "atm_advance_acoustic_step_work[ss>0-old]";
    return small_step == 0 ? "atm_advance_acoustic_step_work[ss0]" : "atm_advance_acoustic_step_work[ss>0]";
}

// the buffer pairs of the deferred damping (k_acoustic MODE 2), swapped by atm_srk3 after
// each launch; restored on exit (the ru_p pair by a copy if a step ended on the second
// buffer, which the reference schedule's even number of fused launches never does)
struct FuseBuffers {
    mpas_ctx* c;
    void *rup, *rupB, *dvA, *dvB;
    explicit FuseBuffers(mpas_ctx* c_) : c(c_) {
        rup = c->S.f[F_ru_p];
        rupB = c->S.f[X_rupB];
        dvA = c->S.f[X_dvA];
        dvB = c->S.f[X_dvB];
    }
    // (a decomposed context's halo keeps the ghost state of each buffer: it moves with it)
    void swap_rup() {
        std::swap(c->S.f[F_ru_p], c->S.f[X_rupB]);
        if (c->halo) std::swap(c->halo->stale[F_ru_p], c->halo->stale[X_rupB]);
    }
    void swap_dv() {
        std::swap(c->S.f[X_dvA], c->S.f[X_dvB]);
        if (c->halo) std::swap(c->halo->stale[X_dvA], c->halo->stale[X_dvB]);
    }
    void finish() {
        if (c->S.f[F_ru_p] != rup)
            hipcheck(hipMemcpyAsync(rup, c->S.f[F_ru_p], dev_bytes(c, F_ru_p), hipMemcpyDeviceToDevice, c->stream),
                     "hipMemcpyAsync ru_p");
        restore();
    }
    void restore() {
        const bool moved = c->S.f[X_rupB] != rupB || c->S.f[X_dvA] != dvA;
        c->S.f[F_ru_p] = rup;
        c->S.f[X_rupB] = rupB;
        c->S.f[X_dvA] = dvA;
        c->S.f[X_dvB] = dvB;
        // (ru_p's state moved with its data, which finish() copied back; the scratch
        // buffers hold anything)
        if (c->halo && moved) c->halo->stale[X_rupB] = c->halo->stale[X_dvA] = c->halo->stale[X_dvB] = 1;
    }
    ~FuseBuffers() { restore(); }
};
const char* recover_name(int rk_step) {
    return rk_step == 2 ? "atm_recover_large_step_variables_work[rk2]" : "atm_recover_large_step_variables_work[rk<2]";
}

void srk3(mpas_ctx* c, double dt, int schedule) {
    // rk_timestep.rg:378-399
    const int number_of_sub_steps = 2;
    const int dynamics_split = 1;  // constants.rg:62
    const double dt_dynamics = dt;
    const double rk_sub_timestep[3] = {dt_dynamics / 3, dt_dynamics / number_of_sub_steps,
                                       dt_dynamics / number_of_sub_steps};
    int number_sub_steps[3];
    number_sub_steps[0] = (number_of_sub_steps / 2 > 1) ? number_of_sub_steps / 2 : 1;
    number_sub_steps[1] = number_sub_steps[0];
    number_sub_steps[2] = number_of_sub_steps;
    const DevState& S = c->S;
    hipStream_t st = c->stream;
    // option trsave: the copy below folded into the transport's bounds kernel (its tables decided here:
    // the tiled and LDS-edge forms need none of them built, su stored)
    const bool trfold = c->transport && c->trsave && !c->halo && !c->trtile && !c->tredge && !S.trsu;
    if (c->transport && !trfold) {
        // the time level the transport starts from (MPAS-A scalars(time level 1)); the
        // copy carries the ghosts of scalars, fresh or not, so scalars_old is as stale
        run_task(c, "scalars_save", [&] {
            hipError_t e = hipMemcpyAsync(S.f[F_scalars_old], S.f[F_scalars], dev_bytes(c, F_scalars),
                                          hipMemcpyDeviceToDevice, st);
            if (S.halo && S.halo->stale[F_scalars]) S.halo->wrote({F_scalars_old});
            return e;
        });
    }
    // option fusecopy: ru_save / u_2 by stage 0's dyn_tend edge kernel (reads u and ru there;
    // no task between the setup and that kernel reads ru_save or u_2, in any physics mode)
    const bool fcopy = c->fusesetup && c->fusecopy;
    // option fusedamp (reference semantics): each damping but the step's last is applied by
    // the next acoustic launch (k_acoustic MODE 2), the last from the div the acoustic step
    // stored (launch_div_damping_div); the same bits as the separate task.  Decomposed (option
    // fusedamp_halo): the div is exchanged where rtheta_pp was, the ring-1 edges stay fresh
    const bool fuse = c->fusedamp && S.physics == 0 && (!c->halo || (c->fusedamp_halo && S.ring1 && S.nERing >= S.nEO));
    FuseBuffers fb(c);
    int n_acoustic = 0, done_acoustic = 0;
    for (int r = 0; r < 3; r++) n_acoustic += number_sub_steps[r] + (S.physics ? 0 : 1);
    bool pending = false;
    double coef_prev = 0.0;
    // option tmedge (reference semantics, undecomposed): dyn_tend's edge kernel stores
    // theta_m(cell2) + theta_m(cell1) per edge, which the stage's acoustic substeps and the
    // damping read instead of gathering theta_m at both cells (theta_m unchanged in between)
    const int tme = (c->tmedge && S.physics == 0 && !c->halo) ? 1 : 0;
    // option hfuse (reference semantics, undecomposed): neighbouring kernels that neither
    // read what the other writes share a launch (k_solve.hip combined launches, dyn_tend's
    // rk 0 D beside E); the same values
    const int hf = hfuse_active(c) ? 1 : 0;
    bool vi_done = false;  // stage 1's vert_imp ran beside stage 0's solve_diagnostics edges
    // hfuse with fusedamp (and the default epw, no tmedge): a stage's last acoustic launch
    // beside its solve_diagnostics vertex / cell kernel, and the stage's edge kernel beside
    // the next stage's dyn_tend A (k_acoustic.hip / k_dyn.hip combined launches)
    const bool hf2 = hf && fuse && !tme && S.epw == 2;
    bool vc_done = false, a_done = false, vdyn_on = false;
    // option smlsum (fast path, with fusesml): the slope-flux sum of set_smlstep formed once per
    // step (X_smlS); each stage's fused set_smlstep then reads one column instead of u_tend at
    // the cell's edges and zb_cell / zb3_cell (none of them written within the step)
    const bool smls = fuse && c->fusesml && c->smlsum && !c->exact && S.physics == 0;
    auto stage_args = [&](int r) {
        DynTendArgs a{};
        a.rk_step = schedule == 0 ? (int)rk_sub_timestep[r] : r;  // Q4
        a.dt = dt;
        a.horiz_mixing = 0;  // constants.rg:57 "2d_smagorinsky"
        a.cam_coef = 0.0;
        a.mix_full = 0;
        a.rayleigh_damp_u = 0;
        a.exact_q = c->exact;
        a.tme = tme;
        a.hfuse = hf;
        a.cp = (fcopy && r == 0) ? 1 : 0;
        // option defer4: an rk_step 0 stage followed by an rk_step > 0 one leaves its kernel D
        // (tend_u_euler's del4 part; its tend_u is dead: the next stage rewrites it and no task
        // in between reads it in the reference semantics) to the next stage's edge kernel
        auto rk_of = [&](int s) { return schedule == 0 ? (int)rk_sub_timestep[s] : s; };
        if (c->defer4 && S.physics == 0) {
            a.defer_out = (r < 2 && rk_of(r) == 0 && rk_of(r + 1) != 0) ? 1 : 0;
            a.defer_in = (r > 0 && rk_of(r - 1) == 0 && rk_of(r) != 0) ? 1 : 0;
            // (option ntu: the stages before the last read no tend_u_euler -- their edge kernels form no
            // tend_u -- so the deferred del4 goes to the last stage's edge kernel, the first that reads it;
            // its operands, delsq_divergence / delsq_vorticity / rho_edge, are unchanged until then)
            if (c->ntu) {
                const bool pending = (rk_of(0) == 0 && rk_of(1) != 0) || (rk_of(1) == 0 && rk_of(2) != 0);
                a.defer_in = (r == 2 && pending) ? 1 : 0;
            }
        }
        // option ntu (reference semantics): a stage before the step's last leaves dead tendencies -- the last
        // stage rewrites tend_u, tend_theta, tend_rtheta_adv and rthdynten, and no task in between reads them
        // (set_smlstep reads u_tend, Q2; the acoustic step reads neither tend_u, Q18, nor tend_theta: theta_m
        // is its tend_rt, Q8): that dyn_tend forms none of them (tend_u only where its D, reading it, does not run)
        if (c->ntu && S.physics == 0 && r < 2) {
            a.nth = 1;
            a.ntu = 1;  // (launch_dyn_tend keeps it off where D runs in the call)
        }
        // option mru (the MPAS dynamics, fast path): the kernel that forms the stage's final tend_u also
        // stores the first acoustic substep's ru_p = dts tend_u and ruAvg = ru_p (nothing in between reads
        // or writes them; set_smlstep reads tend_u only)
        if (c->mru && S.physics == 2 && !c->exact && number_sub_steps[r] > 0) a.rud = rk_sub_timestep[r];
        // option msml (the MPAS dynamics): the stage's set_smlstep (:1503-1528) applied by E to the tend_w it
        // forms -- set_smlstep follows dyn_tend directly and reads tend_u, which B / D have finished
        if (c->msml && S.physics == 2) a.smlE = 1;
        return a;
    };
    bool flux_done = false;  // (option smlsum: the step's flux sum, beside setup and A on small grids)
    // option ntu: stage 0's solve_diagnostics is dead where stage 1 runs at rk_step > 0 (a stage before the last
    // reads nothing it writes; an rk_step 0 stage 1 would read divergence and vorticity)
    const int rk1 = schedule == 0 ? (int)rk_sub_timestep[1] : 1;
    const bool solve0_dead = c->ntu && S.physics == 0 && !hf && rk1 != 0;
    // option ntu (reference semantics): the substep finish's rho_zz = rho_zz_old_split is the identity --
    // this step's setup made rho_zz_old_split from rho_zz and nothing writes either in between -- not made
    const bool norz = (c->ntu == 1 || c->ntu == 2) && S.physics == 0 && S.LP == 64 && dynamics_split == 1;
    if (c->fusesetup && S.physics == 0 && hf2) {  // + stage 0's dyn_tend A in the same launch
        run_task(c, smls ? "hfuse[setup+dyn_A+sml_flux]" : "hfuse[setup+dyn_A]", [&] {
            return launch_hf_setup_dyn_A(S, st, stage_args(0), rk_sub_timestep[0], fcopy ? 0 : 1, smls ? 1 : 0);
        });
        a_done = true;
        flux_done = smls;
    } else if (c->fusesetup) {  // :404-417 as one column-local launch (same values; MPAS forms under physics)
        // (option ntu: stage 0's vert_imp leaves b_tri / c_tri unstored -- no task reads them and stage 1's
        // vert_imp, which always runs, rewrites both; "-bc")
        const bool nbc = c->ntu == 1 || c->ntu == 2;
        run_task(c, fcopy ? (nbc ? "atm_rk_integration_setup[cells+moist+vert_imp-bc]" : "atm_rk_integration_setup[cells+moist+vert_imp]")
                          : (nbc ? "atm_rk_integration_setup[+moist+vert_imp-bc]" : "atm_rk_integration_setup[+moist+vert_imp]"),
                 [&] { return launch_setup_moist_vert_imp(S, st, rk_sub_timestep[0], !fcopy, nbc ? 1 : 0); });
    } else {
        run_task(c, "atm_rk_integration_setup", [&] { return launch_rk_integration_setup(S, st); });
        run_task(c, "atm_compute_moist_coefficients", [&] { return launch_moist_coefficients(S, st); });
        run_task(c, "atm_compute_vert_imp_coefs", [&] { return launch_vert_imp_coefs(S, st, rk_sub_timestep[0]); });
    }
    if (smls && !flux_done)
        run_task(c, "atm_set_smlstep_pert_variables_work[flux]", [&] { return launch_sml_flux(S, st); });
    for (int rk_step = 0; rk_step < 3; rk_step++) {  // :426-477
        if (rk_step == 1 && !vi_done)
            run_task(c, "atm_compute_vert_imp_coefs", [&] { return launch_vert_imp_coefs(S, st, rk_sub_timestep[rk_step]); });
        DynTendArgs a = stage_args(rk_step);
        a.skipA = a_done ? 1 : 0;
        // option vdyn (reference semantics): the last stage's v (:429-437) is reconstructed by its
        // dyn_tend edge kernel from the edgesOnEdge u it gathers for q -- u is not written between
        // that kernel and the stage's solve_diagnostics, which then skips v
        if (rk_step == 2) vdyn_on = c->vdyn && S.physics == 0 && a.rk_step > 0 && S.eoe_same;
        a.store_v = (rk_step == 2 && vdyn_on) ? 1 : 0;
        a_done = false;
        // timing key: the variant's read / write set (bench.py parses the tags)
        const std::string dname = std::string("atm_compute_dyn_tend_work[") + (a.rk_step == 0 ? "rk0" : "rk>0") +
                                  (a.cp ? "+copy" : "") + (a.defer_out ? "+d4o" : "") + (a.ntu ? "+ntu" : "") + (a.defer_in ? "+d4i" : "") +
                                  (a.store_v ? "+v" : "") + (a.rud != 0.0 ? "+ru" : "") + (a.smlE ? "+sml" : "") +
                                  (a.skipA ? "-A" : "") + "]";
        run_task(c, dname.c_str(), [&] { return launch_dyn_tend(S, st, a); });
        const bool ru_done = a.rud != 0.0;  // (option mru: the first substep's ru_p / ruAvg stored)
        // option fusesml (with fusedamp): the stage's first acoustic launch runs it first
        const bool sml = fuse && c->fusesml;
        if (!sml && !a.smlE)  // (option msml: run by E)
            run_task(c, "atm_set_smlstep_pert_variables_work", [&] { return launch_set_smlstep(S, st, c->exact); });
        const int n_small = number_sub_steps[rk_step] + (S.physics ? 0 : 1);  // Q5 (the MPAS form: n)
        for (int small_step = 0; small_step < n_small; small_step++) {
            const double dts = rk_sub_timestep[rk_step];
            if (fuse) {
                const int mode = pending ? 2 : 1;
                const int sm = (sml && small_step == 0) ? (smls ? 2 : 1) : 0;
                // rtheta_pp_old is read by the separate damping only: the fused one reads the
                // stored div, so the step's last substep alone leaves it (option fusedamp)
                // option ntu (bit 1): a stage's last substep before the step's last stage leaves rho_pp,
                // rtheta_pp, rw_p and wwAvg unstored -- the next stage's first substep sets them before
                // any task reads them (:1615-1636), and the damping reads the stored div
                const int nst = (c->ntu == 1 || c->ntu == 2) && rk_step < 2 && small_step == n_small - 1 ? 2 : 0;
                const int wold = ((done_acoustic + 1 == n_acoustic) ? 1 : 0) | nst;
                if (hf2 && rk_step < 2 && mode == 2 && small_step > 0 && small_step == n_small - 1) {
                    run_task(c, nst ? "hfuse[acoustic-st+solve_vc]" : "hfuse[acoustic+solve_vc]", [&] {
                        return launch_hf_acoustic_solve_vc(S, st, dts, small_step, c->exact, coef_prev, wold, smls ? 1 : 0);
                    });
                    vc_done = true;
                } else {
                    // ("-st": option ntu's launch that stores no acoustic state, bench.py's accounting)
                    const std::string an = nst ? std::string(acoustic_name(small_step, pending, sm, !(wold & 1))).insert(
                                                     std::strlen(acoustic_name(small_step, pending, sm, !(wold & 1))) - 1, "-st")
                                               : std::string(acoustic_name(small_step, pending, sm, !(wold & 1)));
                    run_task(c, an.c_str(),
                             [&] { return launch_acoustic(S, st, dts, small_step, c->exact, mode, coef_prev, tme, sm, wold,
                                                          smls ? 1 : 0); });
                }
                if (mode == 2) fb.swap_rup();
                fb.swap_dv();  // this substep's div is read next from X_dvB
                if (++done_acoustic == n_acoustic) {
                    if (hf)  // beside the solve_diagnostics vertex / cell kernel that follows
                        run_task(c, "hfuse[damp+solve_vc]", [&] { return launch_hf_damp_solve_vc(S, st, dts, tme); });
                    else
                        run_task(c, "atm_divergence_damping_3d", [&] { return launch_div_damping_div(S, st, dts, tme); });
                    pending = false;
                } else {
                    pending = true;
                    coef_prev = divdamp_coef(dts);
                }
                continue;
            }
            // option mdamp (the MPAS forms): the previous substep's damping in this substep's ru_p kernel, the
            // stage's last one in the recover edge kernel -- each read-modify-write of ru_p goes
            const bool md_fold = c->mdamp && S.physics;
            const int mdp = (md_fold && small_step > 0) ? (small_step == 1 ? 2 : 1) : 0;
            const double cprev = mdp ? divdamp_coef(dts) : 0.0;
            // (option ntu: the last substep of a stage before the last leaves wwAvg unstored -- its recover
            // does not read it (the averages are dead there) and the next stage's first substep sets it)
            const bool nww = S.physics && (c->ntu == 1 || c->ntu == 2) && rk_step < 2 && small_step == n_small - 1;
            const std::string an = std::string(mdp ? "atm_advance_acoustic_step_work[ss>0+damp]" : acoustic_name(small_step));
            const std::string an1 = nww ? an.substr(0, an.size() - 1) + "-ww]" : an;
            // ("-ru": option mru, this first substep's ru_p / ruAvg were stored by the stage's dyn_tend)
            const std::string anw = (small_step == 0 && ru_done) ? an1.substr(0, an1.size() - 1) + "-ru]" : an1;
            run_task(c, anw.c_str(), [&] {
                return launch_acoustic(S, st, dts, small_step, c->exact, 0, cprev, tme, 0, nww ? 3 : 1, 0, mdp,
                                       (small_step == 0 && ru_done) ? 1 : 0);
            });
            if (!md_fold)
                run_task(c, "atm_divergence_damping_3d", [&] { return launch_div_damping(S, st, dts, small_step == 0); });
        }
        if (S.physics) {  // rk_timestep.rg:460, commented out in the reference (Q7)
            // option ntu: a stage before the last leaves ruAvg / wwAvg dead -- the next stage's first
            // acoustic substep sets both before any task reads them
            const bool navg = (c->ntu == 1 || c->ntu == 2) && rk_step < 2;
            // (option mdamp: the stage's last damping in the edge kernel; 2: that substep was the stage's first)
            const int ns_r = number_sub_steps[rk_step];
            const int dmp = (c->mdamp && ns_r > 0) ? (ns_r == 1 ? 2 : 1) : 0;
            const std::string rn = std::string(navg ? (rk_step == 1 ? "atm_recover_large_step_variables_work[rk1-avg]"
                                                                   : "atm_recover_large_step_variables_work[rk<2-avg]")
                                                    : recover_name(rk_step));
            const std::string rnd = dmp ? rn.substr(0, rn.size() - 1) + "+damp]" : rn;
            run_task(c, rnd.c_str(), [&] {
                return launch_recover_large_step(S, st, ns_r, rk_step, dt, navg ? 1 : 0, dmp, rk_sub_timestep[rk_step]);
            });
        }
        if (hf && fuse && rk_step == 2 && S.LP == 64 && !c->transport) {
            // (the vertex / cell kernel ran beside the last damping) the edge kernel beside
            // atm_rk_dynamics_substep_finish, which follows below
            run_task(c, vdyn_on ? (norz ? "hfuse[solve_e-v+finish-rz]" : "hfuse[solve_e-v+finish]")
                                : (norz ? "hfuse[solve_e+finish-rz]" : "hfuse[solve_e+finish]"),
                     [&] { return launch_hf_solve_e_finish(S, st, vdyn_on ? 0 : 1, norz ? 1 : 0); });
        } else if (hf && fuse && rk_step == 2) {
            run_task(c, vdyn_on ? "atm_compute_solve_diagnostics[e-v]" : "atm_compute_solve_diagnostics[e]",
                     [&] { return launch_solve_diagnostics(S, st, 0, 2, 2, vdyn_on ? 1 : 0); });
        } else if (hf2 && vc_done && rk_step < 2) {
            // (the vertex / cell kernel ran beside the last acoustic launch) the edge kernel
            // beside the next stage's dyn_tend A, and after stage 0 beside stage 1's vert_imp
            const DynTendArgs nx = stage_args(rk_step + 1);
            run_task(c, rk_step == 0 ? "hfuse[solve_e+vert_imp+dyn_A]" : "hfuse[solve_e+dyn_A]", [&] {
                return launch_hf_solve_e_dyn_A(S, st, nx, rk_step == 0 ? 1 : 0, rk_sub_timestep[1]);
            });
            if (rk_step == 0) vi_done = true;
            a_done = true;
            vc_done = false;
        } else if (rk_step == 0 && solve0_dead) {
            // option ntu: stage 0's solve_diagnostics is dead -- stage 1's dyn_tend (a stage before the last:
            // no A, no tend_u) reads none of its outputs, no other task reads them, and stage 1's and 2's
            // solve_diagnostics rewrite every one (h_edge, ke_edge, pv_edge, divergence, ke, vorticity, pv_vertex)
        } else if (hf && rk_step == 0) {  // the edge kernel beside stage 1's vert_imp
            run_task(c, "atm_compute_solve_diagnostics[vc]", [&] { return launch_solve_diagnostics(S, st, 0, 0, 1); });
            run_task(c, "hfuse[solve_e+vert_imp]",
                     [&] { return launch_hf_solve_e_vert_imp(S, st, rk_sub_timestep[1]); });
            vi_done = true;
        } else {
            const int nv = (rk_step == 2 && vdyn_on) ? 1 : 0;
            // option ntu: a call before the last stage's, the next stage at rk_step > 0, stores only what
            // that stage reads -- ke and pv_edge (the MPAS forms: rho_edge too); its divergence, vorticity,
            // h_edge and ke_edge have no reader before the last stage's solve_diagnostics rewrites them
            // (dyn_tend reads divergence and vorticity at rk_step 0 only; nothing reads h_edge, ke_edge)
            const int rk_next = rk_step == 2 ? 0 : schedule == 0 ? (int)rk_sub_timestep[rk_step + 1] : rk_step + 1;
            // (ntu = 2: every diagnostic stored, 3: every acoustic state stored -- the A/Bs of these parts)
            const bool live = (c->ntu == 1 || c->ntu == 3) && rk_step < 2 && rk_next != 0;
            run_task(c, live ? "atm_compute_solve_diagnostics[live]"
                             : nv ? "atm_compute_solve_diagnostics[-v]" : "atm_compute_solve_diagnostics",
                     [&] { return launch_solve_diagnostics(S, st, 0, rk_step, live ? 7 : 3, nv); });
        }
    }
    if (c->transport)  // after the last stage's recover: ruAvg / wwAvg / rho_zz of the step
        run_task(c, trfold ? "atm_advance_scalars_mono[save]" : "atm_advance_scalars_mono", [&] {
            trt_ensure(c);  // (built before a capture by prepare_now)
            return launch_advance_scalars_mono(S, st, dt, trfold ? 1 : 0);
        });
    if (S.physics == 2)  // the MPAS dynamics: cell-centre winds for the next step's curvature
        run_task(c, "mpas_reconstruct_2d", [&] { return launch_reconstruct_2d(S, st, 1); });  // (:487, commented)
    if (!(hf && fuse && S.LP == 64 && !c->transport))  // (else it ran beside solve_diagnostics' edges)
        run_task(c, norz ? "atm_rk_dynamics_substep_finish[-rz]" : "atm_rk_dynamics_substep_finish",
                 [&] { return launch_substep_finish(S, st, 1, dynamics_split, norz ? 1 : 0); });
    fb.finish();
    // :492 summarize_timestep(cr, er, false, false, false) (constants.rg:67-69): prints only
}

void graph_free(mpas_ctx::GraphEntry& g) {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (g.graph) (void)hipGraphDestroy(g.graph);
    g.exec = nullptr;
    g.graph = nullptr;
}
void graph_drop(mpas_ctx* c) {
    for (auto& g : c->graphs) graph_free(g);
    c->graphs.clear();
    c->seen_stale0.clear();
}

void prepare_now(mpas_ctx* c) {
    if (c->dirty) {
        hipcheck(launch_prepare(c->S, c->stream), "prepare");
        c->self_ok = c->S.selfc;
        c->S.selfc = c->self_ok && c->self_on;
        c->dirty = false;
    }
    if (c->transport) trt_ensure(c);
    ett_ensure(c);
}

// one atm_srk3 step: replayed from a captured HIP graph when possible
void srk3_step(mpas_ctx* c, double dt, int schedule) {
    Halo* h = c->halo.get();
    const bool halo_graph = h && !h->loop && (h->stub ? c->graph_halo != 0 : (h->rccl && c->graph_halo == 1)) &&
                            !c->graph_refused;
    if (!c->graph_on || c->timing || (h && !halo_graph)) {
        srk3(c, dt, schedule);
        return;
    }
    prepare_now(c);  // (synchronous: never inside a capture)
    static const std::vector<uint8_t> none;
    const std::vector<uint8_t>& start = h ? h->stale : none;
    for (auto& g : c->graphs)
        if (g.dt == dt && g.schedule == schedule && g.stale0 == start) {
            hipcheck(hipGraphLaunch(g.exec, c->stream), "hipGraphLaunch");
            g.used = ++c->graph_clock;
            c->graph_launches++;
            if (h) {
                h->stale = g.stale1;  // the bookkeeping the captured step made
                h->exchanges += g.exch;
                h->fields_moved += g.fields;
            }
            return;
        }
    if (h && std::find(c->seen_stale0.begin(), c->seen_stale0.end(), h->stale) == c->seen_stale0.end()) {
        // a start state not seen before (e.g. the first step after an upload): one eager step
        if (c->seen_stale0.size() >= 16) c->seen_stale0.erase(c->seen_stale0.begin());
        c->seen_stale0.push_back(h->stale);
        srk3(c, dt, schedule);
        return;
    }
    mpas_ctx::GraphEntry g;
    g.dt = dt;
    g.schedule = schedule;
    g.stale0 = start;
    int64_t ex0 = 0, fl0 = 0;
    if (h) {
        ex0 = h->exchanges;
        fl0 = h->fields_moved;
        h->capture_miss = false;
    }
    hipcheck(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    try {
        srk3(c, dt, schedule);
    } catch (...) {
        hipGraph_t gr = nullptr;
        (void)hipStreamEndCapture(c->stream, &gr);
        if (gr) (void)hipGraphDestroy(gr);
        if (h) {  // nothing ran: the bookkeeping goes back to the step's start
            h->stale = g.stale0;
            h->exchanges = ex0;
            h->fields_moved = fl0;
            h->overlapped.clear();  // (the aborted step's overlap record and race flag too)
            h->race.clear();
            if (h->capture_miss) {  // a pack table not built yet (never built inside a capture)
                h->capture_miss = false;
                h->err.clear();
                srk3(c, dt, schedule);  // eagerly: builds it; the next step captures
                return;
            }
            // the transport refused the capture (a communicator that cannot be captured):
            // eager steps from now on, and the step again eagerly (a real error repeats there)
            (void)hipGetLastError();
            h->err.clear();
            c->graph_refused = true;
            c->graph_fallbacks++;
            srk3(c, dt, schedule);
            return;
        }
        throw;
    }
    {
        const hipError_t ee = hipStreamEndCapture(c->stream, &g.graph);
        hipError_t ei = ee;
        if (ee == hipSuccess) ei = hipGraphInstantiate(&g.exec, g.graph, nullptr, nullptr, 0);
        if (h && (ee != hipSuccess || ei != hipSuccess)) {  // (as above: nothing ran)
            graph_free(g);
            (void)hipGetLastError();
            h->stale = g.stale0;
            h->exchanges = ex0;
            h->fields_moved = fl0;
            h->overlapped.clear();
            h->race.clear();
            c->graph_refused = true;
            c->graph_fallbacks++;
            srk3(c, dt, schedule);
            return;
        }
        hipcheck(ee, "hipStreamEndCapture");
        hipcheck(ei, "hipGraphInstantiate");
    }
    c->graph_captures++;
    if (h) {
        g.stale1 = h->stale;
        g.exch = h->exchanges - ex0;
        g.fields = h->fields_moved - fl0;
    }
    g.used = ++c->graph_clock;
    if (c->graphs.size() >= mpas_ctx::kGraphCache) {  // the least recently replayed goes
        auto lru = std::min_element(c->graphs.begin(), c->graphs.end(),
                                    [](const mpas_ctx::GraphEntry& a, const mpas_ctx::GraphEntry& b) { return a.used < b.used; });
        graph_free(*lru);
        c->graphs.erase(lru);
    }
    c->graphs.push_back(g);
    hipcheck(hipGraphLaunch(g.exec, c->stream), "hipGraphLaunch");
    c->graph_launches++;
}

}  // namespace

extern "C" {

int mpas_field_count(void) { return F_COUNT; }
int mpas_field_id(const char* name) {
    if (!name) return MPAS_EINVAL;
    for (int f = 0; f < F_COUNT; f++)
        if (std::strcmp(kFields[f].name, name) == 0) return f;
    return MPAS_EINVAL;
}
const char* mpas_field_name(int f) { return (f >= 0 && f < F_COUNT) ? kFields[f].name : nullptr; }
int mpas_field_kind(int f) { return (f >= 0 && f < F_COUNT) ? kFields[f].kind : MPAS_EINVAL; }
int mpas_field_width(int f) { return (f >= 0 && f < F_COUNT) ? kFields[f].width : MPAS_EINVAL; }

static thread_local std::string g_create_err;

int mpas_ctx_create(mpas_ctx** out, int device, const mpas_dims* dims) {
    if (!out || !dims) return MPAS_EINVAL;
    *out = nullptr;
    if (dims->nCells <= 0 || dims->nEdges <= 0 || dims->nVertices <= 0 || dims->nVertLevels < 1 ||
        dims->nVertLevels + 1 > 64) {
        g_create_err = "mpas_ctx_create: need nCells, nEdges, nVertices > 0 and 1 <= nVertLevels <= 63 "
                       "(one wavefront holds a column of nVertLevels + 1 levels)";
        return MPAS_EINVAL;
    }
    mpas_ctx* c = new (std::nothrow) mpas_ctx();
    if (!c) return MPAS_ENOMEM;
    int rc = guarded(c, [&] {
        int n = 0;
        hipcheck(hipGetDeviceCount(&n), "hipGetDeviceCount");
        if (device < 0 || device >= n) throw Fail{MPAS_EINVAL, "no such HIP device"};
        hipcheck(hipSetDevice(device), "hipSetDevice");
        hipDeviceProp_t prop;
        hipcheck(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            throw Fail{MPAS_ENOTSUP, std::string("libmpasdyn is built for gfx950, device is ") + prop.gcnArchName};
        c->device = device;
        c->dims = *dims;
        int LP = 8;
        while (LP < dims->nVertLevels + 1) LP <<= 1;
        c->S.nCells = dims->nCells;
        c->S.nEdges = dims->nEdges;
        c->S.nVertices = dims->nVertices;
        c->S.nCO = dims->nCells;  // all owned until mpas_halo_owned says otherwise
        c->S.nEO = dims->nEdges;
        c->S.nVO = dims->nVertices;
        c->S.L = dims->nVertLevels;
        c->S.LP = LP;
        c->S.epw = 2;  // tools/kbench.py: div_damp -3 %, solve_diagnostics -4 % vs 1
        c->S.vcmix = 1;
        c->S.physics = 0;
        c->S.ring1 = 1;
        c->S.xcd = 64;  // runs of 64 blocks per XCD (tools/kbench.py: -2.5 % step time vs dispatcher order)
        c->S.trepw = 1;
        c->S.tro = 64;  // transport: pair-major within runs of 64 entities (profiles/r03/transport_v5: -1 to -3 %)
        c->S.bsplit = 2;  // dyn_tend's flux kernel split off under the MPAS dynamics (profiles/r05/bsplit)
        c->S.etm = 1;  // (the tiled E's best form: profiles/r06/etile)
        c->S.etnt = 256;
        hipcheck(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
        // Field f starts (f % 16) * stagger bytes into its allocation (env MPAS_ALLOC_STAGGER,
        // a multiple of 512: whole columns stay aligned; default 2048): equal-sized arrays
        // read together then do not start on the same HBM channel.  Measured at x1.163842 x 56
        // (interleaved A/B on one box): dyn_tend rk>0 -4 %, rk0 -2 %, step -1.5 % against 0
        size_t stagger = 2048;
        if (const char* v = std::getenv("MPAS_ALLOC_STAGGER")) stagger = (size_t)std::strtoull(v, nullptr, 10) / 512 * 512;
        for (int f = 0; f < X_COUNT; f++) {
            const size_t b = dev_bytes(c, f), off = (size_t)(f % 16) * stagger;
            void* p = nullptr;
            hipError_t e = hipMalloc(&p, b + off);
            if (e != hipSuccess) throw Fail{MPAS_ENOMEM, std::string("hipMalloc ") + kFields[f].name};
            hipcheck(hipMemset(p, 0, b + off), "hipMemset");
            c->raw[f] = p;
            c->S.f[f] = (char*)p + off;
        }
        hipcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
        bounds_add(c);
    });
    if (rc != MPAS_OK) {
        g_create_err = c->err;
        fprintf(stderr, "mpas_ctx_create: %s\n", c->err.c_str());
        mpas_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return MPAS_OK;
}

int mpas_ctx_destroy(mpas_ctx* c) {
    if (!c) return MPAS_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->raw[0]) bounds_remove(c);
    for (int f = 0; f < X_COUNT; f++)
        if (c->raw[f]) (void)hipFree(c->raw[f]);
    for (auto& t : c->pending) {
        (void)hipEventDestroy(t.e0);
        (void)hipEventDestroy(t.e1);
    }
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    graph_drop(c);
    trt_free(c);
    ett_free(c);
    c->halo.reset();
    c->loopgrp.reset();
    for (auto p : c->gid_dev)
        if (p) (void)hipFree(p);
    if (c->sum_scratch) (void)hipFree(c->sum_scratch);
    if (c->keep_flag) (void)hipFree(c->keep_flag);
    if (c->sum_out) (void)hipFree(c->sum_out);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return MPAS_OK;
}

const char* mpas_last_error(const mpas_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

int mpas_sync(mpas_ctx* c) {
    return guarded(c, [&] {
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    });
}

int mpas_get_stream(mpas_ctx* c, void** stream) {
    if (!c || !stream) return MPAS_EINVAL;
    *stream = (void*)c->stream;
    return MPAS_OK;
}

int mpas_set_option(mpas_ctx* c, const char* name, int64_t value) {
    return guarded(c, [&] {
        graph_drop(c);  // every option is baked into a captured step
        if (name && std::strcmp(name, "exact") == 0) c->exact = value ? 1 : 0;
        else if (name && std::strcmp(name, "graph") == 0) c->graph_on = value ? 1 : 0;
        else if (name && std::strcmp(name, "fusedamp") == 0) c->fusedamp = value ? 1 : 0;
        else if (name && std::strcmp(name, "fusesetup") == 0) c->fusesetup = value ? 1 : 0;
        else if (name && std::strcmp(name, "fusecopy") == 0) c->fusecopy = value ? 1 : 0;
        else if (name && std::strcmp(name, "defer4") == 0) c->defer4 = value ? 1 : 0;
        else if (name && std::strcmp(name, "ntu") == 0) c->ntu = value < 0 ? 0 : value > 3 ? 3 : value;
        else if (name && std::strcmp(name, "mdamp") == 0) c->mdamp = value ? 1 : 0;
        else if (name && std::strcmp(name, "mru") == 0) c->mru = value ? 1 : 0;
        else if (name && std::strcmp(name, "msml") == 0) c->msml = value ? 1 : 0;
        else if (name && std::strcmp(name, "vdyn") == 0) c->vdyn = value ? 1 : 0;
        else if (name && std::strcmp(name, "tmedge") == 0) c->tmedge = value ? 1 : 0;
        else if (name && std::strcmp(name, "fusesml") == 0) c->fusesml = value ? 1 : 0;
        else if (name && std::strcmp(name, "smlsum") == 0) c->smlsum = value ? 1 : 0;
        else if (name && std::strcmp(name, "fusedamp_halo") == 0) c->fusedamp_halo = value ? 1 : 0;
        else if (name && std::strcmp(name, "hfuse") == 0) c->hfuse = value < 0 ? 0 : value > 2 ? 2 : value;
        else if (name && std::strcmp(name, "graph_halo") == 0) {
            c->graph_halo = (value == 1 || value == 2) ? value : 0;
            c->graph_refused = false;
        } else if (name && std::strcmp(name, "stub_refuse_capture") == 0) {
            if (!c->halo || !c->halo->stub) throw Fail{MPAS_EINVAL, "stub_refuse_capture: a stub-transport context"};
            c->halo->stub_refuse_capture = value ? 1 : 0;
        }
        else if (name && std::strcmp(name, "stub_latency_us") == 0) {
            if (!c->halo || !c->halo->stub || value < 0 || value > 100000)
                throw Fail{MPAS_EINVAL, "stub_latency_us: a stub-transport context and 0..100000 us"};
            c->halo->stub_latency_us = (int)value;
        }
        else if (name && std::strcmp(name, "xcd") == 0) c->S.xcd = (int)value;
        else if (name && std::strcmp(name, "keep_check") == 0) c->keep_check = value ? 1 : 0;
        else if (name && std::strcmp(name, "epw") == 0) {
            if (value != 1 && value != 2 && value != 4) throw Fail{MPAS_EINVAL, "epw must be 1, 2 or 4"};
            c->S.epw = (int)value;
        } else if (name && std::strcmp(name, "vcmix") == 0) {
            c->S.vcmix = value ? 1 : 0;
        } else if (name && std::strcmp(name, "physics") == 0) {
            if (value < 0 || value > 2)
                throw Fail{MPAS_EINVAL, "physics must be 0 (reference), 1 (MPAS vertical solver) or 2 (MPAS dynamics)"};
            c->S.physics = (int)value;
            if (!value) c->transport = 0;
            c->ett_dirty = true;
        } else if (name && std::strcmp(name, "trorder_e") == 0) {
            if (value < 0 || value > (1 << 20)) throw Fail{MPAS_EINVAL, "trorder_e must be 0 (trorder's), 1 or a run length >= 2"};
            c->S.troe = (int)value;
        } else if (name && std::strcmp(name, "cve") == 0) {
            if (value != 0 && value != 1 && value != 4 && value != 8) throw Fail{MPAS_EINVAL, "cve must be 0, 1, 4 or 8"};
            c->S.cve = (int)value;
        } else if (name && std::strcmp(name, "bsplit") == 0) {
            if (value < 0 || value > 2) throw Fail{MPAS_EINVAL, "bsplit must be 0, 1 or 2"};
            c->S.bsplit = (int)value;
        } else if (name && std::strcmp(name, "trepw") == 0) {
            if (value != 1 && value != 2) throw Fail{MPAS_EINVAL, "trepw must be 1 or 2"};
            c->S.trepw = (int)value;
        } else if (name && std::strcmp(name, "trsu") == 0) {
            c->S.trsu = value ? 1 : 0;
        } else if (name && std::strcmp(name, "trorder") == 0) {
            if (value < 0 || value > (1 << 20)) throw Fail{MPAS_EINVAL, "trorder must be 0, 1 or a run length >= 2"};
            c->S.tro = (int)value;
        } else if (name && std::strcmp(name, "ring1") == 0) {
            c->S.ring1 = value ? 1 : 0;
        } else if (name && std::strcmp(name, "trtile") == 0) {
            c->trtile = value ? 1 : 0;
            c->trt_dirty = c->ett_dirty = true;
        } else if (name && std::strcmp(name, "trsave") == 0) {
            c->trsave = value ? 1 : 0;
        } else if (name && std::strcmp(name, "tredge") == 0) {
            c->tredge = value ? 1 : 0;
            c->trt_dirty = c->ett_dirty = true;
        } else if (name && std::strcmp(name, "trtile_ghosts") == 0) {
            c->trt_ghosts = value ? 1 : 0;
            c->trt_dirty = c->ett_dirty = true;
        } else if (name && std::strcmp(name, "trtcells") == 0) {
            if (value < 1 || value > 256) throw Fail{MPAS_EINVAL, "trtcells must be 1..256"};
            c->trt_cells = (int)value;
            c->trt_dirty = c->ett_dirty = true;
        } else if (name && std::strcmp(name, "trtclo") == 0) {
            if (value < 1 + NF * (2 + AF) || value > 120) throw Fail{MPAS_EINVAL, "trtclo must be 67..120 (LDS columns)"};
            c->trt_clo = (int)value;
            c->trt_dirty = c->ett_dirty = true;
        } else if (name && std::strcmp(name, "etile") == 0) {
            c->etile = value ? 1 : 0;
            c->ett_dirty = true;
        } else if (name && std::strcmp(name, "etmode") == 0) {
            if (value < 0 || value > 2) throw Fail{MPAS_EINVAL, "etmode must be 0, 1 or 2"};
            c->S.etm = (int)value;
        } else if (name && std::strcmp(name, "etthreads") == 0) {
            if (value != 256 && value != 512) throw Fail{MPAS_EINVAL, "etthreads must be 256 or 512"};
            c->S.etnt = (int)value;
        } else if (name && std::strcmp(name, "etcells") == 0) {
            if (value < 1 || value > 40) throw Fail{MPAS_EINVAL, "etcells must be 1..40 (a tile's edges index in one byte)"};
            c->ett_cells = (int)value;
            c->ett_dirty = true;
        } else if (name && std::strcmp(name, "etclo") == 0) {
            if (value < 20 || value > 160) throw Fail{MPAS_EINVAL, "etclo must be 20..160 (LDS columns)"};
            c->ett_clo = (int)value;
            c->ett_dirty = true;
        } else if (name && std::strcmp(name, "transport") == 0) {
            if (value && !c->S.physics) throw Fail{MPAS_EINVAL, "transport needs physics = 1 (it reads the recovered ruAvg, wwAvg, rho_zz)"};
            c->transport = value ? 1 : 0;
        } else if (name && std::strcmp(name, "overlap") == 0) {
            c->overlap = value ? 1 : 0;
            if (c->halo) c->halo->overlap = c->overlap;
        } else if (name && std::strcmp(name, "self") == 0) {
            c->self_on = value ? 1 : 0;
            c->S.selfc = c->self_ok && c->self_on;
        } else if (name && std::strcmp(name, "bounds_probe") == 0) {  // bounds-checked build only
#if MPAS_BOUNDS
            hipcheck(hipSetDevice(c->device), "hipSetDevice");
            hipcheck(launch_bounds_probe(c->S, c->stream, (int)value), "bounds_probe");
#else
            throw Fail{MPAS_ENOTSUP, "bounds_probe needs the bounds-checked build (libmpasdyn_bounds.so)"};
#endif
        } else throw Fail{MPAS_EINVAL, std::string("unknown option ") + (name ? name : "(null)")};
    });
}

int mpas_get_option(mpas_ctx* c, const char* name, int64_t* value) {
    return guarded(c, [&] {
        if (!value) throw Fail{MPAS_EINVAL, "mpas_get_option: null value"};
        if (name && std::strcmp(name, "exact") == 0) *value = c->exact;
        else if (name && std::strcmp(name, "xcd") == 0) *value = c->S.xcd;
        else if (name && std::strcmp(name, "keep_check") == 0) *value = c->keep_check;
        else if (name && std::strcmp(name, "epw") == 0) *value = c->S.epw;
        else if (name && std::strcmp(name, "vcmix") == 0) *value = c->S.vcmix;
        else if (name && std::strcmp(name, "physics") == 0) *value = c->S.physics;
        else if (name && std::strcmp(name, "transport") == 0) *value = c->transport;
        else if (name && std::strcmp(name, "trorder") == 0) *value = c->S.tro;
        else if (name && std::strcmp(name, "trsu") == 0) *value = c->S.trsu;
        else if (name && std::strcmp(name, "trepw") == 0) *value = c->S.trepw;
        else if (name && std::strcmp(name, "cve") == 0) *value = c->S.cve;
        else if (name && std::strcmp(name, "bsplit") == 0) *value = c->S.bsplit;
        else if (name && std::strcmp(name, "trorder_e") == 0) *value = c->S.troe;
        else if (name && std::strcmp(name, "trtile") == 0) *value = c->trtile;
        else if (name && std::strcmp(name, "tredge") == 0) *value = c->tredge;
        else if (name && std::strcmp(name, "trsave") == 0) *value = c->trsave;
        else if (name && std::strcmp(name, "tredge_active") == 0) {  // edge groups built for this mesh
            trt_ensure(c);
            *value = c->S.tre != nullptr;
        } else if (name && std::strcmp(name, "tredge_irregular") == 0) {
            trt_ensure(c);
            *value = c->tre.nirr;
        }
        else if (name && std::strcmp(name, "ring1") == 0) *value = c->S.ring1;
        else if (name && std::strcmp(name, "trtcells") == 0) *value = c->trt_cells;
        else if (name && std::strcmp(name, "trtile_ghosts") == 0) *value = c->trt_ghosts;
        else if (name && std::strcmp(name, "trtclo") == 0) *value = c->trt_clo;
        else if (name && std::strcmp(name, "trtile_active") == 0) {  // tiles built for this mesh
            trt_ensure(c);
            *value = c->S.trt ? 1 : 0;
        } else if (name && std::strcmp(name, "trtile_count") == 0) {
            trt_ensure(c);
            *value = c->trt.ntiles;
        }
        else if (name && std::strcmp(name, "etile") == 0) *value = c->etile;
        else if (name && std::strcmp(name, "etcells") == 0) *value = c->ett_cells;
        else if (name && std::strcmp(name, "etmode") == 0) *value = c->S.etm;
        else if (name && std::strcmp(name, "etthreads") == 0) *value = c->S.etnt;
        else if (name && std::strcmp(name, "etclo") == 0) *value = c->ett_clo;
        else if (name && std::strcmp(name, "etile_active") == 0) {  // dyn_tend tiles built for this mesh
            ett_ensure(c);
            *value = c->S.ett ? 1 : 0;
        } else if (name && std::strcmp(name, "etile_count") == 0) {
            ett_ensure(c);
            *value = c->ett.ntiles;
        } else if (name && std::strcmp(name, "etile_columns") == 0) {  // closure columns staged per launch
            ett_ensure(c);
            *value = c->ett.nclo;
        } else if (name && std::strcmp(name, "etile_maxclo") == 0) {
            ett_ensure(c);
            *value = c->ett.maxclo;
        }
        else if (name && std::strcmp(name, "overlap") == 0) *value = c->overlap;
        else if (name && std::strcmp(name, "fusedamp") == 0) *value = c->fusedamp;
        else if (name && std::strcmp(name, "fusesetup") == 0) *value = c->fusesetup;
        else if (name && std::strcmp(name, "fusecopy") == 0) *value = c->fusecopy;
        else if (name && std::strcmp(name, "defer4") == 0) *value = c->defer4;
        else if (name && std::strcmp(name, "ntu") == 0) *value = c->ntu;
        else if (name && std::strcmp(name, "mdamp") == 0) *value = c->mdamp;
        else if (name && std::strcmp(name, "mru") == 0) *value = c->mru;
        else if (name && std::strcmp(name, "msml") == 0) *value = c->msml;
        else if (name && std::strcmp(name, "vdyn") == 0) *value = c->vdyn;
        else if (name && std::strcmp(name, "eoe_same") == 0) {
            prepare_now(c);
            *value = c->S.eoe_same;
        }
        else if (name && std::strcmp(name, "tmedge") == 0) *value = c->tmedge;
        else if (name && std::strcmp(name, "fusesml") == 0) *value = c->fusesml;
        else if (name && std::strcmp(name, "smlsum") == 0) *value = c->smlsum;
        else if (name && std::strcmp(name, "fusedamp_halo") == 0) *value = c->fusedamp_halo;
        else if (name && std::strcmp(name, "hfuse") == 0) *value = c->hfuse;
        else if (name && std::strcmp(name, "hfuse_active") == 0) *value = hfuse_active(c);
        else if (name && std::strcmp(name, "graph_halo") == 0) *value = c->graph_halo;
        else if (name && std::strcmp(name, "graph_fallbacks") == 0) *value = c->graph_fallbacks;
        else if (name && std::strcmp(name, "graph_refused") == 0) *value = c->graph_refused ? 1 : 0;
        else if (name && std::strcmp(name, "stub_latency_us") == 0) *value = c->halo ? c->halo->stub_latency_us : 0;
        else if (name && std::strcmp(name, "halo_state") == 0) {  // hash of the halo bookkeeping (debug)
            uint64_t hsh = 1469598103934665603ull;
            if (c->halo)
                for (uint8_t v : c->halo->stale) hsh = (hsh ^ v) * 1099511628211ull;
            *value = (int64_t)(hsh >> 1);
        }
        else if (name && std::strcmp(name, "fusedamp_active") == 0)
            *value = c->fusedamp && c->S.physics == 0 &&
                     (!c->halo || (c->fusedamp_halo && c->S.ring1 && c->S.nERing >= c->S.nEO));
        else if (name && std::strcmp(name, "orphan_edges") == 0) {  // edges no cell lists (k_prepare)
            prepare_now(c);
            *value = c->S.n_orph;
        }
        else if (name && std::strcmp(name, "self") == 0) *value = c->self_on;
        else if (name && std::strcmp(name, "graph") == 0) *value = c->graph_on;
        else if (name && std::strcmp(name, "graph_captures") == 0) *value = c->graph_captures;
        else if (name && std::strcmp(name, "graph_launches") == 0) *value = c->graph_launches;
        else if (name && std::strcmp(name, "bounds") == 0) *value = MPAS_BOUNDS;  // the bounds-checked build
#if MPAS_BOUNDS
        else if (name && std::strcmp(name, "bounds_units") == 0) {  // kernel units checking / registered
            *value = ((int64_t)bounds_units() << 32) | (int64_t)bounds_tus().size();
        }
#endif
        else if (name && std::strcmp(name, "selfc") == 0) {
            if (c->dirty) {  // decide now (needs the mesh uploaded)
                hipcheck(hipSetDevice(c->device), "hipSetDevice");
                hipcheck(launch_prepare(c->S, c->stream), "prepare");
                c->self_ok = c->S.selfc;
                c->S.selfc = c->self_ok && c->self_on;
                c->dirty = false;
            }
            *value = c->S.selfc;
        } else throw Fail{MPAS_EINVAL, std::string("unknown option ") + (name ? name : "(null)")};
    });
}

int mpas_upload(mpas_ctx* c, int f, const void* host, int64_t se, int64_t sl, int64_t sc) {
    return guarded(c, [&] {
        if (f < 0 || f >= F_COUNT || !host) throw Fail{MPAS_EINVAL, "mpas_upload: bad field or pointer"};
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
        const FieldInfo& fi = kFields[f];
        const int n = entity_count(c, fi.kind), L = c->S.L, LP = c->S.LP, W = fi.width;
        const char* h = (const char*)host;
        std::vector<char> staged;  // a device view of a 2-D field / ZV: staged through the host
        if (is_device_ptr(host)) {
            if (is_3d(fi.kind)) {  // device to device, no host round trip
                hipcheck(launch_view_copy(c->S.f[f], (void*)host, fi.kind == K_C3B ? 1 : 8, n, W, L, LP, se, sl, sc, 1,
                                          c->stream),
                         "upload view");
                if (fi.kind != K_C3V && fi.kind != K_C3B && W == 1)
                    hipcheck(launch_keep_refresh(c->S, c->stream, f, keep_kind(f)), "keep_refresh");
                hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
                c->dirty = true;
                c->trt_dirty = c->ett_dirty = true;
                graph_drop(c);
                if (c->halo) c->halo->stale[f] = 0;
                return;
            }
            const size_t span = fi.kind == K_ZV ? (size_t)(L * sl + 8)
                                                : view_span(n, W, 0, se, 0, sc, elem_size(fi.kind));
            staged.resize(span);
            hipcheck(hipMemcpy(staged.data(), host, span, hipMemcpyDeviceToHost), "hipMemcpy D2H (view)");
            h = staged.data();
        }
        size_t bytes = dev_bytes(c, f);
        std::vector<char> buf(bytes, 0);
        if (fi.kind == K_C3 || fi.kind == K_E3 || fi.kind == K_V3) {
            double* d = (double*)buf.data();
            for (int e = 0; e < n; e++)
                for (int k = 0; k <= L; k++) d[(size_t)e * LP + lpos(LP, k)] = *(const double*)(h + e * se + k * sl);
            if (W == 1) {  // the keep tails: level L and level 0 of every column (the zero slot's: 0)
                const size_t rows = (size_t)n + 1;
                for (int e = 0; e < n; e++) {
                    d[rows * LP + e] = d[(size_t)e * LP + lpos(LP, L)];
                    d[rows * LP + rows + e] = d[(size_t)e * LP + lpos(LP, 0)];
                }
            }
        } else if (fi.kind == K_C3V) {
            double* d = (double*)buf.data();
            for (int e = 0; e < n; e++)
                for (int i = 0; i < W; i++)
                    for (int k = 0; k <= L; k++)
                        d[vidx(W, LP, e, i, k)] = *(const double*)(h + e * se + k * sl + i * sc);
        } else if (fi.kind == K_C3B) {
            uint8_t* d = (uint8_t*)buf.data();
            for (int e = 0; e < n; e++)
                for (int k = 0; k <= L; k++) d[(size_t)e * LP + lpos(LP, k)] = *(const uint8_t*)(h + e * se + k * sl);
        } else if (fi.kind == K_ZV) {
            double* d = (double*)buf.data();
            for (int k = 0; k <= L; k++) d[k] = *(const double*)(h + k * sl);
        } else if (elem_size(fi.kind) == 4) {
            int32_t* d = (int32_t*)buf.data();
            int tgt = id_target(f);
            int lim = tgt < 0 ? 0 : entity_count(c, tgt);
            // list lengths: the kernels index rows of this width with them (tail loops past
            // the unrolled entries), so a longer list would read past the row -- refused
            const int width = count_width(f);
            for (int e = 0; e < n; e++)
                for (int i = 0; i < W; i++) {
                    int32_t v = *(const int32_t*)(h + e * se + i * sc);
                    if (tgt >= 0 && (v < 0 || v > lim)) v = lim;  // Q1 zero slot
                    if (width > 0 && v > width)
                        throw Fail{MPAS_EINVAL, std::string("mpas_upload: ") + fi.name + " " + std::to_string(v) +
                                                    " at entity " + std::to_string(e) + " exceeds its list width " +
                                                    std::to_string(width)};
                    d[(size_t)e * W + i] = v;
                }
        } else {
            double* d = (double*)buf.data();
            for (int e = 0; e < n; e++)
                for (int i = 0; i < W; i++) d[(size_t)e * W + i] = *(const double*)(h + e * se + i * sc);
        }
        hipcheck(hipMemcpy(c->S.f[f], buf.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy H2D");
        c->dirty = true;
        c->trt_dirty = c->ett_dirty = true;
        graph_drop(c);
        if (c->halo) c->halo->stale[f] = 0;  // uploaded ghosts are the global values
        // derived mesh arrays: cos()/sin() on the host with the same libm as the oracle
        struct { int src, dst; double (*fn)(double); } der[] = {
            {F_angleEdge, X_cosAngleEdge, ::cos}, {F_latEdge, X_cosLatEdge, ::cos}, {F_lat, X_cosLatCell, ::cos},
            {F_lat, X_sinLatCell, ::sin},         {F_lon, X_cosLonCell, ::cos},      {F_lon, X_sinLonCell, ::sin}};
        for (const auto& dv : der) {
            if (dv.src != f) continue;
            std::vector<double> cs((size_t)n + 1, 0.0);
            const double* d = (const double*)buf.data();
            for (int e = 0; e < n; e++) cs[e] = dv.fn(d[e]);
            cs[n] = dv.fn(0.0);  // zero slot: as the oracle computes it from its zero row
            hipcheck(hipMemcpy(c->S.f[dv.dst], cs.data(), cs.size() * 8, hipMemcpyHostToDevice), "hipMemcpy H2D");
        }
    });
}

int mpas_download(mpas_ctx* c, int f, void* host, int64_t se, int64_t sl, int64_t sc) {
    return guarded(c, [&] {
        if (f < 0 || f >= F_COUNT || !host) throw Fail{MPAS_EINVAL, "mpas_download: bad field or pointer"};
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
        const FieldInfo& fi = kFields[f];
        const int n = entity_count(c, fi.kind), L = c->S.L, LP = c->S.LP, W = fi.width;
        void* dview = nullptr;  // a device view of a 2-D field / ZV: staged through the host
        std::vector<char> staged;
        if (is_device_ptr(host)) {
            if (is_3d(fi.kind)) {
                hipcheck(launch_view_copy(c->S.f[f], host, fi.kind == K_C3B ? 1 : 8, n, W, L, LP, se, sl, sc, 0,
                                          c->stream),
                         "download view");
                hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
                return;
            }
            const size_t span = fi.kind == K_ZV ? (size_t)(L * sl + 8)
                                                : view_span(n, W, 0, se, 0, sc, elem_size(fi.kind));
            staged.resize(span);
            hipcheck(hipMemcpy(staged.data(), host, span, hipMemcpyDeviceToHost), "hipMemcpy D2H (view)");
            dview = host;
            host = staged.data();
        }
        size_t bytes = dev_bytes(c, f);
        std::vector<char> buf(bytes);
        hipcheck(hipMemcpy(buf.data(), c->S.f[f], bytes, hipMemcpyDeviceToHost), "hipMemcpy D2H");
        char* h = (char*)host;
        if (fi.kind == K_C3 || fi.kind == K_E3 || fi.kind == K_V3) {
            const double* d = (const double*)buf.data();
            for (int e = 0; e < n; e++)
                for (int k = 0; k <= L; k++) *(double*)(h + e * se + k * sl) = d[(size_t)e * LP + lpos(LP, k)];
        } else if (fi.kind == K_C3V) {
            const double* d = (const double*)buf.data();
            for (int e = 0; e < n; e++)
                for (int i = 0; i < W; i++)
                    for (int k = 0; k <= L; k++)
                        *(double*)(h + e * se + k * sl + i * sc) = d[vidx(W, LP, e, i, k)];
        } else if (fi.kind == K_C3B) {
            const uint8_t* d = (const uint8_t*)buf.data();
            for (int e = 0; e < n; e++)
                for (int k = 0; k <= L; k++) *(uint8_t*)(h + e * se + k * sl) = d[(size_t)e * LP + lpos(LP, k)];
        } else if (fi.kind == K_ZV) {
            const double* d = (const double*)buf.data();
            for (int k = 0; k <= L; k++) *(double*)(h + k * sl) = d[k];
        } else if (elem_size(fi.kind) == 4) {
            const int32_t* d = (const int32_t*)buf.data();
            for (int e = 0; e < n; e++)
                for (int i = 0; i < W; i++) *(int32_t*)(h + e * se + i * sc) = d[(size_t)e * W + i];
        } else {
            const double* d = (const double*)buf.data();
            for (int e = 0; e < n; e++)
                for (int i = 0; i < W; i++) *(double*)(h + e * se + i * sc) = d[(size_t)e * W + i];
        }
        if (dview)  // the staged image back into the device view (the bytes between its
                    // elements came from it, so they are unchanged)
            hipcheck(hipMemcpy(dview, staged.data(), staged.size(), hipMemcpyHostToDevice), "hipMemcpy H2D (view)");
    });
}

int mpas_fill_synthetic(mpas_ctx* c, uint64_t seed) {
    return guarded(c, [&] {
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        hipcheck(launch_fill_synthetic(c->S, c->stream, seed), "fill_synthetic");
        keep_refresh_all(c);
        hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
        if (c->halo)  // filled from global ids: ghosts hold the global values
            for (auto& v : c->halo->stale) v = 0;
    });
}

// ---- decomposition (mpasdyn/decomp.py builds the local state and the plan) ----------
namespace {
Halo* halo_of(mpas_ctx* c) {
    if (!c->halo) {
        c->halo.reset(new Halo());
        c->halo->stale.assign(X_COUNT, 0);
        c->S.halo = c->halo.get();
    }
    return c->halo.get();
}
int* dev_ints(const int32_t* h, int n) {
    int* d = nullptr;
    hipcheck(hipMalloc(&d, sizeof(int) * (size_t)(n > 0 ? n : 1)), "hipMalloc");
    if (n > 0) hipcheck(hipMemcpy(d, h, sizeof(int) * (size_t)n, hipMemcpyHostToDevice), "hipMemcpy H2D");
    return d;
}
}  // namespace

int mpas_halo_owned(mpas_ctx* c, int32_t nCellsOwned, int32_t nEdgesOwned, int32_t nVerticesOwned) {
    return guarded(c, [&] {
        graph_drop(c);
        if (nCellsOwned < 0 || nCellsOwned > c->S.nCells || nEdgesOwned < 0 || nEdgesOwned > c->S.nEdges ||
            nVerticesOwned < 0 || nVerticesOwned > c->S.nVertices)
            throw Fail{MPAS_EINVAL, "mpas_halo_owned: owned counts exceed the local counts"};
        c->S.nCO = nCellsOwned;
        c->S.nEO = nEdgesOwned;
        c->S.nVO = nVerticesOwned;
        c->dirty = true;
        c->trt_dirty = c->ett_dirty = true;
    });
}

int mpas_halo_ring1(mpas_ctx* c, int32_t nEdgesRing1, int32_t nVerticesRing1) {
    return guarded(c, [&] {
        graph_drop(c);
        if (nEdgesRing1 < c->S.nEO || nEdgesRing1 > c->S.nEdges || nVerticesRing1 < c->S.nVO ||
            nVerticesRing1 > c->S.nVertices)
            throw Fail{MPAS_EINVAL, "mpas_halo_ring1: needs owned <= count <= local, edges and vertices"};
        c->S.nERing = nEdgesRing1;
        c->S.nVRing = nVerticesRing1;
    });
}

int mpas_halo_interior(mpas_ctx* c, int32_t nCI, int32_t nEI, int32_t nVI) {
    return guarded(c, [&] {
        graph_drop(c);
        if (nCI < 0 || nCI > c->S.nCO || nEI < 0 || nEI > c->S.nEO || nVI < 0 || nVI > c->S.nVO)
            throw Fail{MPAS_EINVAL, "mpas_halo_interior: interior counts exceed the owned counts"};
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        Halo* h = halo_of(c);
        h->nint[0] = nCI;
        h->nint[1] = nEI;
        h->nint[2] = nVI;
        h->interior = true;
        h->overlap = c->overlap;
        c->trt_dirty = c->ett_dirty = true;
        if (!h->comm) {  // the halo stream, at the device's highest priority
            int least = 0, greatest = 0;
            hipcheck(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
            hipcheck(hipStreamCreateWithPriority(&h->comm, hipStreamNonBlocking, greatest), "hipStreamCreate");
            hipcheck(hipEventCreateWithFlags(&h->ev_ready, hipEventDisableTiming), "hipEventCreate");
            hipcheck(hipEventCreateWithFlags(&h->ev_done, hipEventDisableTiming), "hipEventCreate");
        }
    });
}

int mpas_halo_plan(mpas_ctx* c, int kind, int peer, const int32_t* send_ids, int32_t nsend, const int32_t* recv_ids,
                   int32_t nrecv) {
    return guarded(c, [&] {
        if (kind < 0 || kind > 2 || peer < 0 || nsend < 0 || nrecv < 0 || (nsend && !send_ids) || (nrecv && !recv_ids))
            throw Fail{MPAS_EINVAL, "mpas_halo_plan: bad arguments"};
        const int lim = kind == 0 ? c->S.nCells : kind == 1 ? c->S.nEdges : c->S.nVertices;
        const int own = kind == 0 ? c->S.nCO : kind == 1 ? c->S.nEO : c->S.nVO;
        for (int i = 0; i < nsend; i++)
            if (send_ids[i] < 0 || send_ids[i] >= own) throw Fail{MPAS_EINVAL, "mpas_halo_plan: send id not owned"};
        for (int i = 0; i < nrecv; i++)
            if (recv_ids[i] < own || recv_ids[i] >= lim) throw Fail{MPAS_EINVAL, "mpas_halo_plan: recv id not a ghost"};
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        Halo* h = halo_of(c);
        HaloPeer p;
        p.peer = peer;
        p.nsend = nsend;
        p.nrecv = nrecv;
        p.d_send = dev_ints(send_ids, nsend);
        p.d_recv = dev_ints(recv_ids, nrecv);
        h->peers[kind].push_back(p);
        h->clear_tabs();  // the pack / unpack tables follow the plan
        c->graph_refused = false;
        graph_drop(c);
    });
}

int mpas_set_global_ids(mpas_ctx* c, int kind, const int32_t* gids, int32_t n) {
    return guarded(c, [&] {
        const int lim = kind == 0 ? c->S.nCells : kind == 1 ? c->S.nEdges : c->S.nVertices;
        if (kind < 0 || kind > 2 || n != lim || !gids) throw Fail{MPAS_EINVAL, "mpas_set_global_ids: bad arguments"};
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        if (c->gid_dev[kind]) hipcheck(hipFree(c->gid_dev[kind]), "hipFree");
        c->gid_dev[kind] = dev_ints(gids, n);
        c->S.gid[kind] = c->gid_dev[kind];
    });
}

int mpas_halo_loopback(mpas_ctx** ctxs, int n) {
    if (!ctxs || n < 1) return MPAS_EINVAL;
    for (int i = 0; i < n; i++)
        if (!ctxs[i] || ctxs[i]->device != ctxs[0]->device) return MPAS_EINVAL;
    return guarded(ctxs[0], [&] {
        hipcheck(hipSetDevice(ctxs[0]->device), "hipSetDevice");
        auto g = std::make_shared<LoopGroup>();
        g->n = n;
        g->packed.resize(n);
        g->copied.resize(n);
        for (int i = 0; i < n; i++) {
            hipcheck(hipEventCreateWithFlags(&g->packed[i], hipEventDisableTiming), "hipEventCreate");
            hipcheck(hipEventCreateWithFlags(&g->copied[i], hipEventDisableTiming), "hipEventCreate");
            hipcheck(hipEventRecord(g->copied[i], ctxs[i]->stream), "hipEventRecord");
        }
        for (int i = 0; i < n; i++) {
            Halo* h = halo_of(ctxs[i]);
            hipcheck(h->reserve(ctxs[i]->S.LP), "halo buffers");
            h->nranks = n;
            h->rank = i;
            h->loop = g.get();
            g->members.push_back(h);
            g->streams.push_back(ctxs[i]->stream);
            ctxs[i]->loopgrp = g;
        }
    });
}

int mpas_rccl_unique_id(void* out128) {
    if (!out128) return MPAS_EINVAL;
    std::string err;
    if (rccl_unique_id(out128, err) != 0) {
        g_create_err = err;
        return MPAS_ERCCL;
    }
    return MPAS_OK;
}

int mpas_halo_rccl(mpas_ctx* c, int nranks, int rank, const void* id128) {
    return guarded(c, [&] {
        if (nranks < 1 || rank < 0 || rank >= nranks || !id128) throw Fail{MPAS_EINVAL, "mpas_halo_rccl: bad arguments"};
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        Halo* h = halo_of(c);
        hipcheck(h->reserve(c->S.LP), "halo buffers");
        std::string err;
        if (rccl_init(h, nranks, rank, id128, err) != 0) throw Fail{MPAS_ERCCL, err};
    });
}

int mpas_halo_socket(mpas_ctx* c, int nranks, int rank, const char* host, int base_port) {
    return guarded(c, [&] {
        if (nranks < 1 || rank < 0 || rank >= nranks || !host || base_port <= 0 || base_port + nranks > 65535)
            throw Fail{MPAS_EINVAL, "mpas_halo_socket: bad arguments"};
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        Halo* h = halo_of(c);
        if (h->rccl || h->loop || h->stub || h->sock) throw Fail{MPAS_EINVAL, "mpas_halo_socket: the context already has a transport"};
        hipcheck(h->reserve(c->S.LP), "halo buffers");
        std::string err;
        if (sock_init(h, nranks, rank, host, base_port, err) != 0) throw Fail{MPAS_EINVAL, err};
        graph_drop(c);
    });
}

int mpas_halo_stub(mpas_ctx* c) {
    return guarded(c, [&] {
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        Halo* h = halo_of(c);
        if (h->rccl || h->loop || h->sock) throw Fail{MPAS_EINVAL, "mpas_halo_stub: the context already has a transport"};
        hipcheck(h->reserve(c->S.LP), "halo buffers");
        h->stub = true;
        graph_drop(c);
    });
}

int mpas_halo_stats(mpas_ctx* c, int64_t* exchanges, int64_t* fields) {
    if (!c || !exchanges || !fields) return MPAS_EINVAL;
    *exchanges = c->halo ? c->halo->exchanges : 0;
    *fields = c->halo ? c->halo->fields_moved : 0;
    return MPAS_OK;
}

#define MPAS_TASK(NAME, CALL) \
    return guarded(c, [&] { run_task(c, NAME, [&] { return CALL; }); })

int mpas_atm_rk_integration_setup(mpas_ctx* c) {
    MPAS_TASK("atm_rk_integration_setup", launch_rk_integration_setup(c->S, c->stream));
}
int mpas_atm_compute_moist_coefficients(mpas_ctx* c) {
    MPAS_TASK("atm_compute_moist_coefficients", launch_moist_coefficients(c->S, c->stream));
}
int mpas_atm_compute_vert_imp_coefs(mpas_ctx* c, double dts) {
    MPAS_TASK("atm_compute_vert_imp_coefs", launch_vert_imp_coefs(c->S, c->stream, dts));
}
int mpas_atm_compute_dyn_tend_work(mpas_ctx* c, int rk_step, double dt, int horiz_mixing, double cam_coef, int mix_full,
                                   int rayleigh_damp_u) {
    if (!c) return MPAS_EINVAL;
    DynTendArgs a{rk_step, dt, horiz_mixing, cam_coef, mix_full, rayleigh_damp_u, c->exact};
    MPAS_TASK(rk_step == 0 ? "atm_compute_dyn_tend_work[rk0]" : "atm_compute_dyn_tend_work[rk>0]",
              launch_dyn_tend(c->S, c->stream, a));
}
int mpas_atm_set_smlstep_pert_variables_work(mpas_ctx* c) {
    MPAS_TASK("atm_set_smlstep_pert_variables_work", launch_set_smlstep(c->S, c->stream, c->exact));
}
int mpas_atm_advance_acoustic_step_work(mpas_ctx* c, double dts, int small_step) {
    MPAS_TASK(acoustic_name(small_step), launch_acoustic(c->S, c->stream, dts, small_step, c->exact));
}
int mpas_atm_divergence_damping_3d(mpas_ctx* c, double dts) {
    MPAS_TASK("atm_divergence_damping_3d", launch_div_damping(c->S, c->stream, dts));
}
int mpas_atm_compute_solve_diagnostics(mpas_ctx* c, int hollingsworth, int rk_step) {
    MPAS_TASK("atm_compute_solve_diagnostics", launch_solve_diagnostics(c->S, c->stream, hollingsworth, rk_step));
}
int mpas_atm_rk_dynamics_substep_finish(mpas_ctx* c, int substep, int split) {
    if (split == 0) return MPAS_EINVAL;
    MPAS_TASK("atm_rk_dynamics_substep_finish", launch_substep_finish(c->S, c->stream, substep, split));
}

int mpas_atm_recover_large_step_variables_work(mpas_ctx* c, int ns, int rk_step, double dt) {
    if (ns == 0) return MPAS_EINVAL;
    MPAS_TASK(recover_name(rk_step), launch_recover_large_step(c->S, c->stream, ns, rk_step, dt));
}
int mpas_reconstruct_2d(mpas_ctx* c, int includeHalos, int on_a_sphere) {
    (void)includeHalos;  // :1909-1912: the range is nCells either way
    MPAS_TASK("mpas_reconstruct_2d", launch_reconstruct_2d(c->S, c->stream, on_a_sphere ? 1 : 0));
}
// (the init tasks write state fields at every level from outside the step: the keep tails
// follow them, mpas_dev.h)
int mpas_atm_compute_damping_coefs(mpas_ctx* c, double config_zd, double config_xnutr) {
    return guarded(c, [&] {
        run_task(c, "atm_compute_damping_coefs",
                 [&] { return launch_damping_coefs(c->S, c->stream, config_zd, config_xnutr); });
        keep_refresh_all(c);
    });
}
int mpas_atm_init_coupled_diagnostics(mpas_ctx* c) {
    return guarded(c, [&] {
        run_task(c, "atm_init_coupled_diagnostics", [&] { return launch_init_coupled_diagnostics(c->S, c->stream); });
        keep_refresh_all(c);
    });
}
// the mesh tasks of atm_core_init (k_mesh.hip); the adv lists feed k_prepare's edge
// records and the transport tiles, so they are re-derived before the next task
int mpas_atm_compute_signs(mpas_ctx* c) { MPAS_TASK("atm_compute_signs", launch_compute_signs(c->S, c->stream)); }
int mpas_atm_adv_coef_compression(mpas_ctx* c) {
    return guarded(c, [&] {
        run_task(c, "atm_adv_coef_compression", [&] { return launch_adv_coef_compression(c->S, c->stream); });
        c->dirty = true;
        c->trt_dirty = c->ett_dirty = true;
        graph_drop(c);
    });
}
int mpas_atm_couple_coef_3rd_order(mpas_ctx* c, double config_coef_3rd_order) {
    MPAS_TASK("atm_couple_coef_3rd_order", launch_couple_coef_3rd_order(c->S, c->stream, config_coef_3rd_order));
}
int mpas_atm_compute_mesh_scaling(mpas_ctx* c, int config_h_ScaleWithMesh) {
    MPAS_TASK("atm_compute_mesh_scaling", launch_mesh_scaling(c->S, c->stream, config_h_ScaleWithMesh));
}
int mpas_atm_core_init(mpas_ctx* c) {
    // atm_core.rg:22-42 in order (physics_init is a stub, OUT OF SCOPE; the namelist values
    // config_coef_3rd_order = 0.25, config_h_ScaleWithMesh = true, config_zd = 22000,
    // config_xnutr = 0.2)
    return guarded(c, [&] {
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        const DevState& S = c->S;
        hipStream_t st = c->stream;
        run_task(c, "atm_compute_signs", [&] { return launch_compute_signs(S, st); });
        run_task(c, "atm_adv_coef_compression", [&] { return launch_adv_coef_compression(S, st); });
        c->dirty = true;  // (k_prepare re-derives the edge records before the next task)
        c->trt_dirty = c->ett_dirty = true;
        graph_drop(c);
        run_task(c, "atm_couple_coef_3rd_order", [&] { return launch_couple_coef_3rd_order(S, st, 0.25); });
        run_task(c, "atm_init_coupled_diagnostics", [&] { return launch_init_coupled_diagnostics(S, st); });
        run_task(c, "atm_compute_solve_diagnostics", [&] { return launch_solve_diagnostics(S, st, 0, -1); });
        run_task(c, "mpas_reconstruct_2d", [&] { return launch_reconstruct_2d(S, st, 1); });
        run_task(c, "atm_compute_mesh_scaling", [&] { return launch_mesh_scaling(S, st, 1); });
        run_task(c, "atm_compute_damping_coefs", [&] { return launch_damping_coefs(S, st, 22000.0, 0.2); });
        keep_refresh_all(c);  // (the init tasks write the state from outside the step)
    });
}
int mpas_atm_advance_scalars_mono(mpas_ctx* c, double dt) {
    if (!c) return MPAS_EINVAL;
    return guarded(c, [&] {
        run_task(c, "atm_advance_scalars_mono", [&] {
            trt_ensure(c);
            return launch_advance_scalars_mono(c->S, c->stream, dt);
        });
    });
}
int mpas_atm_compute_output_diagnostics(mpas_ctx* c) {
    MPAS_TASK("atm_compute_output_diagnostics", launch_output_diagnostics(c->S, c->stream));
}
int mpas_summarize_timestep(mpas_ctx* c, int detailed, int global_vel, int global_sca, double* out) {
    (void)global_sca;  // prints a blank line only (rk_timestep.rg:352-357)
    return guarded(c, [&] {
        if (!out) throw Fail{MPAS_EINVAL, "mpas_summarize_timestep: null out"};
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        double h[31] = {0};
        if (detailed || global_vel) {
            if (!c->sum_scratch) hipcheck(hipMalloc(&c->sum_scratch, summarize_scratch_bytes()), "hipMalloc");
            if (!c->sum_out) hipcheck(hipMalloc((void**)&c->sum_out, 31 * sizeof(double)), "hipMalloc");
            run_task(c, "summarize_timestep", [&] { return launch_summarize(c->S, c->stream, c->sum_scratch, c->sum_out); });
            hipcheck(hipMemcpyAsync(h, c->sum_out, sizeof h, hipMemcpyDeviceToHost, c->stream), "hipMemcpy D2H");
            hipcheck(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
            if (!detailed)
                for (int i = 0; i < 27; i++) h[i] = 0.0;
            if (!global_vel)
                for (int i = 27; i < 31; i++) h[i] = 0.0;
        }
        std::memcpy(out, h, sizeof h);
    });
}

int mpas_atm_srk3(mpas_ctx* c, double dt, int schedule) {
    return guarded(c, [&] {
        hipcheck(hipSetDevice(c->device), "hipSetDevice");
        srk3_step(c, dt, schedule);
    });
}
int mpas_atm_timestep(mpas_ctx* c, double dt) { return mpas_atm_srk3(c, dt, 0); }

int mpas_timing_enable(mpas_ctx* c, int on) {
    return guarded(c, [&] { c->timing = on != 0; });
}
int mpas_timing_reset(mpas_ctx* c) {
    return guarded(c, [&] {
        harvest(c);
        for (auto& x : c->task_calls) x = 0;
        for (auto& x : c->task_ms) x = 0.0;
    });
}
int mpas_timing_count(mpas_ctx* c) {
    if (!c) return MPAS_EINVAL;
    int rc = guarded(c, [&] { harvest(c); });
    return rc != MPAS_OK ? rc : (int)c->task_names.size();
}
int mpas_timing_get(mpas_ctx* c, int idx, const char** name, int64_t* calls, double* total_ms) {
    return guarded(c, [&] {
        harvest(c);
        if (idx < 0 || idx >= (int)c->task_names.size()) throw Fail{MPAS_EINVAL, "timing index"};
        if (name) *name = c->task_names[idx].c_str();
        if (calls) *calls = c->task_calls[idx];
        if (total_ms) *total_ms = c->task_ms[idx];
    });
}

}  // extern "C"
