// mpas_halo.h -- halo exchange of the horizontally decomposed hot path.
//
// Each rank owns a subdomain plus the ghost entities its owned entities reach through
// the index arrays (mpasdyn/decomp.py builds the local numbering and the plan).  Every
// kernel computes owned entities only.  A field gathered by a kernel must be fresh on
// the ghosts: the launchers declare, per kernel, the fields it gathers through an index
// array (halo_before) and the fields it writes (halo_wrote).  A written field becomes
// stale; the next kernel that gathers it first exchanges it (one grouped exchange of
// all its stale gathered fields), after which it is fresh.  Correct by construction
// given complete gather lists -- the loopback N-shard = 1-shard parity test checks them.
//
// Overlap: the owned entities are numbered interior first -- an interior
// entity reaches no ghost through any index array (decomp.py) -- so a kernel that needs
// an exchange computes its interior entities while the exchange runs on the halo stream
// (pack, send/recv, unpack), then its boundary entities once the ghosts have arrived.
// The launchers hand the kernel launch to HALO_RUN as a function of the DevState range.
//
// Transport: RCCL point-to-point (ncclSend/ncclRecv of one packed buffer per peer inside
// ncclGroupStart/End, on the task stream; librccl resolved with dlopen, so the process
// shares the RCCL that torch.distributed loaded) for one process per GPU, or an
// in-process loopback for N contexts on one device driven by N host threads (hipMemcpy
// between the contexts' buffers; the single-GPU test of the decomposition), or a
// host-staged TCP transport for N processes that may share one device (RCCL refuses two
// ranks on one GPU): the packed regions go device -> host -> socket -> host -> device,
// synchronously -- the multi-process test of the same pack / plan / unpack code.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <initializer_list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace mpas {

struct DevState;

enum HaloKind { HK_CELL = 0, HK_EDGE = 1, HK_VERTEX = 2 };

struct HaloPeer {
    int peer = -1;
    int nsend = 0, nrecv = 0;
    int* d_send = nullptr;  // local ids, device
    int* d_recv = nullptr;
};

struct LoopGroup;  // loopback transport shared by the contexts of one process
struct HaloSeg;    // one segment of a pack / unpack (mpas_halo.hip)
struct HaloCopyTab {  // the device segment table of one direction of one exchange signature
    HaloSeg* dev = nullptr;
    double** addr = nullptr;  // per buffer column: the field column it moves (built once, on the device)
    int nseg = 0;
    long ncol = 0;  // buffer columns covered
    std::shared_ptr<std::vector<HaloSeg>> host;
};
struct RcclComm;   // RCCL transport
struct SockComm;   // host-staged TCP transport (multi-process runs without RCCL)

struct Halo {
    int nranks = 1, rank = 0;
    std::vector<HaloPeer> peers[3];
    // per field id: 0 fresh on every ghost, 1 stale, 2 fresh on the ring-1 ghosts of its
    // kind only (edges of owned cells [nEO, nERing), vertices of owned edges [nVO, nVRing)):
    // written there by a launcher that computes them too, wrote_ring1
    std::vector<uint8_t> stale;
    // per-peer packed buffers: [cell fields][edge fields][vertex fields] columns of LP doubles
    double* sendbuf = nullptr;
    double* recvbuf = nullptr;
    size_t cap = 0;  // doubles per buffer
    LoopGroup* loop = nullptr;
    RcclComm* rccl = nullptr;
    SockComm* sock = nullptr;
    bool stub = false;  // mpas_halo_stub: pack, a device copy for the wire, unpack
    // option "stub_latency_us": the stub's wire also waits this long on the device (a one-wave
    // kernel spinning on the wall clock), standing in for a transport's per-exchange latency
    int stub_latency_us = 0;
    // option "stub_refuse_capture" (test hook): the stub fails an exchange made inside a stream
    // capture, as a transport that cannot be captured does -- the graph fallback's test
    int stub_refuse_capture = 0;
    int wall_khz = 0;  // hipDeviceAttributeWallClockRate
    std::string err;
    int64_t exchanges = 0, fields_moved = 0;
    // overlap of the exchange with interior compute
    hipStream_t comm = nullptr;  // the halo stream
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
    int nint[3] = {0, 0, 0};  // interior cells, edges, vertices: the first owned ones
    bool interior = false;     // nint set (mpas_halo_interior)
    int overlap = 1;           // option "overlap"
    std::vector<int> overlapped;  // fields exchanged beside the last interior launch
    std::string race;             // set by wrote() when a kernel wrote one of them
    std::map<std::vector<int>, HaloCopyTab> tabs;  // pack / unpack tables per exchange signature
    // set when an exchange inside a stream capture needed a table not built yet: tables are
    // built and uploaded outside captures only, so that capture fails and the step runs
    // eagerly (mpas_ctx.cpp srk3_step)
    bool capture_miss = false;

    ~Halo();
    void clear_tabs();  // free every pack / unpack table (a plan change)
    hipError_t reserve(int LP);  // size the packed buffers for the largest exchange
    // make every field in `gathers` that is stale fresh on the ghosts
    hipError_t before(const DevState& S, hipStream_t st, std::initializer_list<int> gathers);
    void wrote(std::initializer_list<int> fields);
    // the fields were written on the owned entities and, identically to their owners, on the
    // ring-1 ghost edges: those stay fresh if they were (0 or 2 -> 2), else stale
    void wrote_ring1(std::initializer_list<int> fields);
    // the fields were written on the owned entities and on the ring-1 ghosts from inputs the
    // launch gathered fresh (a buffer a launcher fills anew, e.g. the fused damping's ru_p):
    // fresh on the ring-1 ghosts whatever they were before (state 2)
    void fresh_ring1(std::initializer_list<int> fields);
    hipError_t exchange(const DevState& S, hipStream_t st, const std::vector<int>& fields);
    // launch `fn` (a kernel launch over the entities of the DevState it is given) with the
    // stale fields of `gathers` exchanged first: interior / exchange / boundary when the
    // overlap is on, else exchange then one launch over every owned entity
    // `ring1`: fields of `gathers` the kernel reads on ring-1 ghost edges only (edges of
    // owned cells), for which stale state 2 counts as fresh
    hipError_t launch(const DevState& S, hipStream_t st, std::initializer_list<int> gathers,
                      const std::function<void(const DevState&)>& fn, std::initializer_list<int> ring1 = {});
};

// launchers: without a decomposition HALO_RUN is one call of FN over the owned entities
#define HALO_RUN(S, st, FN, ...)                                                           \
    do {                                                                                   \
        if ((S).halo) {                                                                    \
            hipError_t he_ = (S).halo->launch((S), (st), {__VA_ARGS__}, (FN));              \
            if (he_ != hipSuccess) return he_;                                             \
        } else {                                                                           \
            (FN)(S);                                                                       \
        }                                                                                  \
    } while (0)
#define HALO_WROTE(S, ...)                          \
    do {                                            \
        if ((S).halo) (S).halo->wrote({__VA_ARGS__}); \
    } while (0)
// HALO_RUN whose gathers of field R1 touch its ring-1 ghosts only (edges of owned cells,
// vertices of owned edges)
#define HALO_RUN_R1(S, st, FN, R1, ...)                                                    \
    do {                                                                                   \
        if ((S).halo) {                                                                    \
            hipError_t he_ = (S).halo->launch((S), (st), {__VA_ARGS__}, (FN), {R1});        \
            if (he_ != hipSuccess) return he_;                                             \
        } else {                                                                           \
            (FN)(S);                                                                       \
        }                                                                                  \
    } while (0)

// loopback group (one per process, N shards)
struct LoopGroup {
    int n = 0;
    std::vector<Halo*> members;
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> packed, copied;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t generation = 0;
    bool broken = false;
    bool barrier(double timeout_s);  // false on timeout (a shard stopped driving)
    ~LoopGroup() {
        for (auto e : packed) (void)hipEventDestroy(e);
        for (auto e : copied) (void)hipEventDestroy(e);
    }
};

// transports (mpas_halo.hip)
int rccl_unique_id(void* out128, std::string& err);
int rccl_init(Halo* h, int nranks, int rank, const void* id128, std::string& err);
void rccl_free(RcclComm* c);
int sock_init(Halo* h, int nranks, int rank, const char* host, int base_port, std::string& err);
void sock_free(SockComm* c);

}  // namespace mpas
