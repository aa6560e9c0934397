// mpas_halo.hip -- halo exchange (see mpas_halo.h): pack/unpack kernels, staleness
// bookkeeping, RCCL, loopback and host-staged TCP transports.
#include "mpas_halo.h"

#include <cstdio>
#include <cstdlib>

#include <dlfcn.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <arpa/inet.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "mpas_dev.h"

namespace mpas {

// ------------------------------------------------------------------ pack / unpack
// One launch per direction and exchange, over the columns of every peer region: the
// segments (field component x peer's id list, contiguous in the buffer) are a device
// table built once per exchange signature (the fields moved) and cached -- a step repeats
// the same ~10 signatures -- and each wavefront copies whole columns, finding its
// segment by a wave-uniform binary search over the segment starts.
struct HaloSeg {
    double* f;        // field base (LP doubles per column)
    const int* ids;   // local entity ids
    long start;       // first buffer column of the segment
    int W, comp;      // columns per entity and the one this segment moves (x8 fields)
};

// the column address of every buffer column of a table (once per exchange signature: the
// segment search and the id lookup -- five or six dependent memory round trips -- leave the
// per-exchange copies, which then load one address per column)
__global__ __launch_bounds__(256) void k_halo_addr(const HaloSeg* seg, int nseg, long ncol, int LP, double** addr) {
    const long col = (long)blockIdx.x * 256 + threadIdx.x;
    if (col >= ncol) return;
    int lo = 0, hi = nseg - 1;  // the last segment starting at or before col
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (seg[mid].start <= col) lo = mid;
        else hi = mid - 1;
    }
    const HaloSeg& g = seg[lo];
    addr[col] = g.f + ((size_t)g.ids[col - g.start] * g.W + g.comp) * LP;
}

template <bool PACK>
__global__ __launch_bounds__(256) void k_halo_copy(double* const* addr, long ncol, int LP, double* buf) {
    const long col = (long)blockIdx.x * (256 / LP) + threadIdx.x / LP;
    const int k = (int)(threadIdx.x % LP);
    if (col >= ncol) return;
    double* f = addr[col] + k;
    double* b = buf + (size_t)col * LP + k;
    if (PACK) *b = *f;
    else *f = *b;
}

// the stub transport's modelled wire latency: one wave spins on the device wall clock
// (bounded: it leaves after `ticks` whatever happens)
__global__ __launch_bounds__(64) void k_halo_wait(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

static int kind_of_field(int f) {
    switch (kFields[f].kind) {
        case K_C3: case K_C3V: return HK_CELL;
        case K_E3: return HK_EDGE;
        case K_V3: return HK_VERTEX;
        default: return -1;
    }
}

static hipError_t tables_ready(const DevState& S, Halo& h, hipStream_t st, const std::vector<int>& fields);

void Halo::clear_tabs() {
    for (auto& kv : tabs) {
        if (kv.second.dev) (void)hipFree(kv.second.dev);
        if (kv.second.addr) (void)hipFree(kv.second.addr);
    }
    tabs.clear();
}

Halo::~Halo() {
    for (auto& v : peers)
        for (auto& p : v) {
            if (p.d_send) (void)hipFree(p.d_send);
            if (p.d_recv) (void)hipFree(p.d_recv);
        }
    if (sendbuf) (void)hipFree(sendbuf);
    if (recvbuf) (void)hipFree(recvbuf);
    clear_tabs();
    if (rccl) rccl_free(rccl);
    if (sock) sock_free(sock);
    if (comm) {
        (void)hipStreamSynchronize(comm);
        (void)hipStreamDestroy(comm);
    }
    if (ev_ready) (void)hipEventDestroy(ev_ready);
    if (ev_done) (void)hipEventDestroy(ev_done);
}

hipError_t Halo::reserve(int LP) {
    // the largest exchange moves every field of every kind at once
    long fk[3] = {0, 0, 0};
    for (int f = 0; f < X_COUNT; f++) {
        int k = kind_of_field(f);
        if (k >= 0) fk[k] += kFields[f].width;  // columns per entity
    }
    long s = 0, r = 0;
    for (int k = 0; k < 3; k++)
        for (const auto& p : peers[k]) {
            s += (long)p.nsend * fk[k];
            r += (long)p.nrecv * fk[k];
        }
    const size_t need = (size_t)std::max(std::max(s, r), 1L) * LP;
    if (need <= cap) return hipSuccess;
    if (sendbuf) (void)hipFree(sendbuf);
    if (recvbuf) (void)hipFree(recvbuf);
    sendbuf = recvbuf = nullptr;
    cap = 0;
    hipError_t e;
    if ((e = hipMalloc(&sendbuf, need * sizeof(double))) != hipSuccess) return e;
    if ((e = hipMalloc(&recvbuf, need * sizeof(double))) != hipSuccess) return e;
    cap = need;
    return hipSuccess;
}

void Halo::wrote_ring1(std::initializer_list<int> fields) {
    std::vector<uint8_t> was;
    for (int f : fields) was.push_back(stale[f]);
    wrote(fields);  // (the overlap race check)
    size_t i = 0;
    for (int f : fields) stale[f] = was[i++] == 1 ? 1 : 2;
}

void Halo::fresh_ring1(std::initializer_list<int> fields) {
    wrote(fields);  // (the overlap race check)
    for (int f : fields) stale[f] = 2;
}

void Halo::wrote(std::initializer_list<int> fields) {
    // Overlap safety: the interior launch of the kernel that just ran executed beside the
    // pack of `overlapped`.  If that kernel writes one of those fields, the pack may read
    // a half-updated column (send entities can be interior).  Flag it; run_task turns it
    // into an error of the task (every rank runs the same launcher sequence, so the
    // loopback tests catch a launcher that breaks the invariant).
    for (int f : fields) {
        for (int g : overlapped)
            if (g == f && race.empty())
                race = std::string("field ") + kFields[f].name +
                       " is written by a kernel whose interior launch overlapped its halo exchange";
        stale[f] = 1;
    }
    overlapped.clear();
}

hipError_t Halo::before(const DevState& S, hipStream_t st, std::initializer_list<int> gathers) {
    std::vector<int> need;
    for (int f : gathers)
        if (stale[f]) need.push_back(f);
    if (need.empty()) return hipSuccess;
    hipError_t e = exchange(S, st, need);
    if (e == hipSuccess)
        for (int f : need) stale[f] = 0;
    return e;
}

hipError_t Halo::launch(const DevState& S, hipStream_t st, std::initializer_list<int> gathers,
                        const std::function<void(const DevState&)>& fn, std::initializer_list<int> ring1) {
    std::vector<int> need;
    for (int f : gathers) {
        bool r1 = false;
        for (int g : ring1) r1 = r1 || g == f;
        if (stale[f] == 1 || (stale[f] == 2 && !r1)) need.push_back(f);
    }
    hipError_t e;
    overlapped.clear();
    if (need.empty()) {
        fn(S);
        return hipGetLastError();
    }
    if (!(overlap && interior && comm)) {  // the exchange on the critical path
        if ((e = exchange(S, st, need)) != hipSuccess) return e;
        for (int f : need) stale[f] = 0;
        fn(S);
        return hipGetLastError();
    }
    // (the pack / unpack tables first: nothing is forked if one cannot be built here)
    if ((e = tables_ready(S, *this, st, need)) != hipSuccess) return e;
    // the halo stream starts after everything the task stream holds (the stale values
    // were written there); the interior launch reads no ghost and writes no gathered
    // field, so it runs beside the pack / send / recv / unpack
    if ((e = hipEventRecord(ev_ready, st)) != hipSuccess) return e;
    overlapped = need;  // checked against the kernel's writes by wrote()
    DevState in = S;
    in.nCO = nint[0];
    in.nEO = nint[1];
    in.nVO = nint[2];
    in.interior = 1;
    fn(in);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(comm, ev_ready, 0)) != hipSuccess) return e;
    if ((e = exchange(S, comm, need)) != hipSuccess) {
        // the halo stream was forked from the task stream: join it back before failing, so
        // that a stream capture in progress stays joined and can be ended
        (void)hipEventRecord(ev_done, comm);
        (void)hipStreamWaitEvent(st, ev_done, 0);
        overlapped.clear();
        return e;
    }
    for (int f : need) stale[f] = 0;
    if ((e = hipEventRecord(ev_done, comm)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(st, ev_done, 0)) != hipSuccess) return e;
    DevState bd = S;
    bd.lo[0] = nint[0];
    bd.lo[1] = nint[1];
    bd.lo[2] = nint[2];
    fn(bd);
    return hipGetLastError();
}

// ------------------------------------------------------------------ RCCL (dlopen)
struct Uid128 {
    char b[128];
};
struct RcclApi {
    void* h = nullptr;
    int (*GetUniqueId)(Uid128*) = nullptr;
    int (*CommInitRank)(void**, int, Uid128, int) = nullptr;
    int (*CommDestroy)(void*) = nullptr;
    int (*GroupStart)() = nullptr;
    int (*GroupEnd)() = nullptr;
    int (*Send)(const void*, size_t, int, int, void*, hipStream_t) = nullptr;
    int (*Recv)(void*, size_t, int, int, void*, hipStream_t) = nullptr;
    const char* (*GetErrorString)(int) = nullptr;
};
constexpr int kNcclFloat64 = 8;  // ncclDouble in rccl.h's ncclDataType_t

static RcclApi* rccl_api(std::string& err) {
    static RcclApi api;
    static bool tried = false;
    if (!tried) {
        tried = true;
        // share the RCCL already in the process (torch.distributed), else load ROCm's
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (h) {
            api.h = h;
            api.GetUniqueId = (int (*)(Uid128*))dlsym(h, "ncclGetUniqueId");
            api.CommInitRank = (int (*)(void**, int, Uid128, int))dlsym(h, "ncclCommInitRank");
            api.CommDestroy = (int (*)(void*))dlsym(h, "ncclCommDestroy");
            api.GroupStart = (int (*)())dlsym(h, "ncclGroupStart");
            api.GroupEnd = (int (*)())dlsym(h, "ncclGroupEnd");
            api.Send = (int (*)(const void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclSend");
            api.Recv = (int (*)(void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclRecv");
            api.GetErrorString = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
        }
    }
    if (!api.h || !api.GetUniqueId || !api.CommInitRank || !api.GroupStart || !api.GroupEnd || !api.Send ||
        !api.Recv) {
        err = "librccl.so.1 not loadable or incomplete";
        return nullptr;
    }
    return &api;
}

struct RcclComm {
    void* comm = nullptr;
    ~RcclComm() {
        std::string e;
        RcclApi* a = rccl_api(e);
        if (a && comm && a->CommDestroy) a->CommDestroy(comm);
    }
};

int rccl_unique_id(void* out128, std::string& err) {
    RcclApi* a = rccl_api(err);
    if (!a) return -1;
    int r = a->GetUniqueId((Uid128*)out128);
    if (r != 0) {
        err = std::string("ncclGetUniqueId: ") + (a->GetErrorString ? a->GetErrorString(r) : "error");
        return -1;
    }
    return 0;
}

int rccl_init(Halo* h, int nranks, int rank, const void* id128, std::string& err) {
    RcclApi* a = rccl_api(err);
    if (!a) return -1;
    Uid128 id;
    std::memcpy(id.b, id128, 128);
    auto* c = new RcclComm();
    int r = a->CommInitRank(&c->comm, nranks, id, rank);
    if (r != 0) {
        err = std::string("ncclCommInitRank: ") + (a->GetErrorString ? a->GetErrorString(r) : "error");
        delete c;
        return -1;
    }
    h->rccl = c;
    h->nranks = nranks;
    h->rank = rank;
    return 0;
}
void rccl_free(RcclComm* c) { delete c; }

// ------------------------------------------------------------------ TCP (host-staged)
// Rank r listens on base_port + r; for every pair i < j, j connects to i and sends its rank.
// Each exchange moves, per peer in increasing rank order, an 8-byte byte count and the
// packed region: the lower rank of a pair sends first, the higher receives first (a
// total order of pairwise exchanges: no cycle of blocked senders).  Sockets time out after
// 120 s, so a plan mismatch or a dead peer fails the call instead of hanging it.
struct SockComm {
    int nranks = 0, rank = 0;
    std::vector<int> fd;  // per peer rank (-1: self)
    std::vector<double> hsend, hrecv;
    ~SockComm() {
        for (int f : fd)
            if (f >= 0) ::close(f);
    }
};
void sock_free(SockComm* c) { delete c; }

static bool sock_all(int fd, void* p, size_t n, bool snd) {
    char* b = (char*)p;
    while (n) {
        const ssize_t k = snd ? ::send(fd, b, n, MSG_NOSIGNAL) : ::recv(fd, b, n, 0);
        if (k <= 0) return false;
        b += k;
        n -= (size_t)k;
    }
    return true;
}
static void sock_opts(int fd) {
    timeval tv{120, 0};
    (void)setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    (void)setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    int one = 1;
    (void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

int sock_init(Halo* h, int nranks, int rank, const char* host, int base_port, std::string& err) {
    auto* c = new SockComm();
    c->nranks = nranks;
    c->rank = rank;
    c->fd.assign(nranks, -1);
    auto fail = [&](const std::string& m) {
        err = m;
        delete c;
        return -1;
    };
    sockaddr_in a{};
    a.sin_family = AF_INET;
    if (inet_pton(AF_INET, host, &a.sin_addr) != 1) return fail(std::string("socket halo: bad host ") + host);
    const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return fail("socket halo: socket()");
    int one = 1;
    (void)setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in me = a;
    me.sin_port = htons((uint16_t)(base_port + rank));
    if (::bind(ls, (sockaddr*)&me, sizeof(me)) != 0 || ::listen(ls, nranks) != 0) {
        ::close(ls);
        return fail("socket halo: bind/listen on port " + std::to_string(base_port + rank));
    }
    // connect to every lower rank (retrying while it starts), then accept the higher ones
    for (int p = 0; p < rank; p++) {
        sockaddr_in to = a;
        to.sin_port = htons((uint16_t)(base_port + p));
        int fd = -1;
        for (int t = 0; t < 1200 && fd < 0; t++) {  // up to 120 s
            fd = ::socket(AF_INET, SOCK_STREAM, 0);
            if (fd >= 0 && ::connect(fd, (sockaddr*)&to, sizeof(to)) != 0) {
                ::close(fd);
                fd = -1;
            }
            if (fd < 0) usleep(100000);
        }
        if (fd < 0) {
            ::close(ls);
            return fail("socket halo: cannot reach rank " + std::to_string(p));
        }
        sock_opts(fd);
        int32_t me32 = rank;
        if (!sock_all(fd, &me32, 4, true)) {
            ::close(fd);
            ::close(ls);
            return fail("socket halo: hello to rank " + std::to_string(p));
        }
        c->fd[p] = fd;
    }
    timeval tv{120, 0};
    (void)setsockopt(ls, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    for (int n = rank + 1; n < nranks; n++) {
        const int fd = ::accept(ls, nullptr, nullptr);
        int32_t who = -1;
        if (fd < 0) {
            ::close(ls);
            return fail("socket halo: accept timed out");
        }
        sock_opts(fd);
        if (!sock_all(fd, &who, 4, false) || who <= rank || who >= nranks || c->fd[who] >= 0) {
            ::close(fd);
            ::close(ls);
            return fail("socket halo: bad hello");
        }
        c->fd[who] = fd;
    }
    ::close(ls);
    h->sock = c;
    h->nranks = nranks;
    h->rank = rank;
    return 0;
}

// ------------------------------------------------------------------ loopback barrier
bool LoopGroup::barrier(double timeout_s) {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const int64_t gen = generation;
    if (++arrived == n) {
        arrived = 0;
        generation++;
        cv.notify_all();
        return true;
    }
    bool ok = cv.wait_for(lk, std::chrono::duration<double>(timeout_s), [&] { return generation != gen || broken; });
    if (!ok || broken) {
        broken = true;
        cv.notify_all();
        return false;
    }
    return true;
}

// ------------------------------------------------------------------ exchange
// per-peer packed regions, identical order on both sides: cells, edges, vertices; in
// each kind the fields in the order of `fields` (the same on every rank: the stale sets
// evolve identically because every rank runs the same task sequence)
struct Region {
    int peer;
    long soff, scols, roff, rcols;  // columns
};

static void plan_regions(const Halo& h, const std::vector<int>& fields, std::vector<Region>& reg,
                         std::vector<int> (&byk)[3]) {
    for (auto& v : byk) v.clear();
    for (int f : fields) {
        int k = kind_of_field(f);
        if (k >= 0) byk[k].push_back(f);
    }
    reg.clear();
    for (int k = 0; k < 3; k++)
        for (const auto& p : h.peers[k]) {
            Region* r = nullptr;
            for (auto& x : reg)
                if (x.peer == p.peer) r = &x;
            if (!r) {
                reg.push_back({p.peer, 0, 0, 0, 0});
                r = &reg.back();
            }
            long w = 0;  // columns per entity of the kind's fields
            for (int f : byk[k]) w += kFields[f].width;
            r->scols += (long)p.nsend * w;
            r->rcols += (long)p.nrecv * w;
        }
    long so = 0, ro = 0;
    for (auto& r : reg) {
        r.soff = so;
        r.roff = ro;
        so += r.scols;
        ro += r.rcols;
    }
}

// the segment table of one direction of an exchange (cached per signature)
static const HaloCopyTab* copy_table(const DevState& S, Halo& h, const std::vector<Region>& reg,
                                     const std::vector<int> (&byk)[3], const std::vector<int>& fields, bool pack,
                                     hipStream_t st, hipError_t& e) {
    std::vector<int> key(fields);
    key.push_back(pack ? 1 : 0);
    for (int f : fields) {  // (the fields' buffers: atm_srk3's fused damping swaps two pairs of them)
        const uint64_t a = (uint64_t)(uintptr_t)S.f[f];
        key.push_back((int)(uint32_t)a);
        key.push_back((int)(uint32_t)(a >> 32));
    }
    auto it = h.tabs.find(key);
    if (it != h.tabs.end()) return &it->second;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) {  // (no allocation or upload inside a capture)
        h.capture_miss = true;
        h.err = "halo pack table built inside a graph capture";
        e = hipErrorInvalidValue;
        return nullptr;
    }
    HaloCopyTab t;
    std::vector<HaloSeg> segs;
    for (const auto& r : reg) {
        long col = pack ? r.soff : r.roff;
        for (int k = 0; k < 3; k++) {
            const HaloPeer* p = nullptr;
            for (const auto& x : h.peers[k])
                if (x.peer == r.peer) p = &x;
            if (!p) continue;
            const int n = pack ? p->nsend : p->nrecv;
            if (n == 0) continue;
            for (int f : byk[k])
                for (int comp = 0; comp < kFields[f].width; comp++) {
                    segs.push_back({(double*)S.f[f], pack ? p->d_send : p->d_recv, col, kFields[f].width, comp});
                    col += n;
                }
        }
        t.ncol = std::max(t.ncol, col);
    }
    t.nseg = (int)segs.size();
    t.host = std::make_shared<std::vector<HaloSeg>>(segs);
    e = hipSuccess;
    if (t.nseg) {
        if ((e = hipMalloc(&t.dev, sizeof(HaloSeg) * segs.size())) != hipSuccess) return nullptr;
        if ((e = hipMemcpy(t.dev, t.host->data(), sizeof(HaloSeg) * segs.size(), hipMemcpyHostToDevice)) != hipSuccess ||
            (t.ncol && (e = hipMalloc(&t.addr, sizeof(double*) * t.ncol)) != hipSuccess)) {
            (void)hipFree(t.dev);
            return nullptr;
        }
        if (t.ncol) {  // (stream-ordered before every copy that uses the table)
            k_halo_addr<<<(unsigned)((t.ncol + 255) / 256), 256, 0, st>>>(t.dev, t.nseg, t.ncol, S.LP, t.addr);
            if ((e = hipGetLastError()) != hipSuccess) {
                (void)hipFree(t.dev);
                (void)hipFree(t.addr);
                return nullptr;
            }
        }
    }
    return &(h.tabs[key] = t);
}

static hipError_t run_copy(const DevState& S, hipStream_t st, Halo& h, const std::vector<Region>& reg,
                           const std::vector<int> (&byk)[3], const std::vector<int>& fields, bool pack) {
    hipError_t e = hipSuccess;
    const HaloCopyTab* t = copy_table(S, h, reg, byk, fields, pack, st, e);
    if (!t) return e;
    if (!t->nseg || !t->ncol) return hipSuccess;
    const int cpb = 256 / S.LP;
    const unsigned grid = (unsigned)((t->ncol + cpb - 1) / cpb);
    double* buf = pack ? h.sendbuf : h.recvbuf;
    if (pack) k_halo_copy<true><<<grid, 256, 0, st>>>(t->addr, t->ncol, S.LP, buf);
    else k_halo_copy<false><<<grid, 256, 0, st>>>(t->addr, t->ncol, S.LP, buf);
    return hipGetLastError();
}

// both tables of an exchange of `fields` built (outside a capture) or found; inside a capture
// a missing one fails the call before anything is enqueued (capture_miss)
static hipError_t tables_ready(const DevState& S, Halo& h, hipStream_t st, const std::vector<int>& fields) {
    std::vector<Region> reg;
    std::vector<int> byk[3];
    plan_regions(h, fields, reg, byk);
    hipError_t e = hipSuccess;
    for (bool pack : {true, false})
        if (!copy_table(S, h, reg, byk, fields, pack, st, e)) return e;
    return hipSuccess;
}

hipError_t Halo::exchange(const DevState& S, hipStream_t st, const std::vector<int>& fields) {
    hipError_t e0 = tables_ready(S, *this, st, fields);
    if (e0 != hipSuccess) return e0;
    std::vector<Region> reg;
    std::vector<int> byk[3];
    plan_regions(*this, fields, reg, byk);
    long stot = 0, rtot = 0;
    for (auto& r : reg) {
        stot += r.scols;
        rtot += r.rcols;
    }
    const size_t need = (size_t)std::max(stot, rtot) * S.LP;
    if (need > cap) {  // reserve() sized the buffers for every halo field at once
        err = "halo buffers too small";
        return hipErrorInvalidValue;
    }
    exchanges++;
    fields_moved += (int64_t)fields.size();
    static const bool log = [] {  // MPAS_HALO_LOG=1: one stderr line per exchange (rank 0)
        const char* v = std::getenv("MPAS_HALO_LOG");
        return v && *v && *v != '0';
    }();
    if (log && rank == 0) {
        std::string names;
        for (int f : fields) names += std::string(" ") + kFields[f].name;
        fprintf(stderr, "halo exchange %lld:%s\n", (long long)exchanges, names.c_str());
    }
    hipError_t e;
    if (loop) {
        // reuse of our send buffer: every peer's copies of the previous exchange are done
        for (int s = 0; s < loop->n; s++)
            if (s != rank && (e = hipStreamWaitEvent(st, loop->copied[s], 0)) != hipSuccess) return e;
    }
    if ((e = run_copy(S, st, *this, reg, byk, fields, true)) != hipSuccess) return e;
    if (rccl) {
        std::string dummy;
        RcclApi* a = rccl_api(dummy);
        int r = a->GroupStart();
        for (auto& x : reg) {
            if (r == 0 && x.scols) r = a->Send(sendbuf + x.soff * S.LP, (size_t)x.scols * S.LP, kNcclFloat64, x.peer, rccl->comm, st);
            if (r == 0 && x.rcols) r = a->Recv(recvbuf + x.roff * S.LP, (size_t)x.rcols * S.LP, kNcclFloat64, x.peer, rccl->comm, st);
        }
        int r2 = a->GroupEnd();
        if (r != 0 || r2 != 0) {
            err = std::string("RCCL halo exchange: ") + (a->GetErrorString ? a->GetErrorString(r ? r : r2) : "error");
            return hipErrorUnknown;
        }
    } else if (sock) {  // host-staged: the packed buffer down, the regions over TCP, back up
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        (void)hipStreamIsCapturing(st, &cs);
        if (cs != hipStreamCaptureStatusNone) {
            err = "socket halo transport inside a graph capture";
            return hipErrorInvalidValue;
        }
        SockComm& c = *sock;
        const size_t sn = (size_t)stot * S.LP, rn = (size_t)rtot * S.LP;
        if (c.hsend.size() < sn) c.hsend.resize(sn);
        if (c.hrecv.size() < rn) c.hrecv.resize(rn);
        if (sn && (e = hipMemcpyAsync(c.hsend.data(), sendbuf, sn * sizeof(double), hipMemcpyDeviceToHost, st)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        std::vector<const Region*> order;
        for (auto& x : reg) order.push_back(&x);
        std::sort(order.begin(), order.end(), [](const Region* a, const Region* b) { return a->peer < b->peer; });
        for (const Region* x : order) {
            const int fd = c.fd[x->peer];
            const uint64_t nb = (uint64_t)x->scols * S.LP * sizeof(double);
            const uint64_t want = (uint64_t)x->rcols * S.LP * sizeof(double);
            uint64_t got = 0;
            bool header = false;  // the peer's byte count arrived
            auto snd = [&] {
                return sock_all(fd, (void*)&nb, 8, true) && sock_all(fd, c.hsend.data() + x->soff * S.LP, nb, true);
            };
            auto rcv = [&] {
                if (!sock_all(fd, &got, 8, false)) return false;
                header = true;
                if (got != want) return false;
                return sock_all(fd, c.hrecv.data() + x->roff * S.LP, want, false);
            };
            const bool ok = rank < x->peer ? (snd() && rcv()) : (rcv() && snd());
            if (!ok) {  // a plan mismatch only when the header came and disagrees; else the transport failed
                err = "socket halo exchange with rank " + std::to_string(x->peer) +
                      (header && got != want
                           ? " (plan mismatch: " + std::to_string(got) + " bytes for " + std::to_string(want) + ")"
                           : " (transport failure: peer closed, timed out or unreachable)");
                return hipErrorUnknown;
            }
        }
        if (rn && (e = hipMemcpyAsync(recvbuf, c.hrecv.data(), rn * sizeof(double), hipMemcpyHostToDevice, st)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;  // (hrecv is reused by the next exchange)
    } else if (stub) {  // the received bytes land from the send buffer (no peer)
        if (stub_refuse_capture) {  // test hook: a transport that cannot be captured
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            (void)hipStreamIsCapturing(st, &cs);
            if (cs != hipStreamCaptureStatusNone) {
                err = "stub halo transport refuses the capture (option stub_refuse_capture)";
                return hipErrorInvalidValue;
            }
        }
        const size_t n = (size_t)std::min(stot, rtot) * S.LP;
        if (n && (e = hipMemcpyAsync(recvbuf, sendbuf, n * sizeof(double), hipMemcpyDeviceToDevice, st)) != hipSuccess)
            return e;
        if (stub_latency_us > 0) {
            if (!wall_khz) {
                int dev = 0;
                (void)hipGetDevice(&dev);
                if ((e = hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, dev)) != hipSuccess) return e;
            }
            k_halo_wait<<<1, 64, 0, st>>>((long long)stub_latency_us * wall_khz / 1000);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
    } else if (loop) {
        if ((e = hipEventRecord(loop->packed[rank], st)) != hipSuccess) return e;
        if (!loop->barrier(120.0)) {
            err = "loopback barrier timed out";
            return hipErrorUnknown;
        }
        for (auto& x : reg) {
            if (!x.rcols) continue;
            Halo* ph = loop->members[x.peer];
            // the peer packed its region for us with the same layout rule
            std::vector<Region> preg;
            std::vector<int> pbyk[3];
            plan_regions(*ph, fields, preg, pbyk);
            const Region* pr = nullptr;
            for (auto& y : preg)
                if (y.peer == rank) pr = &y;
            if (!pr || pr->scols != x.rcols) {
                err = "loopback halo plan mismatch";
                return hipErrorInvalidValue;
            }
            if ((e = hipStreamWaitEvent(st, loop->packed[x.peer], 0)) != hipSuccess) return e;
            if ((e = hipMemcpyAsync(recvbuf + x.roff * S.LP, ph->sendbuf + pr->soff * S.LP,
                                    (size_t)x.rcols * S.LP * sizeof(double), hipMemcpyDeviceToDevice, st)) != hipSuccess)
                return e;
        }
        if ((e = hipEventRecord(loop->copied[rank], st)) != hipSuccess) return e;
        if (!loop->barrier(120.0)) {
            err = "loopback barrier timed out";
            return hipErrorUnknown;
        }
    }
    return run_copy(S, st, *this, reg, byk, fields, false);
}

}  // namespace mpas
