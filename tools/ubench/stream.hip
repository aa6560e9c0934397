// stream.hip -- HBM streaming ceiling on the allocation sizes of the benchmark workload
// (VERDICT r02 item 7).  x1.163842 x 56 levels in the library's layout: one cell field is
// (nCells + 1) * 64 doubles = 84 MB, one edge field (nEdges + 1) * 64 doubles = 252 MB.
// Kernels: 16 B per lane (double2), grid-stride, 256-thread blocks, enough blocks to fill
// the chip; arrays staggered by 2 KB like mpas_ctx.cpp's allocations.
//   copy   1 read + 1 write stream            (setup / finish copies)
//   multi  R read streams + W write streams   (vert_imp: 10 + 9; set_smlstep-like 13 + 1)
//   read   1 read stream (sum kept live)      write  1 write stream
// Each case: 3 warm-up launches, then 20 timed launches (HIP events), median reported as
// GB/s of the bytes the kernel must move (each array read / written once).
// build: hipcc --offload-arch=gfx950 -O3 -o stream stream.hip   (tools/ubench/stream.sh)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr int kMaxArr = 24;
struct Arrs {
    const double2* r[kMaxArr];
    double2* w[kMaxArr];
    int nr, nw;
};

__global__ __launch_bounds__(256) void k_multi(Arrs a, size_t n2, double2* sink) {
    double2 acc = make_double2(0.0, 0.0);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        double2 s = make_double2(0.0, 0.0);
#pragma unroll 4
        for (int j = 0; j < a.nr; j++) {
            const double2 v = a.r[j][i];
            s.x += v.x;
            s.y += v.y;
        }
        for (int j = 0; j < a.nw; j++) a.w[j][i] = make_double2(s.x + j, s.y);
        acc.x += s.x;
    }
    if (a.nw == 0 && acc.x == 1.2345e300) *sink = acc;  // keeps read-only loads live
}

int main(int argc, char** argv) {
    const size_t nC = 163842 + 1, nE = 491520 + 1, LP = 64;
    int dev = 0;
    CK(hipSetDevice(dev));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, dev));
    const int grid = prop.multiProcessorCount * 16;
    struct Case {
        const char* name;
        size_t rows;
        int nr, nw;
    };
    std::vector<Case> cases = {
        {"copy_cell_84MB", nC, 1, 1},   {"copy_edge_252MB", nE, 1, 1},  {"read_cell", nC, 1, 0},
        {"read_edge", nE, 1, 0},        {"write_cell", nC, 0, 1},       {"write_edge", nE, 0, 1},
        {"multi_cell_10r_9w", nC, 10, 9}, {"multi_cell_13r_1w", nC, 13, 1}, {"multi_cell_6r_7w", nC, 6, 7},
    };
    std::vector<void*> raw;
    const size_t maxb = nE * LP * 8 + 16 * 2048;
    for (int i = 0; i < kMaxArr * 2; i++) {
        void* p;
        CK(hipMalloc(&p, maxb));
        CK(hipMemset(p, 0, maxb));
        raw.push_back(p);
    }
    double2* sink;
    CK(hipMalloc(&sink, 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\"device\": \"%s\", \"cus\": %d, \"grid\": %d, \"cases\": [", prop.gcnArchName, prop.multiProcessorCount,
           grid);
    for (size_t ci = 0; ci < cases.size(); ci++) {
        const Case& c = cases[ci];
        const size_t bytes1 = c.rows * LP * 8, n2 = bytes1 / 16;
        Arrs a{};
        a.nr = c.nr;
        a.nw = c.nw;
        for (int j = 0; j < c.nr; j++) a.r[j] = (const double2*)((char*)raw[j] + (j % 16) * 2048);
        for (int j = 0; j < c.nw; j++) a.w[j] = (double2*)((char*)raw[kMaxArr + j] + ((c.nr + j) % 16) * 2048);
        std::vector<float> ms;
        for (int it = 0; it < 23; it++) {
            CK(hipEventRecord(e0, 0));
            k_multi<<<grid, 256>>>(a, n2, sink);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (it >= 3) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        const double gb = (double)bytes1 * (c.nr + c.nw) / 1e9;
        printf("%s{\"case\": \"%s\", \"array_MB\": %.1f, \"reads\": %d, \"writes\": %d, \"ms\": %.4f, \"GBs\": %.1f, "
               "\"frac_of_8TBs\": %.3f}",
               ci ? ", " : "", c.name, bytes1 / 1e6, c.nr, c.nw, med, gb / (med * 1e-3), gb / (med * 1e-3) / 8000.0);
    }
    printf("]}\n");
    return 0;
}
