// gather.hip -- microbenchmark for the column-gather pattern of the dyn_tend cell
// kernels: each destination cell sums the 512-B columns (64 doubles) of its edges.
// Variants: lane = level with 8-B loads (one column per wave) vs two levels per lane
// with 16-B loads (two columns per wave), optional grouped XCD block order.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ int xcdmap(int G) {
    const int b = (int)blockIdx.x, nb = (int)gridDim.x;
    if (G <= 0) return b;
    const int W = G << 3;
    if (b >= (nb / W) * W) return b;
    const int w = b / W, r = b - w * W;
    return w * W + (r & 7) * G + (r >> 3);
}

template <int NG>
__global__ __launch_bounds__(256) void g8(const double* __restrict__ T, const int* __restrict__ idx, int nd,
                                          double* __restrict__ out, int G) {
    int d = xcdmap(G) * 4 + (int)(threadIdx.x >> 6);
    d = __builtin_amdgcn_readfirstlane(d);
    if (d >= nd) return;
    const int k = threadIdx.x & 63;
    double v[NG];
#pragma unroll
    for (int i = 0; i < NG; i++) v[i] = T[(size_t)idx[d * 10 + i] * 64 + k];
    double s = 0;
#pragma unroll
    for (int i = 0; i < NG; i++) s += v[i];
    out[(size_t)d * 64 + k] = s;
}

template <int NG>
__global__ __launch_bounds__(256) void g16(const double* __restrict__ T, const int* __restrict__ idx, int nd,
                                           double* __restrict__ out, int G) {
    // 32 lanes per column, lane holds levels 2j, 2j+1
    const int half = (threadIdx.x >> 5) & 1;
    int d0 = xcdmap(G) * 8 + (int)(threadIdx.x >> 6) * 2;
    d0 = __builtin_amdgcn_readfirstlane(d0);
    const int d = d0 + half;
    if (d0 >= nd) return;
    const int j = threadIdx.x & 31;
    const bool ok = d < nd;
    const int dd = ok ? d : d0;
    double2 v[NG];
#pragma unroll
    for (int i = 0; i < NG; i++) v[i] = *(const double2*)(T + (size_t)idx[dd * 10 + i] * 64 + 2 * j);
    double2 s = make_double2(0, 0);
#pragma unroll
    for (int i = 0; i < NG; i++) {
        s.x += v[i].x;
        s.y += v[i].y;
    }
    if (ok) *(double2*)(out + (size_t)d * 64 + 2 * j) = s;
}

// lane-masked gathers: only lanes k < W load (levels 0..W-1 of a 64-double column); do
// the idle lanes of a column's last 64-B chunk still cost request bandwidth?
template <int NG>
__global__ __launch_bounds__(256) void g8m(const double* __restrict__ T, const int* __restrict__ idx, int nd,
                                           double* __restrict__ out, int G, int W) {
    int d = xcdmap(G) * 4 + (int)(threadIdx.x >> 6);
    d = __builtin_amdgcn_readfirstlane(d);
    if (d >= nd) return;
    const int k = threadIdx.x & 63;
    double v[NG];
    int id[NG];
#pragma unroll
    for (int i = 0; i < NG; i++) id[i] = idx[d * 10 + i];
    if (k < W) {
#pragma unroll
        for (int i = 0; i < NG; i++) v[i] = T[(size_t)id[i] * 64 + k];
    } else {
#pragma unroll
        for (int i = 0; i < NG; i++) v[i] = 0.0;
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NG; i++) s += v[i];
    out[(size_t)d * 64 + k] = s;
}

extern "C" int ub_gather_masked(const double* T, const int* idx, int nd, double* out, int G, int W, void* stream) {
    g8m<10><<<(nd + 3) / 4, 256, 0, (hipStream_t)stream>>>(T, idx, nd, out, G, W);
    return (int)hipGetLastError();
}

// two fields gathered at the same ids: two 8-B loads per id from separate arrays vs one
// 16-B load from a pair-interleaved array (column = LP (a, b) pairs, 1 KB)
template <int NG>
__global__ __launch_bounds__(256) void g8two(const double* __restrict__ A, const double* __restrict__ B,
                                             const int* __restrict__ idx, int nd, double* __restrict__ out, int G) {
    int d = xcdmap(G) * 4 + (int)(threadIdx.x >> 6);
    d = __builtin_amdgcn_readfirstlane(d);
    if (d >= nd) return;
    const int k = threadIdx.x & 63;
    double a[NG], b[NG];
#pragma unroll
    for (int i = 0; i < NG; i++) {
        const size_t o = (size_t)idx[d * 10 + i] * 64 + k;
        a[i] = A[o];
        b[i] = B[o];
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NG; i++) s += a[i] * b[i];
    out[(size_t)d * 64 + k] = s;
}
template <int NG>
__global__ __launch_bounds__(256) void g16pair(const double2* __restrict__ AB, const int* __restrict__ idx, int nd,
                                               double* __restrict__ out, int G) {
    int d = xcdmap(G) * 4 + (int)(threadIdx.x >> 6);
    d = __builtin_amdgcn_readfirstlane(d);
    if (d >= nd) return;
    const int k = threadIdx.x & 63;
    double2 v[NG];
#pragma unroll
    for (int i = 0; i < NG; i++) v[i] = AB[(size_t)idx[d * 10 + i] * 64 + k];
    double s = 0;
#pragma unroll
    for (int i = 0; i < NG; i++) s += v[i].x * v[i].y;
    out[(size_t)d * 64 + k] = s;
}
extern "C" int ub_gather_two(int pair, const double* A, const double* B, const int* idx, int nd, double* out, int G,
                             void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (pair) g16pair<10><<<(nd + 3) / 4, 256, 0, st>>>((const double2*)A, idx, nd, out, G);
    else g8two<10><<<(nd + 3) / 4, 256, 0, st>>>(A, B, idx, nd, out, G);
    return (int)hipGetLastError();
}

// two columns per 16-B gather with a level-permuted column layout: position 2j holds
// level j, position 2j+1 level j+32.  Lanes 0-31 load pair j of column A, lanes 32-63
// pair j of column B; one permlane32_swap per dword puts A and B back in lane = level.
__device__ __forceinline__ void swap_halves(double& x, double& y) {
    // lanes 32-63 of x <-> lanes 0-31 of y
    int2 xi = *reinterpret_cast<int2*>(&x), yi = *reinterpret_cast<int2*>(&y);
    auto r0 = __builtin_amdgcn_permlane32_swap(xi.x, yi.x, false, false);
    auto r1 = __builtin_amdgcn_permlane32_swap(xi.y, yi.y, false, false);
    xi.x = r0[0]; yi.x = r0[1]; xi.y = r1[0]; yi.y = r1[1];
    x = *reinterpret_cast<double*>(&xi);
    y = *reinterpret_cast<double*>(&yi);
}
template <int NG>
__global__ __launch_bounds__(256) void g8swap(const double* __restrict__ T, const int* __restrict__ idx, int nd,
                                              double* __restrict__ out, int G) {
    int d = xcdmap(G) * 4 + (int)(threadIdx.x >> 6);
    d = __builtin_amdgcn_readfirstlane(d);
    if (d >= nd) return;
    const int k = threadIdx.x & 63;
    const int hi = k >> 5, j = k & 31;
    double v[NG];
#pragma unroll
    for (int i = 0; i < NG; i += 2) {
        const int ia = idx[d * 10 + i], ib = idx[d * 10 + i + 1];
        const int id = hi ? ib : ia;
        const double2 t = *(const double2*)(T + (size_t)id * 64 + 2 * j);
        double x = t.x, y = t.y;
        swap_halves(x, y);
        v[i] = x;
        v[i + 1] = y;
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NG; i++) s += v[i];
    out[(size_t)d * 64 + (j * 2 + hi)] = s;
}
extern "C" int ub_gather_swap(const double* T, const int* idx, int nd, double* out, int G, void* stream) {
    g8swap<10><<<(nd + 3) / 4, 256, 0, (hipStream_t)stream>>>(T, idx, nd, out, G);
    return (int)hipGetLastError();
}

extern "C" int ub_gather(int variant, const double* T, const int* idx, int nd, double* out, int G, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (variant == 0) g8<6><<<(nd + 3) / 4, 256, 0, st>>>(T, idx, nd, out, G);
    else if (variant == 1) g16<6><<<(nd + 7) / 8, 256, 0, st>>>(T, idx, nd, out, G);
    else if (variant == 2) g8<10><<<(nd + 3) / 4, 256, 0, st>>>(T, idx, nd, out, G);
    else if (variant == 3) g16<10><<<(nd + 7) / 8, 256, 0, st>>>(T, idx, nd, out, G);
    return (int)hipGetLastError();
}

// streaming: dst[row][k] = a[row][k] + b[row][k] for lanes k < W (W = 56, 57 or 64 of a
// 64-double row): does a write covering part of the last 64-B chunk of a row cost more?
__global__ __launch_bounds__(256) void s_add(const double* __restrict__ a, const double* __restrict__ b, int n,
                                             double* __restrict__ d, int W) {
    int r = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    r = __builtin_amdgcn_readfirstlane(r);
    if (r >= n) return;
    const int k = threadIdx.x & 63;
    double x = a[(size_t)r * 64 + k] + b[(size_t)r * 64 + k];
    if (k < W) d[(size_t)r * 64 + k] = x;
}
// the same with the level-pair layout's holes: mode 0 positions < 56 (contiguous), 1 the
// positions of levels < 56 (odd positions 49..63 skipped), 2 all but position 49, 3 all
__global__ __launch_bounds__(256) void s_addp(const double* __restrict__ a, const double* __restrict__ b, int n,
                                              double* __restrict__ d, int mode) {
    int r = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    r = __builtin_amdgcn_readfirstlane(r);
    if (r >= n) return;
    const int p = threadIdx.x & 63;
    const int lev = (p >> 1) | ((p & 1) << 5);
    double x = a[(size_t)r * 64 + p] + b[(size_t)r * 64 + p];
    bool w = mode == 0 ? p < 56 : mode == 1 ? lev < 56 : mode == 2 ? p != 49 : true;
    if (mode == 4) {  // position 49 keeps its value: read it back and write the full column
        if (p == 49) x = d[(size_t)r * 64 + p];
        w = true;
    }
    if (w) d[(size_t)r * 64 + p] = x;
}
extern "C" int ub_streamp(const double* a, const double* b, int n, double* d, int mode, void* stream) {
    s_addp<<<(n + 3) / 4, 256, 0, (hipStream_t)stream>>>(a, b, n, d, mode);
    return (int)hipGetLastError();
}
// streaming-ceiling variants, 16 B per lane, grid-stride over n doubles2:
// 0 copy a->d, 1 d = a + b, 2 = 1 with nontemporal stores, 3 = 0 with nontemporal
// stores, 4 read-only (a + b summed per thread, one store per thread block)
__global__ __launch_bounds__(256) void s_var(const double2* __restrict__ a, const double2* __restrict__ b, size_t n,
                                             double2* __restrict__ d, int mode) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    double acc = 0.0;
    for (; i < n; i += stride) {
        double2 x = a[i];
        if (mode == 0) d[i] = x;
        else if (mode == 3) { __builtin_nontemporal_store(x.x, &d[i].x); __builtin_nontemporal_store(x.y, &d[i].y); }
        else {
            const double2 y = b[i];
            x.x += y.x;
            x.y += y.y;
            if (mode == 1) d[i] = x;
            else if (mode == 2) { __builtin_nontemporal_store(x.x, &d[i].x); __builtin_nontemporal_store(x.y, &d[i].y); }
            else acc += x.x + x.y;
        }
    }
    if (mode == 4 && acc == 12345.678) d[0].x = acc;
}
extern "C" int ub_svar(const double* a, const double* b, long n2, double* d, int mode, int grid, void* stream) {
    s_var<<<grid, 256, 0, (hipStream_t)stream>>>((const double2*)a, (const double2*)b, (size_t)n2, (double2*)d, mode);
    return (int)hipGetLastError();
}
extern "C" int ub_stream(const double* a, const double* b, int n, double* d, int W, void* stream) {
    s_add<<<(n + 3) / 4, 256, 0, (hipStream_t)stream>>>(a, b, n, d, W);
    return (int)hipGetLastError();
}

// the same stream with 16-B lanes (two levels per lane, two rows per wavefront)
__global__ __launch_bounds__(256) void s_add16(const double* __restrict__ a, const double* __restrict__ b, int n,
                                               double* __restrict__ d) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // double2 index
    if (i >= (size_t)n * 32) return;
    const double2 x = ((const double2*)a)[i], y = ((const double2*)b)[i];
    ((double2*)d)[i] = make_double2(x.x + y.x, x.y + y.y);
}
extern "C" int ub_stream16(const double* a, const double* b, int n, double* d, void* stream) {
    s_add16<<<(n * 32 + 255) / 256, 256, 0, (hipStream_t)stream>>>(a, b, n, d);
    return (int)hipGetLastError();
}
// 8-B lanes, plain 1-D (no row structure): the streaming ceiling of dwordx2
__global__ __launch_bounds__(256) void s_add8(const double* __restrict__ a, const double* __restrict__ b, size_t n,
                                              double* __restrict__ d) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    d[i] = a[i] + b[i];
}
extern "C" int ub_stream8(const double* a, const double* b, int n, double* d, void* stream) {
    s_add8<<<((size_t)n * 64 + 255) / 256, 256, 0, (hipStream_t)stream>>>(a, b, (size_t)n * 64, d);
    return (int)hipGetLastError();
}
