// pitch.hip -- microbenchmark for VERDICT r04 item 2: the level pitch of a column.
//
// The library stores a column of L+1 = 57 levels in LP = 64 slots, levels paired for 16-B
// loads (position 2j = level j, 2j+1 = level j+32).  A packed pitch P = 58 keeps the pairing
// of the levels that have a partner (j < NP = L+1-32: positions 2j, 2j+1) and stores the
// levels NP..31 that have none singly after them (position NP + j): one 16-B load per lane
// still brings lane j its level(s), the single lanes read one element of slack.  Stores: a
// 16-B store for the paired lanes, an 8-B store for the single ones.
//
// Kernels (one wavefront per column, lane = level after the permlane32 swap):
//   stream<P>  NIN input fields read at the own column (two fields per load), NOUT written
//              (two per store): the shape of the column-local tasks (setup, vert_imp, finish,
//              the acoustic step's own columns)
//   gath<P>    per edge NG gathered columns of two fields at the edgesOnEdge ids (two ids per
//              load, the gather2s of dyn_tend B) + the own column written: B's q gather
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ void swap_halves(double& x, double& y) {
    int2 xi = *reinterpret_cast<int2*>(&x), yi = *reinterpret_cast<int2*>(&y);
    auto r0 = __builtin_amdgcn_permlane32_swap(xi.x, yi.x, false, false);
    auto r1 = __builtin_amdgcn_permlane32_swap(xi.y, yi.y, false, false);
    xi.x = r0[0];
    yi.x = r0[1];
    xi.y = r1[0];
    yi.y = r1[1];
    x = *reinterpret_cast<double*>(&xi);
    y = *reinterpret_cast<double*>(&yi);
}

// element offset of lane j's 16-B load within a column (j = lane & 31)
template <int P>
__device__ __forceinline__ int poff(int j, int NP) {
    return P == 64 ? 2 * j : (j < NP ? 2 * j : NP + j);
}

// ALN (P = 58 only): the single lanes load the 16-B-aligned pair that holds their level and
// select it (two v_cndmask), instead of one 8-B-aligned (unaligned) 16-B load
template <int P, bool ALN = false>
__device__ __forceinline__ void ld2(const double* fa, int ca, const double* fb, int cb, int NP, double& a, double& b) {
    const int l = threadIdx.x & 63, j = l & 31;
    const double* base = l < 32 ? fa + (size_t)ca * P : fb + (size_t)cb * P;
    const int o = poff<P>(j, NP);
    double2 v = *(const double2*)(base + (ALN ? (o & ~1) : o));
    a = v.x;
    b = v.y;
    if (ALN && P != 64) a = (o & 1) ? v.y : v.x;
    swap_halves(a, b);
}

// HOLE (P = 64): the level-L slot (level NP - 1 + 32 = L, in pair NP - 1) is not written
// -- the library's stores of the fields whose level L the reference never writes: that
// lane stores its 8-B level NP - 1 only, so the column's last line is written partially.
// HOLE0: level 0 (pair 0) not written either (vert_imp's tridiagonal coefficients)
template <int P, bool HOLE = false, bool HOLE0 = false>
__device__ __forceinline__ void st2(double* fa, int ca, double* fb, int cb, int NP, double a, double b) {
    const int l = threadIdx.x & 63, j = l & 31;
    swap_halves(a, b);  // back to the pair layout
    double* base = l < 32 ? fa + (size_t)ca * P : fb + (size_t)cb * P;
    if (HOLE && j == NP - 1) {
        base[2 * j] = a;
    } else if (HOLE0 && j == 0) {
        base[1] = b;
    } else if (P == 64 || j < NP) {
        *(double2*)(base + 2 * j) = make_double2(a, b);
    } else if (j < 32) {
        base[NP + j] = a;  // (the partner level j+32 > L does not exist)
    }
}

template <int P, int NIN, int NOUT, bool ALN, bool HOLE = false, bool HOLE0 = false>
__global__ __launch_bounds__(256) void kstream(const double* const* in, double* const* out, int n, int NP) {
    const int c = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (c >= n) return;
    double v[NIN];
#pragma unroll
    for (int i = 0; i < NIN; i += 2) ld2<P, ALN>(in[i], c, in[i + 1], c, NP, v[i], v[i + 1]);
    double s = 0.0, t = 1.0;
#pragma unroll
    for (int i = 0; i < NIN; i++) {
        s += v[i];
        t += 0.5 * v[i];
    }
#pragma unroll
    for (int o = 0; o < NOUT; o += 2) st2<P, HOLE, HOLE0>(out[o], c, out[o + 1], c, NP, s + o, t - o);
}

template <int P, int NG, bool ALN>
__global__ __launch_bounds__(256) void gath(const double* u, const double* pv, const int* eoe, double* out, int n,
                                            int NP) {
    const int e = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (e >= n) return;
    int id[NG];
#pragma unroll
    for (int i = 0; i < NG; i++) id[i] = __builtin_amdgcn_readfirstlane(eoe[(size_t)e * 10 + i]);
    double a[NG], b[NG];
#pragma unroll
    for (int i = 0; i < NG; i += 2) {
        ld2<P, ALN>(u, id[i], u, id[i + 1], NP, a[i], a[i + 1]);
        ld2<P, ALN>(pv, id[i], pv, id[i + 1], NP, b[i], b[i + 1]);
    }
    double s = 0.0, t = 0.0;
#pragma unroll
    for (int i = 0; i < NG; i++) {
        s += a[i] * b[i];
        t += a[i];
    }
    st2<P>(out, e, out + (size_t)(n + 1) * P, e, NP, s, t);
}

extern "C" int ub_stream(int P, int nin, const double* const* in, double* const* out, int n, int NP, void* stream) {
    // P: 64, 58 (unaligned single-lane loads) or 59 (= 58 with the aligned-select loads)
    hipStream_t st = (hipStream_t)stream;
    const int nb = (n + 3) / 4;
    if (P == 64 && nin == 12) kstream<64, 12, 2, false><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 58 && nin == 12) kstream<58, 12, 2, false><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 59 && nin == 12) kstream<58, 12, 2, true><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 64 && nin == 4) kstream<64, 4, 4, false><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 58 && nin == 4) kstream<58, 4, 4, false><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 59 && nin == 4) kstream<58, 4, 4, true><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 65 && nin == 12) kstream<64, 12, 2, false, true><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 65 && nin == 4) kstream<64, 4, 4, false, true><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 66 && nin == 12) kstream<64, 12, 2, false, true, true><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 66 && nin == 4) kstream<64, 4, 4, false, true, true><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 65 && nin == 10) kstream<64, 10, 10, false, true><<<nb, 256, 0, st>>>(in, out, n, NP);
    else if (P == 64 && nin == 10) kstream<64, 10, 10, false><<<nb, 256, 0, st>>>(in, out, n, NP);
    else return -1;
    return (int)hipGetLastError();
}

extern "C" int ub_gath(int P, const double* u, const double* pv, const int* eoe, double* out, int n, int NP,
                       void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int nb = (n + 3) / 4;
    if (P == 64) gath<64, 10, false><<<nb, 256, 0, st>>>(u, pv, eoe, out, n, NP);
    else if (P == 58) gath<58, 10, false><<<nb, 256, 0, st>>>(u, pv, eoe, out, n, NP);
    else if (P == 59) gath<58, 10, true><<<nb, 256, 0, st>>>(u, pv, eoe, out, n, NP);
    else return -1;
    return (int)hipGetLastError();
}
