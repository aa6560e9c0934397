// qstage.hip -- microbenchmark for the edgesOnEdge gather of dyn_tend's edge kernel
// (the q term, dynamics_tasks.rg:993-1001): q(e,k) = sum_j w(e,j) u(eoe_j,k) * 0.5 (pv(e,k) + pv(eoe_j,k)).
// Variants:
//   0  one wavefront per edge, 256-thread blocks (today's k_dyn_B form)
//   1  one wavefront per edge, 1024-thread blocks (16 adjacent edges per CU at once)
//   2  256-thread blocks, each wave loops over Q edges, the 4 waves on adjacent edges
//   3  LDS staging: a block stages the union of its E edges' edgesOnEdge columns of u
//      and pv once (host-built list), then every wave computes from LDS
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GPTR __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ GPTR T* sp(T* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (GPTR T*)(((uint64_t)hi << 32) | lo);
}

// grouped XCD block order (mpas_dev.h xcd_block): G = 1 one contiguous eighth of the
// grid per XCD; G > 1 runs of G blocks per XCD in windows of 8G
__device__ __forceinline__ int xblk(int on) {
    const int b = (int)blockIdx.x, nb = (int)gridDim.x;
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

__device__ __forceinline__ void q_edge(int e, int k, const double* u, const double* pv, const int* eoe,
                                       const double* w, double* out) {
    int ee[10];
    double ue[10], pe[10];
#pragma unroll
    for (int j = 0; j < 10; j++) ee[j] = eoe[e * 10 + j];
#pragma unroll
    for (int j = 0; j < 10; j++) {
        ue[j] = sp(u + (size_t)ee[j] * 64)[k];
        pe[j] = sp(pv + (size_t)ee[j] * 64)[k];
    }
    const double p0 = sp(pv + (size_t)e * 64)[k];
    double q = 0;
#pragma unroll
    for (int j = 0; j < 10; j++) q += w[e * 10 + j] * ue[j] * 0.5 * (p0 + pe[j]);
    sp(out + (size_t)e * 64)[k] = q;
}

template <int TB>
__global__ __launch_bounds__(TB) void qv0(const double* u, const double* pv, const int* eoe, const double* w, int nE,
                                         double* out, int G = 0) {
    int e = xblk(G) * (TB / 64) + (int)(threadIdx.x >> 6);
    e = __builtin_amdgcn_readfirstlane(e);
    if (e >= nE) return;
    q_edge(e, threadIdx.x & 63, u, pv, eoe, w, out);
}

template <int Q>
__global__ __launch_bounds__(256) void qv2(const double* u, const double* pv, const int* eoe, const double* w, int nE,
                                           double* out) {
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (int i = 0; i < Q; i++) {
        int e = blockIdx.x * (4 * Q) + i * 4 + wv;
        if (e >= nE) return;
        q_edge(e, threadIdx.x & 63, u, pv, eoe, w, out);
    }
}

// LDS staging.  blk_off[b], blk_n[b]: the block's slice of ulist (global edge ids of the
// union of its edges' edgesOnEdge + the edges themselves); lidx[e*10+j]: slot of eoe_j in
// the block's LDS image; lself[e]: slot of e itself.  Levels: 56 (one row = 56 doubles).
template <int E, int MAXU, int TB>
__global__ __launch_bounds__(TB) void qv3(const double* u, const double* pv, const int* eoe, const double* w, int nE,
                                           double* out, const int* blk_off, const int* blk_n, const int* ulist,
                                           const uint16_t* lidx, const uint16_t* lself) {
    __shared__ double su[MAXU * 56];
    __shared__ double sv[MAXU * 56];
    const int b = blockIdx.x;
    const int off = blk_off[b], n = blk_n[b];
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int k = threadIdx.x & 63;
    // stage: each wave copies whole rows (lanes 0..55), 8 rows in flight per wave
    constexpr int NW = TB / 64;
    for (int s0 = wv; s0 < n; s0 += NW * 8) {
        double a[8], c[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const int s = min(s0 + NW * r, n - 1);
            const int g = __builtin_amdgcn_readfirstlane(ulist[off + s]);
            a[r] = sp(u + (size_t)g * 64)[k];
            c[r] = sp(pv + (size_t)g * 64)[k];
        }
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const int s = s0 + NW * r;
            if (s < n && k < 56) {
                su[s * 56 + k] = a[r];
                sv[s * 56 + k] = c[r];
            }
        }
    }
    __syncthreads();
    if (k >= 56) return;
    for (int i = 0; i < E / NW; i++) {
        const int e = __builtin_amdgcn_readfirstlane(b * E + i * NW + wv);
        if (e >= nE) return;
        const uint16_t* li = lidx + (size_t)e * 10;
        const double p0 = sv[lself[e] * 56 + k];
        double q = 0;
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const int s = li[j];
            q += w[e * 10 + j] * su[s * 56 + k] * 0.5 * (p0 + sv[s * 56 + k]);
        }
        sp(out + (size_t)e * 64)[k] = q;
    }
}


// 16-B lanes: a wavefront holds two edges, lane j of each half levels 2j and 2j+1
template <int TB>
__global__ __launch_bounds__(TB) void qv16(const double* u, const double* pv, const int* eoe, const double* w, int nE,
                                          double* out, int G = 0) {
    int e0 = xblk(G) * (TB / 32) + (int)(threadIdx.x >> 6) * 2;
    e0 = __builtin_amdgcn_readfirstlane(e0);
    if (e0 >= nE) return;
    const int half = (threadIdx.x >> 5) & 1, j = threadIdx.x & 31;
    const int e = min(e0 + half, nE - 1);
    int ee[10];
    double2 ue[10], pe[10];
#pragma unroll
    for (int i = 0; i < 10; i++) ee[i] = eoe[e * 10 + i];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        ue[i] = *(const double2*)(u + (size_t)ee[i] * 64 + 2 * j);
        pe[i] = *(const double2*)(pv + (size_t)ee[i] * 64 + 2 * j);
    }
    const double2 p0 = *(const double2*)(pv + (size_t)e * 64 + 2 * j);
    double qx = 0, qy = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const double wi = w[e * 10 + i];
        qx += wi * ue[i].x * 0.5 * (p0.x + pe[i].x);
        qy += wi * ue[i].y * 0.5 * (p0.y + pe[i].y);
    }
    if (e0 + half < nE) *(double2*)(out + (size_t)e * 64 + 2 * j) = make_double2(qx, qy);
}


// LDS staging of 16-level slices: block (edge block eb, level chunk kc) stages the union
// rows' levels [16kc, 16kc+16) (128-B pieces, 4 rows per wave-instruction); a wave
// computes 4 edges x 16 levels at a time (lane = 16*edge + level).
template <int E, int TB, int MAXU>
__global__ __launch_bounds__(TB) void qv4(const double* u, const double* pv, const int* eoe, const double* w, int nE,
                                          double* out, const int* blk_off, const int* blk_n, const int* ulist,
                                          const uint16_t* lidx, const uint16_t* lself, int nKC) {
    __shared__ double su[MAXU * 16];
    __shared__ double sv[MAXU * 16];
    constexpr int NW = TB / 64;
    const int b = blockIdx.x / nKC, kc = blockIdx.x - b * nKC;
    const int off = blk_off[b], n = min(blk_n[b], MAXU);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63, r = lane >> 4, kk = lane & 15, k = kc * 16 + kk;
    for (int s0 = wv * 4; s0 < n; s0 += NW * 16) {
        double a[4], c[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int s = min(s0 + NW * 4 * i + r, n - 1);
            const int g = ulist[off + s];
            a[i] = u[(size_t)g * 64 + k];
            c[i] = pv[(size_t)g * 64 + k];
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int s = s0 + NW * 4 * i + r;
            if (s < n) {
                su[s * 16 + kk] = a[i];
                sv[s * 16 + kk] = c[i];
            }
        }
    }
    __syncthreads();
    for (int i0 = wv * 4; i0 < E; i0 += NW * 4) {
        const int e = b * E + i0 + r;
        if (e >= nE) break;
        const uint16_t* li = lidx + (size_t)e * 10;
        const double p0 = sv[lself[e] * 16 + kk];
        double q = 0;
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const int sl = li[j];
            q += w[e * 10 + j] * su[sl * 16 + kk] * 0.5 * (p0 + sv[sl * 16 + kk]);
        }
        if (k < 56) out[(size_t)e * 64 + k] = q;
    }
}


// LDS staging with lane = level (full 56-level rows), a bounded LDS image of MAXU rows
// per field and a per-edge fallback: an edge whose neighbours are not all staged
// (lslot == 255) gathers them from global memory.  Slots come through the scalar unit.
template <int E, int MAXU>
__global__ __launch_bounds__(256) void qv5(const double* u, const double* pv, const int* eoe, const double* w, int nE,
                                           double* out, const int* blk_off, const int* blk_n, const int* ulist,
                                           const uint8_t* lslot) {
    __shared__ double su[MAXU * 56];
    __shared__ double sv[MAXU * 56];
    const int b = blockIdx.x;
    const int off = blk_off[b], n = min(blk_n[b], MAXU);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int k = threadIdx.x & 63;
    for (int s0 = wv; s0 < n; s0 += 32) {
        double a[8], c[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const int s = min(s0 + 4 * r, n - 1);
            const int g = __builtin_amdgcn_readfirstlane(ulist[off + s]);
            a[r] = sp(u + (size_t)g * 64)[k];
            c[r] = sp(pv + (size_t)g * 64)[k];
        }
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const int s = s0 + 4 * r;
            if (s < n && k < 56) {
                su[s * 56 + k] = a[r];
                sv[s * 56 + k] = c[r];
            }
        }
    }
    __syncthreads();
    if (k >= 56) return;
    for (int i = 0; i < E / 4; i++) {
        const int e = __builtin_amdgcn_readfirstlane(b * E + i * 4 + wv);
        if (e >= nE) return;
        const uint8_t* ls = lslot + (size_t)e * 11;  // 10 neighbours + the edge itself
        uint32_t sl[11];
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 11; j++) {
            sl[j] = ls[j];
            ok = ok && sl[j] != 255u;
        }
        if (ok) {
            const double p0 = sv[sl[10] * 56 + k];
            double q = 0;
#pragma unroll
            for (int j = 0; j < 10; j++) q += w[e * 10 + j] * su[sl[j] * 56 + k] * 0.5 * (p0 + sv[sl[j] * 56 + k]);
            sp(out + (size_t)e * 64)[k] = q;
        } else {
            q_edge(e, k, u, pv, eoe, w, out);
        }
    }
}


// qv5 with the staging done by LDS-DMA (global_load_lds_dwordx4: one wave-instruction
// copies two 512-B rows, lanes 0-31 the first, 32-63 the second; no VGPRs, so every wave
// keeps all its rows in flight)
template <int E, int MAXU>
__global__ __launch_bounds__(256) void qv6(const double* u, const double* pv, const int* eoe, const double* w, int nE,
                                           double* out, const int* blk_off, const int* blk_n, const int* ulist,
                                           const uint8_t* lslot) {
    __shared__ double su[MAXU * 64];
    __shared__ double sv[MAXU * 64];
    const int b = blockIdx.x;
    const int off = blk_off[b], n = min(blk_n[b], MAXU);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63, k = lane;
    for (int s0 = 2 * wv; s0 < n; s0 += 8) {
        const int r = min(s0 + (lane >> 5), n - 1);
        const int g = ulist[off + r];
        const double* src_u = u + (size_t)g * 64 + (lane & 31) * 2;
        const double* src_v = pv + (size_t)g * 64 + (lane & 31) * 2;
        __builtin_amdgcn_global_load_lds((const void*)src_u, (__attribute__((address_space(3))) void*)(su + s0 * 64), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)src_v, (__attribute__((address_space(3))) void*)(sv + s0 * 64), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
    __syncthreads();
    if (k >= 56) return;
    for (int i = 0; i < E / 4; i++) {
        const int e = __builtin_amdgcn_readfirstlane(b * E + i * 4 + wv);
        if (e >= nE) return;
        const uint8_t* ls = lslot + (size_t)e * 11;
        uint32_t sl[11];
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 11; j++) {
            sl[j] = ls[j];
            ok = ok && sl[j] != 255u;
        }
        if (ok) {
            const double p0 = sv[sl[10] * 64 + k];
            double q = 0;
#pragma unroll
            for (int j = 0; j < 10; j++) q += w[e * 10 + j] * su[sl[j] * 64 + k] * 0.5 * (p0 + sv[sl[j] * 64 + k]);
            sp(out + (size_t)e * 64)[k] = q;
        } else {
            q_edge(e, k, u, pv, eoe, w, out);
        }
    }
}

extern "C" int ub_q(int variant, const double* u, const double* pv, const int* eoe, const double* w, int nE,
                    double* out, const int* blk_off, const int* blk_n, const int* ulist, const uint16_t* lidx,
                    const uint16_t* lself, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    switch (variant) {
        case 0: qv0<256><<<(nE + 3) / 4, 256, 0, st>>>(u, pv, eoe, w, nE, out); break;
        case 1: qv0<1024><<<(nE + 15) / 16, 1024, 0, st>>>(u, pv, eoe, w, nE, out); break;
        case 2: qv2<4><<<(nE + 15) / 16, 256, 0, st>>>(u, pv, eoe, w, nE, out); break;
        case 3: qv2<16><<<(nE + 63) / 64, 256, 0, st>>>(u, pv, eoe, w, nE, out); break;
        case 4: qv3<32, 160, 256><<<(nE + 31) / 32, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself); break;
        case 5: qv3<32, 160, 512><<<(nE + 31) / 32, 512, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself); break;
        case 6: qv3<16, 120, 256><<<(nE + 15) / 16, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself); break;
        case 7: qv3<16, 120, 512><<<(nE + 15) / 16, 512, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself); break;
        case 8: qv16<256><<<(nE + 7) / 8, 256, 0, st>>>(u, pv, eoe, w, nE, out); break;
        case 9: qv16<1024><<<(nE + 31) / 32, 1024, 0, st>>>(u, pv, eoe, w, nE, out); break;
        case 10: qv0<512><<<(nE + 7) / 8, 512, 0, st>>>(u, pv, eoe, w, nE, out); break;
        case 11: qv0<256><<<(nE + 3) / 4, 256, 0, st>>>(u, pv, eoe, w, nE, out, 1); break;
        case 12: qv0<1024><<<(nE + 15) / 16, 1024, 0, st>>>(u, pv, eoe, w, nE, out, 1); break;
        case 13: qv16<256><<<(nE + 7) / 8, 256, 0, st>>>(u, pv, eoe, w, nE, out, 1); break;
        case 14: qv16<1024><<<(nE + 31) / 32, 1024, 0, st>>>(u, pv, eoe, w, nE, out, 1); break;
        case 15: qv0<256><<<(nE + 3) / 4, 256, 0, st>>>(u, pv, eoe, w, nE, out, 64); break;
        case 16: qv0<1024><<<(nE + 15) / 16, 1024, 0, st>>>(u, pv, eoe, w, nE, out, 16); break;
        case 17: qv16<256><<<(nE + 7) / 8, 256, 0, st>>>(u, pv, eoe, w, nE, out, 64); break;
        case 18: qv16<1024><<<(nE + 31) / 32, 1024, 0, st>>>(u, pv, eoe, w, nE, out, 16); break;
        case 19: qv4<16, 256, 120><<<((nE + 15) / 16) * 4, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself, 4); break;
        case 20: qv4<32, 256, 160><<<((nE + 31) / 32) * 4, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself, 4); break;
        case 21: qv4<32, 512, 160><<<((nE + 31) / 32) * 4, 512, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself, 4); break;
        case 22: qv4<64, 1024, 240><<<((nE + 63) / 64) * 4, 1024, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself, 4); break;
        case 23: qv4<64, 256, 240><<<((nE + 63) / 64) * 4, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, lidx, lself, 4); break;
        case 24: qv5<16, 64><<<(nE + 15) / 16, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, (const uint8_t*)lidx); break;
        case 25: qv5<16, 48><<<(nE + 15) / 16, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, (const uint8_t*)lidx); break;
        case 26: qv5<32, 96><<<(nE + 31) / 32, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, (const uint8_t*)lidx); break;
        case 27: qv6<16, 64><<<(nE + 15) / 16, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, (const uint8_t*)lidx); break;
        case 28: qv6<16, 48><<<(nE + 15) / 16, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, (const uint8_t*)lidx); break;
        case 29: qv6<32, 96><<<(nE + 31) / 32, 256, 0, st>>>(u, pv, eoe, w, nE, out, blk_off, blk_n, ulist, (const uint8_t*)lidx); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}
