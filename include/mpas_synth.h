/* mpas_synth.h -- counter-based synthetic-state generator shared by the oracle (C),
 * the device library (HIP) and the Python harness (numpy mirror in mpasdyn/synth.py).
 *
 * value(seed, field, entity, level, comp) = lo + (hi - lo) * u01(hash)
 * The hash is four chained splitmix64 rounds, so any (field, entity, level, comp)
 * point can be generated independently on any device in any order.
 * seed 20211015 for the benchmark state.
 */
#ifndef MPAS_SYNTH_H
#define MPAS_SYNTH_H
#include <stdint.h>

#if defined(__HIPCC__)
#define MPAS_HD __host__ __device__ __forceinline__
#else
#define MPAS_HD static inline
#endif

MPAS_HD uint64_t mpas_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

MPAS_HD uint64_t mpas_point_hash(uint64_t seed, uint32_t field, uint64_t entity,
                                 uint32_t level, uint32_t comp) {
    uint64_t h = mpas_splitmix64(seed);
    h = mpas_splitmix64(h ^ (uint64_t)field);
    h = mpas_splitmix64(h ^ entity);
    h = mpas_splitmix64(h ^ (((uint64_t)level << 16) | (uint64_t)comp));
    return h;
}

/* uniform in [0, 1) with 53 random bits */
MPAS_HD double mpas_u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

/* DIST codes of mpas_fields.def */
enum { MPAS_DIST_U = 0, MPAS_DIST_Z = 1, MPAS_DIST_B = 2, MPAS_DIST_M = 3, MPAS_DIST_S = 4 };

MPAS_HD double mpas_synth_value(uint64_t seed, uint32_t field, uint64_t entity, uint32_t level,
                                uint32_t comp, int dist, double lo, double hi) {
    uint64_t h = mpas_point_hash(seed, field, entity, level, comp);
    double r = mpas_u01(h);
    if (dist == MPAS_DIST_Z) return 0.0;
    if (dist == MPAS_DIST_B) return (r < hi) ? 1.0 : 0.0;
    if (dist == MPAS_DIST_S) return (r < 0.5) ? -1.0 : 1.0;
    return lo + (hi - lo) * r;
}

#endif
