// jw_host.cpp -- host-side part of the JW baroclinic-wave initial state:
// the per-column hydrostatic iteration of init_atm_case_jw (vertical_init/init_atm_cases.rg
// :366-432, mpasdyn/jw.py), the one loop of the initial state that costs seconds per
// 10^5 columns in NumPy (10 temperature passes x 25 pressure passes x nVertLevels).
// Column-independent: the columns are split over host threads.  The arithmetic is
// jw.py's, in its evaluation order.
#include <cmath>
#include <cstdint>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "mpas_dyn.h"

namespace {
constexpr double RGAS = 287.0, GRAVITY = 9.80616, P0 = 1.0e5;
constexpr double U0 = 35.0, T0B = 250.0, T0 = 288.0, DELTA_T = 4.8e5, DTDZ = 0.005, ETA_T = 0.2;
constexpr double SPHERE_RADIUS = 6371229.0, OMEGA = 7.29212E-5;
const double PI = std::acos(-1.0);

// jw.py _jw_temperature at one point (eta, column sin/cos of latitude)
double jw_temperature(double eta, double s, double c) {
    const double etav = (eta - 0.252) * PI / 2.0;
    double teta = T0 * std::pow(eta, RGAS * DTDZ / GRAVITY);
    if (!(eta >= ETA_T)) teta = teta + DELTA_T * std::pow(std::fabs(ETA_T - eta), 5.0);
    const double ce = std::cos(etav);
    return teta + 0.75 * eta * PI * U0 / RGAS * std::sin(etav) * std::sqrt(ce) *
                      ((-2.0 * std::pow(s, 6.0) * (c * c + 1.0 / 3.0) + 10.0 / 63.0) * 2.0 * U0 * std::pow(ce, 1.5) +
                       (1.6 * std::pow(c, 3.0) * (s * s + 2.0 / 3.0) - PI / 4.0) * SPHERE_RADIUS * OMEGA);
}

void columns(int c0, int c1, int L, const double* phi, const double* pb, const double* rb, const double* zz,
             const double* dzw, const double* dzu, const double* fzm, const double* fzp, double* pp, double* rr,
             double* tt) {
    std::vector<double> p(L), r(L), t(L), ppi(L);
    const double cdz0 = 0.5 * dzw[0] * GRAVITY;
    for (int ci = c0; ci < c1; ci++) {
        const size_t o = (size_t)ci * L;
        const double s = std::sin(phi[ci]), c = std::cos(phi[ci]);
        for (int k = 0; k < L; k++) p[k] = r[k] = 0.0;
        for (int it = 0; it < 10; it++) {
            for (int k = 0; k < L; k++) t[k] = jw_temperature((pb[o + k] + p[k]) / P0, s, c);
            for (int jt = 0; jt < 25; jt++) {
                for (int k = 0; k < L; k++) r[k] = (p[k] / (RGAS * zz[o + k]) - rb[o + k] * (t[k] - T0B)) / t[k];
                ppi[0] = P0 - cdz0 * (1.25 * (r[0] + rb[o]) - 0.25 * (r[1] + rb[o + 1]));
                ppi[0] -= pb[o];
                for (int k = 0; k + 1 < L; k++)
                    ppi[k + 1] = ppi[k] - (dzu[k + 1] * GRAVITY) * (r[k] * fzp[k + 1] + r[k + 1] * fzm[k + 1]);
                for (int k = 0; k < L; k++) p[k] = 0.2 * ppi[k] + 0.8 * p[k];
            }
        }
        for (int k = 0; k < L; k++) {
            pp[o + k] = p[k];
            rr[o + k] = r[k];
            tt[o + k] = t[k];
        }
    }
}
}  // namespace

extern "C" int mpas_jw_hydrostatic(int32_t nCells, int32_t nVertLevels, const double* latCell, const double* pb,
                                   const double* rb, const double* zz, const double* dzw, const double* dzu,
                                   const double* fzm, const double* fzp, double* pressure_p, double* rho_p,
                                   double* temperature, int32_t nthreads) {
    if (nCells < 0 || nVertLevels < 2 || !latCell || !pb || !rb || !zz || !dzw || !dzu || !fzm || !fzp ||
        !pressure_p || !rho_p || !temperature)
        return MPAS_EINVAL;
    int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    if (nt < 1) nt = 1;
    if (nt > 64) nt = 64;
    if (nt > nCells) nt = nCells > 0 ? nCells : 1;
    // (the recurrence reads levels 0 and 1: nVertLevels >= 2.)  No exception crosses the C
    // ABI: a thread that cannot be started leaves its columns to this thread, and an
    // allocation failure is reported as MPAS_ENOMEM.
    try {
        std::vector<std::thread> th;
        th.reserve(nt);  // (emplace_back never reallocates past started threads)
        const int per = (nCells + nt - 1) / nt;
        for (int i = 0; i < nt; i++) {
            const int c0 = i * per, c1 = std::min(nCells, c0 + per);
            if (c0 >= c1) break;
            try {
                th.emplace_back(columns, c0, c1, (int)nVertLevels, latCell, pb, rb, zz, dzw, dzu, fzm, fzp, pressure_p,
                                rho_p, temperature);
            } catch (const std::system_error&) {
                columns(c0, c1, (int)nVertLevels, latCell, pb, rb, zz, dzw, dzu, fzm, fzp, pressure_p, rho_p,
                        temperature);
            }
        }
        for (auto& t : th) t.join();
    } catch (const std::bad_alloc&) {
        return MPAS_ENOMEM;
    } catch (...) {
        return MPAS_EINVAL;
    }
    return MPAS_OK;
}
