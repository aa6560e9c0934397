"""Generate tests/golden/oracle_x1.2562.json: digests of the oracle's outputs for every
hot-path task (and one RK3 step) on the reference's own mesh x1.2562 at 5 and 56
levels, from the seeded synthetic state.  The reference itself cannot be run (SURVEY
§8.4: no Regent/Legion toolchain), so these vectors pin the oracle against regressions
-- PARITY UNPINNED against the reference.  Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "mpas-regent_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]

import oracle as O  # noqa: E402
from helpers import SCRATCH, digest, make_state  # noqa: E402
from mpasdyn import mesh  # noqa: E402
from mpasdyn.registry import FIELDS  # noqa: E402

CASES = {
    "setup": lambda o: o.atm_rk_integration_setup(),
    "moist": lambda o: o.atm_compute_moist_coefficients(),
    "vert_imp": lambda o: o.atm_compute_vert_imp_coefs(240.0),
    "dyn_tend_rk0": lambda o: o.atm_compute_dyn_tend_work(0, 720.0),
    "dyn_tend_rk1": lambda o: o.atm_compute_dyn_tend_work(1, 720.0),
    "smlstep": lambda o: o.atm_set_smlstep_pert_variables_work(),
    "acoustic_s0": lambda o: o.atm_advance_acoustic_step_work(240.0, 0),
    "acoustic_s1": lambda o: o.atm_advance_acoustic_step_work(360.0, 1),
    "div_damp": lambda o: o.atm_divergence_damping_3d(240.0),
    "solve_diag_rk2": lambda o: o.atm_compute_solve_diagnostics(0, 2),
    "finish": lambda o: o.atm_rk_dynamics_substep_finish(1, 1),
    "srk3_ref_schedule": lambda o: o.atm_srk3(720.0, 0),
    "srk3_mpas_schedule": lambda o: o.atm_srk3(720.0, 1),
    "recover_ns2_rk0": lambda o: o.atm_recover_large_step_variables_work(2, 0, 240.0),
    "recover_ns3_rk2": lambda o: o.atm_recover_large_step_variables_work(3, 2, 240.0),
    "reconstruct_2d": lambda o: o.mpas_reconstruct_2d(False, True),
    "output_diagnostics": lambda o: o.atm_compute_output_diagnostics(),
    # monotonic scalar transport (Q26, mpas mode; parity unpinned, tests/test_transport.py)
    "scalars_mono": lambda o: o.mpas_advance_scalars_mono(600.0),
    "mpas_srk3_transport": lambda o: o.mpas_srk3(720.0, 1, transport=True),
    # the one-time tasks of atm_core_init on the device
    "damping_coefs": lambda o: o.atm_compute_damping_coefs(22000.0, 0.2),
    "init_coupled_diagnostics": lambda o: o.atm_init_coupled_diagnostics(),
}


def generate():
    m = mesh.load_x1_2562()
    out = {}
    for L in (5, 56):
        for variant in ("ref", "random"):
            st0 = make_state(m, L, variant)
            key = f"L{L}_{variant}"
            out[key] = {"inputs": {f.name: digest(st0[f.name]) for f in FIELDS}}
            for case, fn in CASES.items():
                st = st0.copy()
                fn(O.Oracle(st))
                out[key][case] = {f.name: digest(st[f.name]) for f in FIELDS
                                  if f.name not in SCRATCH and st[f.name].tobytes() != st0[f.name].tobytes()}
            out[key]["summarize_timestep"] = digest(O.Oracle(st0.copy()).summarize_timestep(True, True))
    return out


if __name__ == "__main__":
    g = generate()
    with open(os.path.join(HERE, "oracle_x1.2562.json"), "w") as f:
        json.dump(g, f, indent=0, sort_keys=True)
    print("wrote", sum(len(v) for v in g.values()), "cases")
