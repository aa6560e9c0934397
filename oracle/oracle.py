"""ctypes driver of the CPU oracle (oracle/mpas_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as
the checker, never by the product package.  PARITY UNPINNED (see mpas_oracle.c).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mpas-regent_amd"))
from mpasdyn.registry import FIELDS, F_COUNT  # noqa: E402

LIB_PATH = os.path.join(HERE, "libmpas_oracle.so")
HORIZ = {"2d_smagorinsky": 0, "2d_fixed": 1}


class OraState(ctypes.Structure):
    _fields_ = [("nCells", ctypes.c_int32), ("nEdges", ctypes.c_int32), ("nVertices", ctypes.c_int32),
                ("L", ctypes.c_int32), ("f", ctypes.c_void_p * F_COUNT)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        p = ctypes.POINTER(OraState)
        i32, dbl = ctypes.c_int, ctypes.c_double
        sig = {
            "ora_field_count": (i32, []),
            "ora_fill_synthetic": (None, [p, ctypes.c_uint64, i32]),
            "ora_atm_rk_integration_setup": (None, [p]),
            "ora_atm_compute_moist_coefficients": (None, [p]),
            "ora_atm_compute_vert_imp_coefs": (None, [p, dbl]),
            "ora_atm_compute_dyn_tend_work": (None, [p, i32, dbl, i32, dbl, i32, i32]),
            "ora_atm_set_smlstep_pert_variables_work": (None, [p]),
            "ora_atm_advance_acoustic_step_work": (None, [p, dbl, i32]),
            "ora_atm_divergence_damping_3d": (None, [p, dbl]),
            "ora_atm_compute_solve_diagnostics": (None, [p, i32, i32]),
            "ora_atm_rk_dynamics_substep_finish": (None, [p, i32, i32]),
            "ora_atm_srk3": (None, [p, dbl, i32]),
            "ora_atm_recover_large_step_variables_work": (None, [p, i32, i32, dbl]),
            "ora_mpas_reconstruct_2d": (None, [p, i32, i32]),
            "ora_atm_compute_output_diagnostics": (None, [p]),
            "ora_mpas_vert_imp_coefs": (None, [p, dbl]),
            "ora_mpas_acoustic_step": (None, [p, dbl, i32]),
            "ora_mpas_srk3": (None, [p, dbl, i32]),
            "ora_mpas_srk3_ex": (None, [p, dbl, i32, i32]),
            "ora_mpas_advance_scalars_mono": (None, [p, dbl]),
            "ora_atm_compute_damping_coefs": (None, [p, dbl, dbl]),
            "ora_atm_compute_signs": (None, [p]),
            "ora_atm_adv_coef_compression": (None, [p]),
            "ora_atm_couple_coef_3rd_order": (None, [p, dbl]),
            "ora_atm_compute_mesh_scaling": (None, [p, i32]),
            "ora_atm_init_coupled_diagnostics": (None, [p]),
            "ora_mpas_recover": (None, [p, i32, i32, dbl]),
            "ora_summarize_timestep": (None, [p, i32, i32, ctypes.POINTER(ctypes.c_double)]),
            "ora_mpas_srk3_dyn": (None, [p, dbl, i32, i32, i32]),
            "ora_mpas_rk_integration_setup": (None, [p]),
            "ora_mpas_moist_coefficients": (None, [p]),
            "ora_mpas_dyn_tend": (None, [p, i32, dbl, i32, dbl, i32, i32]),
            "ora_mpas_set_smlstep": (None, [p]),
            "ora_mpas2_acoustic_step": (None, [p, dbl, i32]),
            "ora_mpas_solve_diagnostics": (None, [p, i32, i32]),
            "ora_mpas_substep_finish": (None, [p, i32, i32]),
            "ora_mpas_surface_pressure": (None, [p]),
        }
        for n, (res, args) in sig.items():
            fn = getattr(L, n)
            fn.restype, fn.argtypes = res, args
        assert L.ora_field_count() == F_COUNT, "oracle built from a different mpas_fields.def"
        _lib = L
    return _lib


class Oracle:
    """Runs the reference tasks on a HostState in place."""

    def __init__(self, state):
        self.state = state
        self.lib = load()
        s = OraState()
        s.nCells, s.nEdges, s.nVertices, s.L = state.dims()
        assert state.L < 128
        for f in FIELDS:
            a = state.arrays[f.name]
            assert a.flags.c_contiguous
            s.f[f.index] = a.ctypes.data
        self.s = s
        self.p = ctypes.byref(s)

    def fill_synthetic(self, seed, include_mesh=False):
        self.lib.ora_fill_synthetic(self.p, seed, 1 if include_mesh else 0)

    def atm_rk_integration_setup(self):
        self.lib.ora_atm_rk_integration_setup(self.p)

    def atm_compute_moist_coefficients(self):
        self.lib.ora_atm_compute_moist_coefficients(self.p)

    def atm_compute_vert_imp_coefs(self, dts):
        self.lib.ora_atm_compute_vert_imp_coefs(self.p, dts)

    def atm_compute_dyn_tend_work(self, rk_step, dt, config_horiz_mixing="2d_smagorinsky", config_mpas_cam_coef=0.0,
                                  config_mix_full=False, config_rayleigh_damp_u=False):
        hm = config_horiz_mixing if isinstance(config_horiz_mixing, int) else HORIZ.get(config_horiz_mixing, 2)
        self.lib.ora_atm_compute_dyn_tend_work(self.p, rk_step, dt, hm, config_mpas_cam_coef, int(config_mix_full),
                                               int(config_rayleigh_damp_u))

    def atm_set_smlstep_pert_variables_work(self):
        self.lib.ora_atm_set_smlstep_pert_variables_work(self.p)

    def atm_advance_acoustic_step_work(self, dts, small_step):
        self.lib.ora_atm_advance_acoustic_step_work(self.p, dts, small_step)

    def atm_divergence_damping_3d(self, dts):
        self.lib.ora_atm_divergence_damping_3d(self.p, dts)

    def atm_compute_solve_diagnostics(self, hollingsworth, rk_step):
        self.lib.ora_atm_compute_solve_diagnostics(self.p, int(hollingsworth), rk_step)

    def atm_rk_dynamics_substep_finish(self, dynamics_substep, dynamics_split):
        self.lib.ora_atm_rk_dynamics_substep_finish(self.p, dynamics_substep, dynamics_split)

    def atm_srk3(self, dt, schedule=0):
        self.lib.ora_atm_srk3(self.p, dt, schedule)

    def atm_recover_large_step_variables_work(self, ns, rk_step, dt):
        self.lib.ora_atm_recover_large_step_variables_work(self.p, ns, rk_step, dt)

    # the MPAS vertical solver ("physics" mpas; mpas_oracle.c)
    def mpas_vert_imp_coefs(self, dts):
        self.lib.ora_mpas_vert_imp_coefs(self.p, dts)

    def mpas_acoustic_step(self, dts, small_step):
        self.lib.ora_mpas_acoustic_step(self.p, dts, small_step)

    def mpas_recover(self, ns, rk_step, dt):
        self.lib.ora_mpas_recover(self.p, ns, rk_step, dt)

    def mpas_srk3(self, dt, schedule=1, transport=False, physics=1):
        """physics 1: the MPAS vertical solver; physics 2: the MPAS dynamics (every quirk fixed)"""
        self.lib.ora_mpas_srk3_dyn(self.p, dt, schedule, int(bool(transport)), int(physics))

    # the MPAS dynamics (physics = 2), task by task
    def mpas_rk_integration_setup(self):
        self.lib.ora_mpas_rk_integration_setup(self.p)

    def mpas_moist_coefficients(self):
        self.lib.ora_mpas_moist_coefficients(self.p)

    def mpas_dyn_tend(self, rk_step, dt, config_horiz_mixing="2d_smagorinsky", config_mpas_cam_coef=0.0,
                      config_mix_full=False, config_rayleigh_damp_u=False):
        hm = config_horiz_mixing if isinstance(config_horiz_mixing, int) else HORIZ.get(config_horiz_mixing, 2)
        self.lib.ora_mpas_dyn_tend(self.p, rk_step, dt, hm, config_mpas_cam_coef, int(config_mix_full),
                                   int(config_rayleigh_damp_u))

    def mpas_set_smlstep(self):
        self.lib.ora_mpas_set_smlstep(self.p)

    def mpas2_acoustic_step(self, dts, small_step):
        self.lib.ora_mpas2_acoustic_step(self.p, dts, small_step)

    def mpas_solve_diagnostics(self, hollingsworth, rk_step):
        self.lib.ora_mpas_solve_diagnostics(self.p, int(hollingsworth), rk_step)

    def mpas_substep_finish(self, dynamics_substep=1, dynamics_split=1):
        self.lib.ora_mpas_substep_finish(self.p, dynamics_substep, dynamics_split)

    def mpas_surface_pressure(self):
        self.lib.ora_mpas_surface_pressure(self.p)

    def atm_compute_damping_coefs(self, config_zd=22000.0, config_xnutr=0.2):
        self.lib.ora_atm_compute_damping_coefs(self.p, config_zd, config_xnutr)

    def atm_init_coupled_diagnostics(self):
        self.lib.ora_atm_init_coupled_diagnostics(self.p)

    def atm_compute_signs(self):
        """dynamics_tasks.rg:46-130"""
        self.lib.ora_atm_compute_signs(self.p)

    def atm_adv_coef_compression(self):
        """dynamics_tasks.rg:133-269"""
        self.lib.ora_atm_adv_coef_compression(self.p)

    def atm_couple_coef_3rd_order(self, config_coef_3rd_order=0.25):
        """dynamics_tasks.rg:303-325"""
        self.lib.ora_atm_couple_coef_3rd_order(self.p, config_coef_3rd_order)

    def atm_compute_mesh_scaling(self, config_h_ScaleWithMesh=True):
        """dynamics_tasks.rg:595-646"""
        self.lib.ora_atm_compute_mesh_scaling(self.p, int(bool(config_h_ScaleWithMesh)))

    def atm_core_init(self):
        """atm_core.rg:22-42: every task in order (physics_init is a stub, OUT OF SCOPE)"""
        self.atm_compute_signs()
        self.atm_adv_coef_compression()
        self.atm_couple_coef_3rd_order(0.25)
        self.atm_init_coupled_diagnostics()
        self.atm_compute_solve_diagnostics(0, -1)
        self.mpas_reconstruct_2d(False, True)
        self.atm_compute_mesh_scaling(True)
        self.atm_compute_damping_coefs(22000.0, 0.2)

    def mpas_advance_scalars_mono(self, dt):
        """monotonic scalar transport (Q26: not in the reference; mpas_oracle.c)"""
        self.lib.ora_mpas_advance_scalars_mono(self.p, dt)

    def atm_compute_output_diagnostics(self):
        self.lib.ora_atm_compute_output_diagnostics(self.p)

    def mpas_reconstruct_2d(self, includeHalos=False, on_a_sphere=True):
        self.lib.ora_mpas_reconstruct_2d(self.p, int(includeHalos), int(on_a_sphere))

    def summarize_timestep(self, config_print_detailed_minmax_vel=True, config_print_global_minmax_vel=True):
        """the 31 values the reference prints (layout: mpas_oracle.c ora_summarize_timestep)"""
        out = np.zeros(31)
        self.lib.ora_summarize_timestep(self.p, int(config_print_detailed_minmax_vel),
                                        int(config_print_global_minmax_vel),
                                        out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        return out
