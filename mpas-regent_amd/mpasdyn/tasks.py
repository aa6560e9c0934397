"""Host-side mirror of the reference's task interface for the RK3 hot path.

Same names, same scalar arguments in the same order as the Regent tasks
(dynamics/dynamics_tasks.rg, dynamics/rk_timestep.rg); the region arguments
(cr, cpr, er, vr, vert_r) are the device-resident state of a Context.  Errors raise
MpasError (the reference's tasks return nothing and abort on failure).
"""
from .lib import HORIZ_MIXING, MpasError


def _mix(config_horiz_mixing):
    if isinstance(config_horiz_mixing, int):
        return config_horiz_mixing
    return HORIZ_MIXING.get(config_horiz_mixing, 2)


def atm_rk_integration_setup(ctx):
    """dynamics_tasks.rg:747"""
    ctx._check(ctx.lib.mpas_atm_rk_integration_setup(ctx.h), "atm_rk_integration_setup")


def atm_compute_moist_coefficients(ctx):
    """dynamics_tasks.rg:460"""
    ctx._check(ctx.lib.mpas_atm_compute_moist_coefficients(ctx.h), "atm_compute_moist_coefficients")


def atm_compute_vert_imp_coefs(ctx, dts):
    """dynamics_tasks.rg:513"""
    ctx._check(ctx.lib.mpas_atm_compute_vert_imp_coefs(ctx.h, float(dts)), "atm_compute_vert_imp_coefs")


def atm_compute_dyn_tend_work(ctx, rk_step, dt, config_horiz_mixing="2d_smagorinsky", config_mpas_cam_coef=0.0,
                              config_mix_full=False, config_rayleigh_damp_u=False):
    """dynamics_tasks.rg:814 (constants.rg:57-60 defaults)"""
    ctx._check(ctx.lib.mpas_atm_compute_dyn_tend_work(ctx.h, int(rk_step), float(dt), _mix(config_horiz_mixing),
                                                       float(config_mpas_cam_coef), int(bool(config_mix_full)),
                                                       int(bool(config_rayleigh_damp_u))), "atm_compute_dyn_tend_work")


atm_compute_dyn_tend = atm_compute_dyn_tend_work  # :1484 wrapper


def atm_set_smlstep_pert_variables_work(ctx):
    """dynamics_tasks.rg:1503; the cpr sub-region is the cprMask field"""
    ctx._check(ctx.lib.mpas_atm_set_smlstep_pert_variables_work(ctx.h), "atm_set_smlstep_pert_variables_work")


atm_set_smlstep_pert_variables = atm_set_smlstep_pert_variables_work  # :1530 wrapper


def atm_advance_acoustic_step_work(ctx, dts, small_step):
    """dynamics_tasks.rg:1546"""
    ctx._check(ctx.lib.mpas_atm_advance_acoustic_step_work(ctx.h, float(dts), int(small_step)),
               "atm_advance_acoustic_step_work")


atm_advance_acoustic_step = atm_advance_acoustic_step_work  # :1707 wrapper


def atm_divergence_damping_3d(ctx, dts):
    """dynamics_tasks.rg:1726"""
    ctx._check(ctx.lib.mpas_atm_divergence_damping_3d(ctx.h, float(dts)), "atm_divergence_damping_3d")


def atm_compute_solve_diagnostics(ctx, hollingsworth, rk_step):
    """dynamics_tasks.rg:328"""
    ctx._check(ctx.lib.mpas_atm_compute_solve_diagnostics(ctx.h, int(bool(hollingsworth)), int(rk_step)),
               "atm_compute_solve_diagnostics")


def atm_rk_dynamics_substep_finish(ctx, dynamics_substep, dynamics_split):
    """dynamics_tasks.rg:1951"""
    ctx._check(ctx.lib.mpas_atm_rk_dynamics_substep_finish(ctx.h, int(dynamics_substep), int(dynamics_split)),
               "atm_rk_dynamics_substep_finish")


def atm_recover_large_step_variables_work(ctx, ns, rk_step, dt):
    """dynamics_tasks.rg:1766 (not called by atm_srk3: rk_timestep.rg:460, Q7)"""
    ctx._check(ctx.lib.mpas_atm_recover_large_step_variables_work(ctx.h, int(ns), int(rk_step), float(dt)),
               "atm_recover_large_step_variables_work")


atm_recover_large_step_variables = atm_recover_large_step_variables_work  # :1876 wrapper


def mpas_reconstruct_2d(ctx, includeHalos=False, on_a_sphere=True):
    """dynamics_tasks.rg:1893 (atm_core.rg:33 calls it with false, true)"""
    ctx._check(ctx.lib.mpas_reconstruct_2d(ctx.h, int(bool(includeHalos)), int(bool(on_a_sphere))),
               "mpas_reconstruct_2d")


def atm_compute_output_diagnostics(ctx):
    """dynamics_tasks.rg:729 (main.rg:70, after the time loop): rho, pressure"""
    ctx._check(ctx.lib.mpas_atm_compute_output_diagnostics(ctx.h), "atm_compute_output_diagnostics")


def atm_compute_damping_coefs(ctx, config_zd=22000.0, config_xnutr=0.2):
    """dynamics_tasks.rg:274 (atm_core_init, atm_core.rg:41; constants.rg defaults)"""
    ctx._check(ctx.lib.mpas_atm_compute_damping_coefs(ctx.h, float(config_zd), float(config_xnutr)),
               "atm_compute_damping_coefs")


def atm_init_coupled_diagnostics(ctx):
    """dynamics_tasks.rg:651 (atm_core_init, atm_core.rg:31)"""
    ctx._check(ctx.lib.mpas_atm_init_coupled_diagnostics(ctx.h), "atm_init_coupled_diagnostics")


def atm_compute_signs(ctx):
    """dynamics_tasks.rg:46 (atm_core_init, atm_core.rg:22)"""
    ctx._check(ctx.lib.mpas_atm_compute_signs(ctx.h), "atm_compute_signs")


def atm_adv_coef_compression(ctx):
    """dynamics_tasks.rg:133 (atm_core_init, atm_core.rg:24)"""
    ctx._check(ctx.lib.mpas_atm_adv_coef_compression(ctx.h), "atm_adv_coef_compression")


def atm_couple_coef_3rd_order(ctx, config_coef_3rd_order=0.25):
    """dynamics_tasks.rg:303 (atm_core_init, atm_core.rg:27; namelist 0.25)"""
    ctx._check(ctx.lib.mpas_atm_couple_coef_3rd_order(ctx.h, float(config_coef_3rd_order)),
               "atm_couple_coef_3rd_order")


def atm_compute_mesh_scaling(ctx, config_h_ScaleWithMesh=True):
    """dynamics_tasks.rg:595 (atm_core_init, atm_core.rg:39)"""
    ctx._check(ctx.lib.mpas_atm_compute_mesh_scaling(ctx.h, int(bool(config_h_ScaleWithMesh))),
               "atm_compute_mesh_scaling")


def atm_core_init(ctx):
    """atm_core.rg:22: every task of atm_core_init in order, on the device"""
    ctx._check(ctx.lib.mpas_atm_core_init(ctx.h), "atm_core_init")


def atm_advance_scalars_mono(ctx, dt):
    """Monotonic scalar transport of scalars_old into scalars over dt (SURVEY §8.7 row 4;
    no reference task exists, Q26 -- MPAS-A's atm_advance_scalars_mono; include/mpas_dyn.h)"""
    ctx._check(ctx.lib.mpas_atm_advance_scalars_mono(ctx.h, float(dt)), "atm_advance_scalars_mono")


def summarize_timestep(ctx, config_print_detailed_minmax_vel=False, config_print_global_minmax_vel=False,
                       config_print_global_minmax_sca=False):
    """rk_timestep.rg:29; returns the 31 values the reference prints (layout: include/mpas_dyn.h)"""
    import ctypes

    import numpy as np
    out = np.zeros(31)
    ctx._check(ctx.lib.mpas_summarize_timestep(ctx.h, int(bool(config_print_detailed_minmax_vel)),
                                               int(bool(config_print_global_minmax_vel)),
                                               int(bool(config_print_global_minmax_sca)),
                                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))),
               "summarize_timestep")
    return out


def atm_srk3(ctx, dt, schedule=0):
    """rk_timestep.rg:361; schedule 0 = the reference's driver, 1 = rk_step 0,1,2 into dyn_tend"""
    ctx._check(ctx.lib.mpas_atm_srk3(ctx.h, float(dt), int(schedule)), "atm_srk3")


def atm_timestep(ctx, dt):
    """rk_timestep.rg:503"""
    ctx._check(ctx.lib.mpas_atm_timestep(ctx.h, float(dt)), "atm_timestep")


def atm_do_timestep(ctx, dt):
    """atm_core.rg:46; the physics stubs (atm_core.rg:64-65) write nothing the dynamics reads"""
    atm_timestep(ctx, dt)


__all__ = [n for n in dir() if n.startswith("atm_")] + ["mpas_reconstruct_2d", "summarize_timestep", "MpasError"]
