"""End-to-end run on the GPU, the reference's `main` (main.rg:47-76): mesh -> JW initial
state -> atm_core_init's one-time precompute -> time steps -> atm_compute_output_diagnostics
-> timestep_output.nc.

    python -m mpasdyn.driver [--grid x1.N.grid.nc] [--levels 26] [--steps 10] [--dt 720]
                             [--schedule 1] [--physics {0,1,2}] [--transport] [--day]
                             [--out timestep_output.nc]

Without --grid the reference's own x1.2562 mesh (tests/golden fixture) is used.  The mesh
is taken in mpas-mode (0-based) ids, the ids the JW state (mpasdyn/jw.py) is defined on.
`--schedule 0 --dt-from-step` reproduces main.rg's call literally: dt = the step index j
(Q3; j = 0 gives rdts = inf in the acoustic step, the reference's NaN).  Prints one line
per step with the reference's global min/max of w and u (summarize_timestep).
`--physics 2` runs the MPAS dynamics (every quirk of the path fixed, include/mpas_dyn.h):
the JW state then evolves as a dynamical core; the run starts from MPAS-A's initial
diagnostics (solve_diagnostics at rk_step -1 and the cell-centre winds, atm_core.rg:30-33)
and reports the surface pressure (min/max/mean, hPa) and the global dry mass after the
last step; `--day` sets the steps to one simulated day (86400 / dt)."""
import argparse
import os
import sys

import numpy as np


def run(m, L, steps, dt, schedule=1, physics=0, transport=False, dt_from_step=False, out=None, device=0,
        log=print):
    from . import build_state as bs
    from . import jw, lib
    from . import mesh as M
    from . import tasks as T
    if np.asarray(m.cellsOnEdge).min() != 0:
        m = M.zero_based(m)
    st = bs.build_state(m, L, "physical", vertical=False)
    jw.init_atm_case_jw(m, st)
    physics = int(physics) if physics else (1 if transport else 0)
    nC = m.nCells
    vol = 1.0 / (st["invAreaCell"][:nC, 0][:, None] * st["rdzw"][:L][None, :])
    mass0 = float(np.sum(st["rho_zz"][:nC, :L] * vol))
    with lib.Context(m.nCells, m.nEdges, m.nVertices, L, device=device) as ctx:
        ctx.set_option("physics", physics)
        ctx.set_option("transport", int(transport))
        ctx.upload(st)
        if physics == 2:  # MPAS-A's atm_core_init diagnostics of the initial state
            T.atm_compute_solve_diagnostics(ctx, False, -1)
            T.mpas_reconstruct_2d(ctx, False, True)
        for j in range(steps):
            T.atm_do_timestep(ctx, float(j) if dt_from_step else dt) if schedule == 0 else \
                T.atm_srk3(ctx, float(j) if dt_from_step else dt, schedule)
            s = T.summarize_timestep(ctx, False, True)
            log(f"step {j}: w in [{s[27]:.6g}, {s[28]:.6g}]  u in [{s[29]:.6g}, {s[30]:.6g}]")
        T.atm_compute_output_diagnostics(ctx)
        ctx.sync()
        ctx.download(st)
    if physics == 2:
        sp = st["surface_pressure"][:nC, 0] / 100.0
        mass = float(np.sum(st["rho_zz"][:nC, :L] * vol))
        log(f"after {steps} steps ({steps * dt / 3600.0:g} h): surface pressure [{sp.min():.4f}, {sp.max():.4f}] "
            f"mean {sp.mean():.6f} hPa; dry mass change {mass / mass0 - 1.0:.3e}")
    if out:
        from .meshio import write_output_plotting
        write_output_plotting(out, m, st)
    return st


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--grid")
    ap.add_argument("--levels", type=int, default=26)
    ap.add_argument("--steps", type=int, default=10)  # constants.NUM_TIMESTEPS
    ap.add_argument("--dt", type=float, default=720.0)
    ap.add_argument("--schedule", type=int, default=1)
    ap.add_argument("--dt-from-step", action="store_true")
    ap.add_argument("--physics", type=int, default=0, choices=[0, 1, 2])
    ap.add_argument("--day", action="store_true", help="one simulated day: steps = 86400 / dt")
    ap.add_argument("--transport", action="store_true")
    ap.add_argument("--out", default="timestep_output.nc")
    a = ap.parse_args(argv)
    from . import mesh as M
    if a.grid:
        from .meshio import read_grid
        m = read_grid(a.grid)
    else:
        m = M.load_x1_2562()
    steps = int(round(86400.0 / a.dt)) if a.day else a.steps
    run(m, a.levels, steps, a.dt, a.schedule, a.physics, a.transport, a.dt_from_step, a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
