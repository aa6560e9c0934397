"""Algorithmic bytes (B_alg) per task launch, SURVEY §8.5:

    B_alg = sum over the distinct arrays a task reads as inputs (once each)
          + sum over the distinct arrays it writes (once each)

3-D fp64 arrays count 8*n_entity*nVertLevels, C3V arrays the components a task reads
(zb_cell/zb3_cell: the nEdgesOnCell = 6 edge slots of a hexagon of their 10), 2-D mesh
arrays their stored bytes.  The read/write sets are the active-branch subsets of each Regent task's
privilege clause (dynamics_tasks.rg), without per-task scratch (flux_arr, ru_edge_w,
wduz, q, wdwz, wdtz, u_mix) and without arrays the task itself writes before reading
(their re-reads are implementation traffic, not algorithmic bytes).  Vertical 1-D
arrays are negligible and omitted.  This is the figure the benchmark's
roofline.achieved divides by the measured launch time.
"""

# name -> (reads, writes); each a list of field names of the registry
def _sets(task, rk_step=0, small_step=1, reconstruct_v=False, physics=0, damp=False, fused=False, sml=False,
          part=None, pair=None, copy=False, noA=False, defer_out=False, store_v=False, wold=True, smls=False,
          ddx=False, ntu=False, live=False, nst=False, navg=False, save=False, nww=False, ru=False,
          rudone=False, nbc=False, norz=False, smle=False):
    md = physics == 2  # the MPAS dynamics (include/mpas_dyn.h option physics = 2)
    if task == "hfuse":  # option hfuse: independent kernels of the step in one launch
        e, vi, dA = ("atm_compute_solve_diagnostics", {"part": "e"}), ("atm_compute_vert_imp_coefs", {}), \
            ("atm_compute_dyn_tend_work", {"rk_step": 1, "part": "A"})
        parts = {"damp+solve_vc": (("atm_divergence_damping_3d", {}), ("atm_compute_solve_diagnostics", {"part": "vc"})),
                 "solve_e+finish": (("atm_compute_solve_diagnostics", {"part": "e", "reconstruct_v": True}),
                                    ("atm_rk_dynamics_substep_finish", {})),
                 "solve_e-v+finish": (("atm_compute_solve_diagnostics", {"part": "e"}),
                                      ("atm_rk_dynamics_substep_finish", {})),
                 "solve_e+finish-rz": (("atm_compute_solve_diagnostics", {"part": "e", "reconstruct_v": True}),
                                       ("atm_rk_dynamics_substep_finish", {"norz": True})),
                 "solve_e-v+finish-rz": (("atm_compute_solve_diagnostics", {"part": "e"}),
                                         ("atm_rk_dynamics_substep_finish", {"norz": True})),
                 "solve_e+vert_imp": (e, vi),
                 "acoustic+solve_vc": (("atm_advance_acoustic_step_work", {"small_step": 1, "damp": True, "wold": False,
                                                                           "ddx": ddx}),
                                       ("atm_compute_solve_diagnostics", {"part": "vc"})),
                 "acoustic-st+solve_vc": (("atm_advance_acoustic_step_work", {"small_step": 1, "damp": True,
                                                                              "wold": False, "ddx": ddx, "nst": True}),
                                          ("atm_compute_solve_diagnostics", {"part": "vc", "live": True})),
                 "solve_e+dyn_A": (e, dA),
                 "solve_e+vert_imp+dyn_A": (e, vi, dA),
                 "setup+dyn_A": (("atm_rk_integration_setup", {"fused": True, "copy": True}),
                                 ("atm_compute_dyn_tend_work", {"rk_step": 0, "part": "A"})),
                 "setup+dyn_A+sml_flux": (("atm_rk_integration_setup", {"fused": True, "copy": True}),
                                          ("atm_compute_dyn_tend_work", {"rk_step": 0, "part": "A"}),
                                          ("atm_set_smlstep_pert_variables_work", {"part": "flux"}))}[pair]
        rs, ws = [], []
        for t, kw in parts:
            r, w = _sets(t, **kw)
            rs += r
            ws += w
        return rs, ws
    if task == "atm_rk_integration_setup" and fused:  # option fusesetup: + moist + vert_imp, one launch
        parts = [_sets(t, physics=physics) for t in ("atm_rk_integration_setup", "atm_compute_moist_coefficients",
                                                     "atm_compute_vert_imp_coefs")]
        writes = sorted(set(w for _, ws in parts for w in ws))
        reads = sorted(set(r for rs, _ in parts for r in rs) - set(writes) | {"gamma_tri"})
        if copy:  # option fusecopy: the edge copies ru_save = ru, u_2 = u moved to dyn_tend
            reads = [r for r in reads if r not in ("ru", "u")]
            writes = [w for w in writes if w not in ("ru_save", "u_2")]
        if nbc:  # option ntu: stage 0's b_tri / c_tri are dead (stage 1's vert_imp rewrites them)
            writes = [w for w in writes if w not in ("b_tri", "c_tri")]
        return reads, writes
    if task == "atm_rk_integration_setup":
        return (["rho_p", "rho_zz", "rtheta_p", "rw", "theta_m", "w", "ru", "u"],
                ["rho_p_save", "rho_zz_2", "rho_zz_old_split", "rtheta_p_save", "rw_save", "theta_m_2", "w_2",
                 "ru_save", "u_2"] + (["theta_m_save"] if md else []))
    if task == "atm_compute_moist_coefficients":
        return [], ["qtot", "cqw"] + (["cqu"] if md else [])
    if task == "atm_compute_vert_imp_coefs":
        return (["cqw", "exner", "exner_base", "qtot", "rho_base", "rtheta_base", "rtheta_p", "theta_m", "zz",
                 "gamma_tri"],
                ["a_tri", "b_tri", "c_tri", "alpha_tri", "gamma_tri", "coftz", "cofwr", "cofwt", "cofwz"])
    if task == "atm_compute_dyn_tend_work" and part == "A":  # its first cell kernel alone
        reads = ["ru", "rw", "rho_zz", "uReconstructZonal", "uReconstructMeridional", "nEdgesOnCell", "edgesOnCell",
                 "edgesOnCell_sign", "dvEdge", "invAreaCell", "lat"]
        if rk_step == 0:  # + the Smagorinsky kdiff, tend_rho and dpdz
            return (reads + ["u", "v", "defc_a", "defc_b", "qtot", "rho_base", "rho_p_save", "tend_rho_physics"],
                    ["h_divergence", "kdiff", "tend_rho", "dpdz"])
        return reads, ["h_divergence"]
    if task == "atm_compute_dyn_tend_work" and noA:  # the rest after A ran in a combined launch
        r, w = _sets(task, rk_step=rk_step, physics=physics, copy=copy, defer_out=defer_out, store_v=store_v, ntu=ntu)
        ra, wa = _sets(task, rk_step=rk_step, part="A")
        return ([x for x in r if x not in ("uReconstructZonal", "uReconstructMeridional")] + wa,
                [x for x in w if x not in wa])
    if task == "atm_compute_dyn_tend_work":
        mesh = ["nEdgesOnCell", "edgesOnCell", "edgesOnCell_sign", "invAreaCell", "lat", "cellsOnEdge",
                "verticesOnEdge", "dvEdge", "invDcEdge", "nEdgesOnEdge", "edgesOnEdge", "weightsOnEdge",
                "nAdvCellsForEdge", "advCellsForEdge", "adv_coefs", "adv_coefs_3rd", "angleEdge", "latEdge"]
        if rk_step == 0:
            mesh += ["defc_a", "defc_b", "dcEdge", "invDvEdge", "meshScalingDel2", "meshScalingDel4",
                     "edgesOnVertex", "edgesOnVertex_sign", "invAreaTriangle"]
            reads = ["cqw", "divergence", "ke", "pressure_p", "qtot", "rho_base", "rho_zz", "rho_p_save",
                     "rt_diabatic_tend", "rw", "rw_save", "tend_rho_physics", "tend_rtheta_physics", "theta_m",
                     "theta_m_save", "uReconstructZonal", "uReconstructMeridional", "w", "zz",
                     "cqu", "pv_edge", "rho_edge", "ru", "tend_ru_physics", "u", "v", "zxu", "vorticity"]
            writes = ["rthdynten", "tend_rho", "tend_rtheta_adv", "delsq_divergence", "delsq_theta", "delsq_w",
                      "dpdz", "h_divergence", "kdiff", "tend_theta", "tend_theta_euler", "w", "tend_w_euler",
                      "delsq_u", "tend_u", "tend_u_euler", "delsq_vorticity"]
        else:
            reads = ["ke", "rho_zz", "rt_diabatic_tend", "rw", "rw_save", "tend_rtheta_physics", "theta_m",
                     "theta_m_save", "uReconstructZonal", "uReconstructMeridional", "w", "tend_w_euler",
                     "tend_theta_euler", "pv_edge", "rho_edge", "ru", "ru_save", "tend_ru_physics", "u",
                     "tend_u_euler"]
            writes = ["h_divergence", "w", "tend_theta", "tend_rtheta_adv", "rthdynten", "tend_u"]
        if md:  # the w tendency goes to tend_w; the curvature reads the reconstructed winds
            writes = [("tend_w" if x == "w" else x) for x in writes]
            reads += ["uReconstructZonal", "uReconstructMeridional", "w"]
        if copy:  # option fusecopy (stage 0): setup's ru_save = ru, u_2 = u (ru, u already read)
            writes = writes + ["ru_save", "u_2"]
        if ru:  # option mru (the MPAS dynamics): the first acoustic substep's ru_p, ruAvg from the final tend_u
            writes = writes + ["ru_p", "ruAvg"]
        if smle:  # option msml (the MPAS dynamics): the stage's set_smlstep in E (tend_w corrected in place)
            reads = reads + ["tend_u", "zb_cell", "zb3_cell", "zz", "bdyMaskCell"]
        if store_v:  # option vdyn (stage 2): solve_diagnostics' v from the gathered edgesOnEdge u
            writes = writes + ["v"]
        if defer_out and rk_step == 0:  # option defer4: tend_u of this call is dead and not stored
            writes = [x for x in writes if x != "tend_u"]  # (its del4 runs in the next call: no credit taken)
        if ntu and not md:
            # option ntu (atm_srk3, a stage before the step's last): the call's tend_u and theta tendencies
            # are dead and not formed -- no credit for them nor for the arrays only they read (B's tend_u
            # terms and flux, E's theta advection and wdtz); at rk_step > 0 no A either (its h_divergence
            # feeds only that tend_u) and B only applies the deferred del4 (no credit, as defer4's)
            dead_w = {"tend_u", "tend_theta", "tend_rtheta_adv", "rthdynten", "h_divergence"}  # (h_divergence: tend_u's)
            dead_r = {"pv_edge", "tend_ru_physics", "ke", "w", "rw_save", "theta_m_save", "rt_diabatic_tend",
                      "tend_rtheta_physics", "ru_save", "nEdgesOnEdge", "edgesOnEdge", "weightsOnEdge", "angleEdge",
                      "latEdge", "nAdvCellsForEdge", "advCellsForEdge", "adv_coefs", "adv_coefs_3rd"}
            if rk_step != 0:
                dead_r |= {"u", "rho_edge", "theta_m", "tend_theta_euler", "tend_u_euler", "cellsOnEdge",
                           "verticesOnEdge", "dvEdge", "invDcEdge"}
            writes = [x for x in writes if x not in dead_w]
            reads = [x for x in reads if x not in dead_r]
            mesh = [x for x in mesh if x not in dead_r]
        return reads + mesh, writes
    if task == "atm_set_smlstep_pert_variables_work" and part == "flux":
        # option smlsum (atm_srk3 fast path): the slope-flux sum, once per step (X_smlS, scratch)
        # (+ X_Dd = rw_save - rw for the stages' acoustic launches: rw_save and rw read here once)
        return ["zb_cell", "zb3_cell", "u_tend", "nEdgesOnCell", "edgesOnCell", "edgesOnCell_sign", "rw_save", "rw"], []
    if task == "atm_set_smlstep_pert_variables_work":
        if md:
            return (["zz", "tend_w", "zb_cell", "zb3_cell", "tend_u", "bdyMaskCell", "nEdgesOnCell", "edgesOnCell",
                     "edgesOnCell_sign"], ["tend_w"])
        return (["zz", "w", "zb_cell", "zb3_cell", "u_tend", "cprMask", "bdyMaskCell", "nEdgesOnCell",
                 "edgesOnCell", "edgesOnCell_sign"], ["w"])
    if task == "atm_advance_acoustic_step_work":
        reads = ["a_tri", "alpha_tri", "coftz", "cofwr", "cofwt", "cofwz", "dss", "rho_zz", "rw", "rw_save",
                 "tend_rho", "theta_m", "w", "zz", "ru_p", "nEdgesOnCell", "edgesOnCell", "edgesOnCellSign",
                 "invAreaCell", "cellsOnEdge", "dvEdge", "specZoneMaskCell"]
        if small_step != 0:
            reads += ["rho_pp", "rtheta_pp", "rw_p", "wwAvg"]
        if ddx and not physics:  # (atm_srk3 with smlsum: rw_save - rw from the step's X_Dd, scratch)
            reads = [r for r in reads if r not in ("rw", "rw_save")]
        # (wold False: a fused launch of option fusedamp other than the step's last, which leaves
        # rtheta_pp_old unwritten -- the fused damping reads the stored div instead)
        writes = (["rtheta_pp_old"] if wold else []) + ["rho_pp", "rtheta_pp", "rw_p", "wwAvg"]
        if nww:  # option ntu, the MPAS forms: a stage's last substep before the last -- its wwAvg is dead
            writes = [w for w in writes if w != "wwAvg"]
            reads = [r for r in reads if r != "wwAvg"]
        if nst:  # option ntu: a stage's last substep before the last stage -- its acoustic state is dead
            writes = [w for w in writes if w not in ("rho_pp", "rtheta_pp", "rw_p", "wwAvg")]
            reads = [r for r in reads if r != "wwAvg"]  # (read only for the dead wwAvg)
        if physics:  # the MPAS form (option physics = 1): the ru_p / ruAvg update of :1581-1613
            reads += ["tend_theta", "c_tri", "gamma_tri", "specZoneMaskEdge"]
            if not rudone:  # (option mru: the first substep's ru_p / ruAvg stored by dyn_tend)
                reads += ["tend_u"]
                writes += ["ru_p", "ruAvg"]
            if small_step != 0:
                reads += ["ru_p", "ruAvg", "exner", "cqu", "zxu", "invDcEdge"]
        if damp:  # option fusedamp: the previous substep's atm_divergence_damping_3d applied here
            reads += ["rtheta_pp", "rtheta_pp_old", "isShared", "specZoneMaskEdge"]
            writes += ["ru_p"]
        if sml and smls:  # option smlsum: set_smlstep from the step's flux sum (X_smlS, scratch)
            reads += ["zz", "w", "cprMask", "bdyMaskCell"]
            writes += ["w"]
        elif sml:  # option fusesml: the stage's atm_set_smlstep_pert_variables_work first
            r2, w2 = _sets("atm_set_smlstep_pert_variables_work", physics=physics)
            reads += r2
            writes += w2
        return reads, writes
    if task == "atm_divergence_damping_3d":
        return (["rtheta_pp", "rtheta_pp_old", "theta_m", "ru_p", "cellsOnEdge", "isShared", "specZoneMaskEdge"],
                ["ru_p"])
    if task == "atm_compute_solve_diagnostics" and part == "vc" and live:  # (ntu: ke, pv_vertex alone)
        return (["u", "dcEdge", "dvEdge", "edgesOnCell", "edgesOnCellSign", "invAreaCell", "nEdgesOnCell",
                 "edgesOnVertex", "edgesOnVertexSign", "fVertex", "invAreaTriangle"], ["ke", "pv_vertex"])
    if task == "atm_compute_solve_diagnostics" and part == "vc":  # its vertex / cell kernel alone
        return (["u", "dcEdge", "dvEdge", "edgesOnCell", "edgesOnCellSign", "invAreaCell", "nEdgesOnCell",
                 "edgesOnVertex", "edgesOnVertexSign", "fVertex", "invAreaTriangle"],
                ["divergence", "ke", "vorticity", "pv_vertex"])
    if task == "atm_compute_solve_diagnostics" and part == "e":  # its edge kernel alone
        reads = ["h", "u", "pv_vertex", "cellsOnEdge", "verticesOnEdge", "dcEdge", "dvEdge"]
        writes = ["h_edge", "ke_edge", "pv_edge"]
        if reconstruct_v:
            reads += ["edgesOnEdge_ECP", "nEdgesOnEdge", "weightsOnEdge"]
            writes.append("v")
        return reads, writes
    if task == "atm_compute_solve_diagnostics" and live:
        # option ntu (stage 1's call, the last stage at rk_step > 0): the diagnostics that stage's dyn_tend
        # reads, alone -- ke, pv_edge (pv_vertex, read back by the edge kernel); no credit for the dead
        # h_edge, ke_edge, divergence, vorticity nor for h, which only h_edge reads
        # (the MPAS forms: also rho_edge = h_edge, from rho_zz; stage 0's call too)
        return (["u", "cellsOnEdge", "dcEdge", "dvEdge", "verticesOnEdge", "edgesOnCell", "edgesOnCellSign",
                 "invAreaCell", "nEdgesOnCell", "edgesOnVertex", "edgesOnVertexSign", "fVertex", "invAreaTriangle"]
                + (["rho_zz"] if md else []), ["pv_edge", "ke", "pv_vertex"] + (["rho_edge"] if md else []))
    if task == "atm_compute_solve_diagnostics":
        writes = ["h_edge", "ke_edge", "pv_edge", "divergence", "ke", "vorticity", "pv_vertex"]
        if reconstruct_v:
            writes.append("v")
        if md:
            writes.append("rho_edge")
        return (["rho_zz" if md else "h", "u", "cellsOnEdge", "dcEdge", "dvEdge", "edgesOnEdge_ECP", "nEdgesOnEdge", "verticesOnEdge",
                 "weightsOnEdge", "edgesOnCell", "edgesOnCellSign", "invAreaCell", "nEdgesOnCell", "edgesOnVertex",
                 "edgesOnVertexSign", "fVertex", "invAreaTriangle"], writes)
    if task == "atm_recover_large_step_variables_work":  # (:1766-1872; rk_step 2 adds the exner part)
        reads = ["rho_p_save", "rho_pp", "rho_base", "wwAvg", "rw_save", "rw_p", "zz", "rtheta_p_save", "rtheta_pp",
                 "rtheta_base", "ruAvg", "ru_save", "ru_p", "zb_cell", "zb3_cell", "edgesOnCell", "edgesOnCell_sign",
                 "nEdgesOnCell", "cellsOnEdge", "bdyMaskCell"]
        writes = ["rho_p", "rho_zz", "wwAvg", "rw", "w", "rtheta_p", "theta_m", "ruAvg", "ru", "u"]
        if rk_step == 2:
            reads += ["rt_diabatic_tend", "exner_base"]
            writes += ["exner", "pressure_p"]
        if damp:  # option mdamp: the stage's last divergence damping in the edge kernel (ru_p updated in place)
            reads += ["rtheta_pp", "rtheta_pp_old", "theta_m", "isShared", "specZoneMaskEdge"]
            writes += ["ru_p"]
        if navg:  # option ntu, a stage before the last: the averages are dead (the next stage's first substep sets
            # them), and so is a damped ru_p (the next stage's first substep sets it from tend_u), rho_p (read
            # by setup only) and, after stage 1, rtheta_p (read by stage 1's vert_imp only)
            reads = [r for r in reads if r not in ("wwAvg", "ruAvg")]
            writes = [w for w in writes if w not in ("wwAvg", "ruAvg", "ru_p", "rho_p")
                      and not (w == "rtheta_p" and rk_step == 1)]
        return reads, writes
    if task == "atm_rk_dynamics_substep_finish":
        # (:1951-2007 with dynamics_substep = dynamics_split = 1, as atm_srk3 calls it: the
        # averages are copied to the *_split fields and divided by 1 -- the kernel stores no
        # unchanged average (no credit for bytes not moved); rho_zz = rho_zz_old_split in the
        # reference semantics, kept under the MPAS dynamics)
        if md or norz:  # (norz, option ntu: rho_zz = rho_zz_old_split is the identity in atm_srk3 -- not made)
            return ["wwAvg", "ruAvg"], ["wwAvg_split", "ruAvg_split"]
        return ["wwAvg", "rho_zz_old_split", "ruAvg"], ["wwAvg_split", "rho_zz", "ruAvg_split"]
    if task == "atm_advance_scalars_mono":  # k_transport.hip (Q26: MPAS-A's, not the reference's)
        # (save, option trsave: scalars_save folded in -- the old values read from scalars, scalars_old stored)
        return (["scalars" if save else "scalars_old", "ruAvg", "wwAvg", "rho_zz_old_split", "rho_zz", "cellsOnEdge",
                 "advCellsForEdge", "nAdvCellsForEdge", "adv_coefs", "adv_coefs_3rd", "dvEdge", "edgesOnCell",
                 "nEdgesOnCell", "invAreaCell"], ["scalars"] + (["scalars_old"] if save else []))
    if task == "scalars_save":  # srk3 with transport: scalars_old = scalars
        return ["scalars"], ["scalars_old"]
    if task == "mpas_reconstruct_2d":
        return (["u", "coeffs_reconstruct", "edgesOnCell", "nEdgesOnCell", "lat", "lon"],
                ["uReconstructX", "uReconstructY", "uReconstructZ", "uReconstructZonal", "uReconstructMeridional"])
    raise KeyError(task)


def field_bytes(name, nCells, nEdges, nVertices, L):
    from .registry import BY_NAME
    f = BY_NAME[name]
    n = {"cell": nCells, "edge": nEdges, "vertex": nVertices, None: 0}[f.entity]
    if f.kind in ("C3", "E3", "V3"):
        return 8 * n * L
    if f.kind == "C3V":
        return 8 * n * L * f.width
    if f.kind == "C3B":
        return n * L
    if f.kind == "ZV":
        return 0
    return n * f.width * (4 if f.kind.endswith("I") else 8)


# C3V arrays indexed by a cell's edge slot (zb_cell / zb3_cell: one component per
# edgesOnCell entry): the tasks read nEdgesOnCell of their 10 components, 6 on the
# hexagons of an x1 mesh (5 on its 12 pentagons)
SLOT_FIELDS = {"zb_cell", "zb3_cell"}
SLOTS_READ = 6


def b_alg(task, dims, **kw):
    """algorithmic bytes of one launch of `task` at dims = (nCells, nEdges, nVertices, L)"""
    reads, writes = _sets(task, **kw)

    def fb(x):
        b = field_bytes(x, *dims)
        return b * SLOTS_READ // 10 if x in SLOT_FIELDS else b
    return sum(fb(x) for x in set(reads)) + sum(fb(x) for x in set(writes))


def step_schedule(schedule=1, physics=0, transport=0, fusedamp=False, fusesetup=False, fusesml=False,
                  fusecopy=False, defer4=False, smlsum=False, ntu=False, mdamp=False, trsave=False, mru=False,
                  msml=False):
    """(task, kwargs, launches) of one atm_srk3 step (rk_timestep.rg:404-481); physics = 1
    (the MPAS vertical solver): number_sub_steps acoustic substeps (4 per step) and
    recover after each stage; transport = 1 adds the scalar save and the transport;
    fusedamp (reference semantics): six of the seven dampings run inside the next acoustic
    launch; fusecopy (with fusesetup): setup's edge copies in stage 0's dyn_tend"""
    copy = bool(fusesetup and fusecopy)
    if physics:
        p = {"physics": physics}
        if fusesetup:  # stage 0's setup + moist + vert_imp in one launch (MPAS forms)
            out = [("atm_rk_integration_setup", {"fused": True, "copy": copy, "nbc": bool(ntu), **p}, 1),
                   ("atm_compute_vert_imp_coefs", {}, 1)]
        else:
            out = [("atm_rk_integration_setup", p, 1), ("atm_compute_moist_coefficients", p, 1),
                   ("atm_compute_vert_imp_coefs", {}, 2)]
        r = {"ru": True} if mru else {}  # (option mru: the first substep's ru_p / ruAvg stored by dyn_tend)
        if msml and physics == 2:  # (option msml: each stage's set_smlstep in dyn_tend's E)
            r = dict(r, smle=True)
        if schedule == 1:
            out += [("atm_compute_dyn_tend_work", {"rk_step": 0, "copy": copy, **p, **r}, 1),
                    ("atm_compute_dyn_tend_work", {"rk_step": 1, **p, **r}, 2)]
        # (option mdamp: each damping applied by the next kernel that reads ru_p -- the next substep's
        # ru_p kernel or the stage's recover)
        d = {"damp": bool(mdamp)}
        out += [("atm_set_smlstep_pert_variables_work", p, 0 if (msml and physics == 2) else 3),
                ("atm_advance_acoustic_step_work", {"small_step": 0, "physics": 1, "rudone": bool(mru)}, 1 if ntu else 3),
                ("atm_advance_acoustic_step_work", {"small_step": 0, "physics": 1, "nww": True, "rudone": bool(mru)},
                 2 if ntu else 0),
                ("atm_advance_acoustic_step_work", {"small_step": 1, "physics": 1, **d}, 1),
                ("atm_divergence_damping_3d", {}, 0 if mdamp else 4),
                ("atm_recover_large_step_variables_work", {"rk_step": 0, "navg": bool(ntu), **d}, 1),
                ("atm_recover_large_step_variables_work", {"rk_step": 1, "navg": bool(ntu), **d}, 1),
                ("atm_recover_large_step_variables_work", {"rk_step": 2, **d}, 1),
                ("atm_compute_solve_diagnostics", {"live": bool(ntu), **p}, 2),
                ("atm_compute_solve_diagnostics", {"reconstruct_v": True, **p}, 1),
                ("atm_rk_dynamics_substep_finish", p, 1)]
        if physics == 2:
            out.append(("mpas_reconstruct_2d", {}, 1))
        if transport and trsave:  # (option trsave: scalars_save folded into the transport)
            out += [("atm_advance_scalars_mono", {"save": True}, 1)]
        elif transport:
            out += [("scalars_save", {}, 1), ("atm_advance_scalars_mono", {}, 1)]
        return out
    if fusesetup:
        out = [("atm_rk_integration_setup", {"fused": True, "copy": copy, "nbc": bool(ntu)}, 1),
               ("atm_compute_vert_imp_coefs", {}, 1)]
    else:
        out = [("atm_rk_integration_setup", {}, 1), ("atm_compute_moist_coefficients", {}, 1),
               ("atm_compute_vert_imp_coefs", {}, 2)]
    if schedule == 1:
        out += [("atm_compute_dyn_tend_work", {"rk_step": 0, "copy": copy, "defer_out": defer4, "ntu": bool(ntu)}, 1),
                ("atm_compute_dyn_tend_work", {"rk_step": 1, "ntu": bool(ntu)}, 1),
                ("atm_compute_dyn_tend_work", {"rk_step": 1}, 1)]
    # (fusedamp: only the step's last acoustic launch stores rtheta_pp_old, wold)
    if fusedamp and fusesml:
        sm = {"sml": True, "smls": bool(smlsum)}
        dd = {"ddx": bool(smlsum)}  # (smlsum: rw_save - rw from the step's X_Dd too)
        if smlsum:  # option smlsum: the slope-flux sum once per step
            out += [("atm_set_smlstep_pert_variables_work", {"part": "flux"}, 1)]
        out += [("atm_advance_acoustic_step_work", {"small_step": 0, **sm, "wold": False, **dd}, 1),
                ("atm_advance_acoustic_step_work", {"small_step": 0, "damp": True, **sm, "wold": False, **dd}, 2),
                ("atm_advance_acoustic_step_work", {"small_step": 1, "damp": True, "wold": False, **dd}, 1 if ntu else 3),
                ("atm_advance_acoustic_step_work", {"small_step": 1, "damp": True, **dd}, 1),
                ("atm_divergence_damping_3d", {}, 1)]
    elif fusedamp:
        out += [("atm_set_smlstep_pert_variables_work", {}, 3),
                ("atm_advance_acoustic_step_work", {"small_step": 0, "wold": False}, 1),
                ("atm_advance_acoustic_step_work", {"small_step": 0, "damp": True, "wold": False}, 2),
                ("atm_advance_acoustic_step_work", {"small_step": 1, "damp": True, "wold": False}, 1 if ntu else 3),
                ("atm_advance_acoustic_step_work", {"small_step": 1, "damp": True}, 1),
                ("atm_divergence_damping_3d", {}, 1)]
    else:
        out += [("atm_set_smlstep_pert_variables_work", {}, 3),
                ("atm_advance_acoustic_step_work", {"small_step": 0}, 3),
                ("atm_advance_acoustic_step_work", {"small_step": 1}, 4),
                ("atm_divergence_damping_3d", {}, 7)]
    # (option ntu: the last substep of stages 0 and 1 stores no acoustic state; stage 0's
    # solve_diagnostics is dead and not run, stage 1's stores what stage 2 reads)
    if ntu and fusedamp:
        out += [("atm_advance_acoustic_step_work", {"small_step": 1, "damp": True, "wold": False, "nst": True,
                                                    "ddx": bool(fusesml and smlsum)}, 2)]
    out += [
            ("atm_compute_solve_diagnostics", {"live": True} if ntu else {}, 1 if ntu else 2),
            ("atm_compute_solve_diagnostics", {"reconstruct_v": True}, 1),
            ("atm_rk_dynamics_substep_finish", {"norz": bool(ntu)}, 1)]
    return out


def b_alg_step(dims, schedule=1, physics=0, transport=0, fusedamp=False, fusesetup=False, fusesml=False,
               fusecopy=False, defer4=False, smlsum=False, ntu=False, mdamp=False, trsave=False, mru=False,
               msml=False):
    return sum(b_alg(t, dims, **kw) * n for t, kw, n in step_schedule(schedule, physics, transport, fusedamp,
                                                                        fusesetup, fusesml, fusecopy, defer4,
                                                                        smlsum, ntu, mdamp, trsave, mru, msml))
