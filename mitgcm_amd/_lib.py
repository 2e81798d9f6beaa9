"""ctypes binding of the C-ABI (include/mitgcm_amd.h) -> mitgcm_amd/libmitgcm_amd.so.

The product path has no CPU fallback: if the library is missing or no HIP
device is visible, the calls below raise.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MGCM_LIB: a diagnostic build of the same library (e.g. tools/cg_stamps.sh) -- never the default
LIBPATH = os.environ.get("MGCM_LIB") or os.path.join(HERE, "libmitgcm_amd.so")
_lib = None


class MgcmError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIBPATH):
        raise MgcmError("libmitgcm_amd.so not built (run __graft_entry__.build() or "
                        "python mitgcm_amd/build.py): the MI355X path has no CPU fallback")
    L = ctypes.CDLL(LIBPATH)
    vp, ci, cd, cs, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_char_p, ctypes.c_long
    PD, PI, PL = ctypes.POINTER(cd), ctypes.POINTER(ci), ctypes.POINTER(cl)
    sig = {
        "mgcm_create": (vp, [ci] * 8),
        "mgcm_destroy": (None, [vp]),
        "mgcm_last_error": (cs, []),
        "mgcm_set_param": (ci, [vp, cs, cd]),
        "mgcm_set_iter": (ci, [vp, ci]),
        "mgcm_add_iter": (ci, [vp, ci]),
        "mgcm_exch2_maps": (ci, [ci] * 6 + [PI] * 16 + [ci] + [PL] * 5),
        "mgcm_tracer_parity": (ci, [vp, ci]),
        "mgcm_get_param": (cd, [vp, cs]),
        "mgcm_put": (ci, [vp, cs, PD, cl]),
        "mgcm_put_async": (ci, [vp, cs, PD, cl]),
        "mgcm_put_batch_async": (ci, [vp, ctypes.c_int, ctypes.POINTER(cs), ctypes.POINTER(PD), ctypes.POINTER(cl)]),
        "mgcm_get": (ci, [vp, cs, PD, cl]),
        "mgcm_device_ptr": (vp, [vp, cs]),
        "mgcm_set_halo_map": (ci, [vp, PL, cl]),
        "mgcm_set_uv_map": (ci, [vp, PL, PL, PL, PL, PI, PI, cl]),
        "mgcm_init": (ci, [vp]),
        "mgcm_dynamics": (ci, [vp]),
        "mgcm_thermodynamics": (ci, [vp]),
        "mgcm_prepare": (ci, [vp]),
        "mgcm_solve_for_pressure": (ci, [vp]),
        "mgcm_momentum_correction_step": (ci, [vp]),
        "mgcm_integr_continuity": (ci, [vp]),
        "mgcm_blocking_exchanges": (ci, [vp]),
        "mgcm_forward_step": (ci, [vp, ci]),
        "mgcm_sync": (ci, [vp]),
        "mgcm_cg2d": (ci, [vp, PD, PD, PD, PD, PD, PI, PI]),
        "mgcm_cg2d_sum_plan": (ci, [vp, PI, cl, PI, PI, PI]),
        "mgcm_solve_stats": (ci, [vp, ci, PD, PD, PI, PD]),
        "mgcm_solve_minres": (ci, [vp, ci, PD, PI]),
        "mgcm_stream_triad": (ci, [ci, cl, ci, PD]),
        "mgcm_solve_history": (ci, [vp, ci, PI, PD, PD]),
        "mgcm_monitor": (ci, [vp, PD]),
        "mgcm_kernel_ms": (cd, [vp, cs, PI]),
        "mgcm_kernel_timing": (None, [vp, ci]),
        "mgcm_set_tile_range": (ci, [vp, ci, ci]),
        "mgcm_set_stream": (ci, [vp, vp]),
        "mgcm_exchange_nfields": (ci, [vp]),
        "mgcm_halo_pack": (ci, [vp, vp, cl, vp, ci]),
        "mgcm_halo_pack_group": (ci, [vp, ci, vp, cl, vp, ci]),
        "mgcm_exchange_nfields_group": (ci, [vp, ci]),
        "mgcm_stream_handoff": (ci, [vp, vp, ci]),
        "mgcm_begin_steps": (ci, [vp]),
        "mgcm_end_steps": (ci, [vp, ci]),
        "mgcm_cg2d_shared_bytes": (ci, [vp]),
        "mgcm_cg2d_shared_export": (ci, [vp, vp]),
        "mgcm_cg2d_shared_import": (ci, [vp, vp]),
        "mgcm_tile_copy": (ci, [vp, cs, ci, ci, vp, ci]),
        "mgcm_step_phase": (ci, [vp, ci]),
        "mgcm_cg2d_op": (ci, [vp, ci, cd, vp]),
        "mgcm_cg2d_record": (ci, [vp, cd, cd, cd, cd, ci, cd, ci]),
        "mgcm_field_pack": (ci, [vp, cs, vp, cl, vp, ci]),
        "mgcm_exchange_field": (ci, [vp, cs]),
        "mgcm_oceanic_phys": (ci, [vp]),
        "mgcm_tracer_step": (ci, [vp]),
        "mgcm_stagger_exchanges": (ci, [vp]),
        "mgcm_exchange_host": (ci, [vp, PD, PD, ci, ci, ci]),
        "mgcm_field_count": (cl, [vp, cs]),
        "mgcm_param_name": (cs, [ci]),
        "mgcm_update_r_star": (ci, [vp]),
        "mgcm_calc_r_star": (ci, [vp]),
        "mgcm_get_stream": (vp, [vp]),
        "mgcm_halo_sources": (cl, [vp, ci, ci, PL, cl]),
        "mgcm_cg2d_tiles": (ci, [vp, ci, ci]),
        "mgcm_cg2d_share": (ci, [vp, vp]),
        "ini_cg2d_amd_": (None, [PI] * 6 + [PD] * 8 + [PI]),
        "cg2d_amd_": (None, [PD, PD, PD, PD, PD, PI, PI, PI]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


EXPORTS = ["mgcm_create", "mgcm_destroy", "mgcm_last_error", "mgcm_set_param", "mgcm_get_param", "mgcm_put", "mgcm_put_async", "mgcm_put_batch_async",
           "mgcm_get", "mgcm_device_ptr", "mgcm_set_halo_map", "mgcm_set_uv_map", "mgcm_init", "mgcm_dynamics", "mgcm_thermodynamics",
           "mgcm_solve_for_pressure", "mgcm_momentum_correction_step", "mgcm_integr_continuity",
           "mgcm_blocking_exchanges", "mgcm_prepare", "mgcm_forward_step", "mgcm_sync", "mgcm_cg2d", "mgcm_cg2d_sum_plan", "mgcm_solve_stats", "mgcm_solve_minres", "mgcm_stream_triad", "mgcm_solve_history", "mgcm_monitor",
           "mgcm_kernel_ms", "mgcm_kernel_timing", "mgcm_set_tile_range", "mgcm_set_stream",
           "mgcm_exchange_nfields", "mgcm_halo_pack", "mgcm_tile_copy", "mgcm_begin_steps", "mgcm_step_phase", "mgcm_cg2d_op",
           "mgcm_cg2d_record", "mgcm_field_pack", "mgcm_exchange_field", "ini_cg2d_amd_",
           "cg2d_amd_", "mgcm_oceanic_phys", "mgcm_tracer_step", "mgcm_stagger_exchanges", "mgcm_exchange_host", "mgcm_field_count", "mgcm_param_name",
           "mgcm_amd_setup_", "mgcm_amd_param_", "mgcm_amd_bind_", "mgcm_amd_init_", "do_oceanic_phys_amd_",
           "thermodynamics_amd_", "dynamics_amd_", "solve_for_pressure_amd_", "momentum_correction_step_amd_",
           "integr_continuity_amd_", "do_fields_blocking_exchanges_amd_", "do_stagger_fields_exchanges_amd_", "exch_xy_rl_amd_", "exch_xyz_rl_amd_",
           "exch_uv_xy_rl_amd_", "exch_uv_xyz_rl_amd_", "global_sum_tile_rl_amd_",
           "mgcm_update_r_star", "mgcm_calc_r_star", "update_r_star_amd_", "update_cg2d_amd_", "calc_r_star_amd_",
           "mgcm_set_iter", "mgcm_add_iter", "mgcm_tracer_parity", "mgcm_exch2_maps", "mgcm_amd_host_sync_", "mgcm_amd_device_sync_", "mgcm_amd_transfer_stats_",
           "mgcm_amd_step_fence_", "mgcm_halo_pack_group", "mgcm_exchange_nfields_group", "mgcm_stream_handoff",
           "mgcm_end_steps", "mgcm_cg2d_shared_bytes", "mgcm_cg2d_shared_export", "mgcm_cg2d_shared_import",
           "mgcm_amd_set_maps_", "mgcm_amd_set_w2_", "mgcm_get_stream", "mgcm_halo_sources", "mgcm_cg2d_tiles", "mgcm_cg2d_share"]


def check(rc, what):
    if rc != 0:
        raise MgcmError("%s failed: %s" % (what, lib().mgcm_last_error().decode()))
