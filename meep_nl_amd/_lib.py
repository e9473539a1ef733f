"""ctypes binding of libmnl.so (include/meep_nl_amd.h).

There is no CPU fallback: if the HIP library cannot be loaded, or there is no
HIP device, creating fields raises RuntimeError (the reference's meep.abort
maps to RuntimeError as in python/meep.i:1429-1441).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmnl.so")
if os.environ.get("MNL_LIB_VARIANT"):  # A/B experiments: meep_nl_amd/variants/<name>/libmnl.so
    LIB_PATH = os.path.join(_HERE, "variants", os.environ["MNL_LIB_VARIANT"], "libmnl.so")
_LIB = None

c_int, c_double, c_void, c_size = ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t
dptr = ctypes.POINTER(ctypes.c_double)
# custom_src_time callback (include/meep_nl_amd.h mnl_src_func)
SRC_FUNC = ctypes.CFUNCTYPE(None, ctypes.c_double, ctypes.c_void_p, dptr, dptr)
# volume-source amplitude function A(r) (include/meep_nl_amd.h mnl_amp_func)
AMP_FUNC = ctypes.CFUNCTYPE(None, dptr, ctypes.c_void_p, dptr, dptr)
iptr = ctypes.POINTER(ctypes.c_int)
llptr = ctypes.POINTER(ctypes.c_longlong)

_SIGS = {
    "mnl_last_error": (ctypes.c_char_p, []),
    "mnl_version": (c_int, []),
    "mnl_device_count": (c_int, [iptr]),
    "mnl_structure_create": (c_void, [c_int, iptr, c_double, c_double, iptr]),
    "mnl_structure_destroy": (None, [c_void]),
    "mnl_structure_add_pml": (c_int, [c_void, c_int, c_int, c_double, c_double, c_double]),
    "mnl_structure_set_chi1inv": (c_int, [c_void, c_int, c_int, dptr]),
    "mnl_structure_set_chi2": (c_int, [c_void, c_int, dptr]),
    "mnl_structure_set_chi3": (c_int, [c_void, c_int, dptr]),
    "mnl_structure_set_conductivity": (c_int, [c_void, c_int, dptr]),
    "mnl_structure_add_lorentzian_tensor": (c_int, [c_void, ctypes.c_double, ctypes.c_double,
                                                    c_int, ctypes.POINTER(dptr)]),
    "mnl_fields_add_custom_point_source": (c_int, [c_void, c_int, SRC_FUNC, ctypes.c_void_p,
                                                   ctypes.c_double, ctypes.c_double, dptr,
                                                   ctypes.c_double, ctypes.c_double, c_int]),
    "mnl_fields_add_volume_source": (c_int, [c_void, c_int, c_int, dptr, c_int, dptr, dptr,
                                             ctypes.c_double, ctypes.c_double, c_int, AMP_FUNC,
                                             ctypes.c_void_p]),
    "mnl_fields_add_custom_volume_source": (c_int, [c_void, c_int, SRC_FUNC, ctypes.c_void_p,
                                                    ctypes.c_double, ctypes.c_double, dptr, dptr,
                                                    ctypes.c_double, ctypes.c_double, c_int,
                                                    AMP_FUNC, ctypes.c_void_p]),
    "mnl_fields_dump": (c_int, [c_void, ctypes.c_char_p]),
    "mnl_fields_array_slice": (c_int, [c_void, c_int, dptr, dptr, c_int, ctypes.POINTER(c_int),
                                       ctypes.POINTER(ctypes.c_longlong), dptr, ctypes.c_longlong]),
    "mnl_fields_load": (c_int, [c_void, ctypes.c_char_p]),
    "mnl_structure_dump": (c_int, [c_void, ctypes.c_char_p]),
    "mnl_structure_load": (c_int, [c_void, ctypes.c_char_p]),
    "mnl_structure_add_lorentzian": (c_int, [c_void, c_double, c_double, c_int, dptr, dptr, dptr]),
    "mnl_structure_add_magnetic_lorentzian": (c_int, [c_void, c_double, c_double, c_int, dptr,
                                                      dptr, dptr]),
    "mnl_structure_set_box": (c_int, [c_void, c_int, c_int, dptr, c_double]),
    "mnl_structure_set_epsilon_geometry": (c_int, [c_void, c_int, c_int, dptr, c_double, c_int,
                                                   c_double, c_int]),
    "mnl_structure_get_chi1inv": (c_int, [c_void, c_int, c_int, dptr]),
    "mnl_sphere_quadrature": (c_int, [c_int, dptr]),
    "mnl_structure_set_nonlinear_mode": (c_int, [c_void, c_int]),
    "mnl_fields_create": (c_void, [c_void, c_int]),
    "mnl_fields_create_dist": (c_void, [c_void, c_int, c_int, c_int, ctypes.c_char_p]),
    "mnl_comm_unique_id": (c_int, [ctypes.c_char_p]),
    "mnl_comm_ipc_id": (c_int, [ctypes.c_char_p, c_int]),
    "mnl_fields_transport": (ctypes.c_char_p, [c_void]),
    "mnl_comm_ipc_unlink": (c_int, [ctypes.c_char_p]),
    "mnl_comm_ipc_reduce": (c_int, [ctypes.c_char_p, c_int, c_int, dptr, c_int, c_int]),
    "mnl_comm_rccl_selftest": (c_int, [c_int, c_int]),
    "mnl_slab_range": (c_int, [c_int, c_int, c_int, iptr, iptr]),
    "mnl_local_hub_create": (c_void, [c_int]),
    "mnl_local_hub_destroy": (None, [c_void]),
    "mnl_fields_create_local": (c_void, [c_void, c_int, c_int, c_int, c_void]),
    "mnl_fields_destroy": (None, [c_void]),
    "mnl_fields_add_point_source": (c_int, [c_void, c_int, c_int, dptr, c_int, dptr, c_double,
                                            c_double, c_int]),
    "mnl_fields_require_component": (c_int, [c_void, c_int]),
    "mnl_fields_step": (c_int, [c_void, c_int]),
    "mnl_fields_tune": (c_int, [c_void, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "mnl_fields_set_nan_check": (c_int, [c_void, c_int]),
    "mnl_fields_energy_in_box": (c_int, [c_void, c_int, dptr, dptr, dptr]),
    "mnl_fields_initialize_field": (c_int, [c_void, c_int, dptr, c_size]),
    "mnl_fields_time": (c_int, [c_void, llptr, dptr]),
    "mnl_fields_get_field": (c_int, [c_void, c_int, dptr, dptr]),
    "mnl_fields_copy_component": (c_int, [c_void, c_int, dptr, c_size]),
    "mnl_fields_ntot": (c_size, [c_void]),
    "mnl_fields_timers": (c_int, [c_void, dptr]),
    "mnl_fields_time_spent": (c_int, [c_void, dptr]),
    "mnl_fields_reset_timers": (c_int, [c_void]),
    "mnl_fields_allreduce": (c_int, [c_void, dptr, c_int]),
    "mnl_set_verbosity": (None, [c_int]),
    "mnl_get_verbosity": (c_int, []),
    "mnl_fields_nr_fallbacks": (c_int, [c_void, llptr]),
    "mnl_fields_set_profiling": (c_int, [c_void, c_int]),
    "mnl_fields_set_fused": (c_int, [c_void, c_int]),
    "mnl_fields_mode": (c_int, [c_void, iptr]),
    "mnl_fields_kernel_stats": (c_int, [c_void, c_int, llptr, dptr, dptr]),
    "mnl_fields_traffic_model": (c_int, [c_void, dptr, dptr]),
    "mnl_fields_tb_info": (c_int, [c_void, dptr, c_int]),
    "mnl_fields_set_temporal_blocking": (c_int, [c_void, c_int]),
    "mnl_fields_set_schedule": (c_int, [c_void, c_int, c_int]),
    "mnl_fields_add_dft_flux": (c_int, [c_void, c_int, dptr, dptr, c_int, c_int, iptr]),
    "mnl_fields_dft_flux": (c_int, [c_void, c_int, dptr]),
    "mnl_fields_dft_size": (c_int, [c_void, c_int, llptr]),
    "mnl_fields_dft_data": (c_int, [c_void, c_int, c_int, dptr, ctypes.c_longlong]),
    "mnl_fields_dft_decimation": (c_int, [c_void, c_int, iptr]),
    "mnl_fields_dft_flush": (c_int, [c_void]),
    "mnl_fields_set_time": (c_int, [c_void, ctypes.c_longlong]),
    "mnl_fields_zero_fields": (c_int, [c_void]),
    "mnl_fields_remove_sources": (c_int, [c_void]),
    "mnl_fields_add_dft_fields": (c_int, [c_void, c_int, iptr, dptr, dptr, dptr, c_int, c_int,
                                          c_int, iptr]),
    "mnl_fields_dft_array": (c_int, [c_void, c_int, c_int, c_int, iptr,
                                     ctypes.POINTER(ctypes.c_longlong), dptr, ctypes.c_longlong]),
}


def exported_symbols():
    return list(_SIGS)


def lib():
    """Load libmnl.so (built in-tree by __graft_entry__.build())."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "meep: libmnl.so not built (run __graft_entry__.build() or "
                "meep_nl_amd/csrc/build.sh); the MI355X path has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(rc):
    if rc != 0:
        raise RuntimeError(lib().mnl_last_error().decode())


def ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(dptr)
