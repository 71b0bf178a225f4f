"""ctypes signatures of libucg_builtin.so (include/ucg_builtin_combine.h)."""
import ctypes

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_int = ctypes.c_int
_u = ctypes.c_uint
_u64 = ctypes.c_uint64

REDUCE_CB = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _vp, _vp, ctypes.c_uint, _vp)
COMP_CB = ctypes.CFUNCTYPE(None, _vp, ctypes.c_int)      # coll_comp_cb_f(req, status)
OP_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp)
CONVERT_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_size_t))
IS_INT_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_int))
DT_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp)


class ReduceParams(ctypes.Structure):
    """ucg_builtin_reduce_params_t (mirror of api/ucg.h:129-160)."""
    _fields_ = [("reduce_cb_f", REDUCE_CB), ("is_sum_f", OP_FN),
                ("is_loc_expected_f", OP_FN), ("is_commutative_f", OP_FN),
                ("convert", CONVERT_FN), ("is_integer_f", IS_INT_FN),
                ("is_floating_point_f", DT_FN)]


class GroupParams(ctypes.Structure):
    """ucg_builtin_lgroup_params_t (include/ucg_builtin_ops.h)."""
    _fields_ = [("distance", ctypes.POINTER(ctypes.c_uint8)), ("tree_radix", ctypes.c_uint),
                ("sock_thresh", ctypes.c_uint), ("recursive_factor", ctypes.c_uint),
                ("mem_reg_opt_cnt", ctypes.c_int)]


class CombineConfig(ctypes.Structure):
    _fields_ = [("dev_enable", ctypes.c_int), ("dev_min_bytes", _sz),
                ("stage_bytes", _sz), ("stage_slots", ctypes.c_uint),
                ("device", ctypes.c_int), ("zcopy_bytes", _sz),
                ("completion", ctypes.c_int), ("stream", _vp)]


HOST_API = {
    "ucg_builtin_combine_config_read": (None, [ctypes.POINTER(CombineConfig)]),
    "ucg_builtin_combine_create": (_int, [ctypes.POINTER(ReduceParams),
                                          ctypes.POINTER(CombineConfig),
                                          ctypes.POINTER(_vp)]),
    "ucg_builtin_combine_destroy": (None, [_vp]),
    "ucg_builtin_combine_set_classifier": (None, [_vp, OP_FN, DT_FN]),
    "ucg_builtin_combine_classify": (_int, [_vp, _vp, _vp, ctypes.POINTER(_int),
                                            ctypes.POINTER(_int)]),
    "ucg_builtin_combine_has_device": (_int, [_vp]),
    "ucg_builtin_combine_dev_ctx": (_vp, [_vp]),
    "ucg_builtin_combine_reduce": (_int, [_vp, _vp, _vp, _vp, _int, _vp]),
    "ucg_builtin_combine_step_begin": (_int, [_vp, _vp, _vp, _vp, _sz]),
    "ucg_builtin_combine_fragment": (_int, [_vp, _sz, _vp, _sz]),
    "ucg_builtin_combine_step_end": (_int, [_vp]),
    "ucg_builtin_combine_step_on_device": (_int, [_vp]),
    "ucg_builtin_combine_stats": (None, [_vp, ctypes.POINTER(_u64)]),
    "ucg_builtin_combine_mem_reg": (_int, [_vp, _vp, _sz]),
    "ucg_builtin_combine_mem_dereg": (None, [_vp, _vp]),
    "ucg_builtin_step_fragment_length": (_sz, [_sz, _sz]),
    "ucg_builtin_step_fragments_total": (_u64, [_sz, _sz, _u]),
    "ucg_builtin_dev_chunk_bytes": (_sz, [_sz, _sz, _sz]),
    "ucg_builtin_recursive_steps": (_u, [_u64, _u]),
    "ucg_builtin_recursive_peer": (_u64, [_u64, _u, _u, _u]),
    "ucg_builtin_combine_dtype_length": (_sz, [_vp, _vp]),
    "ucg_builtin_combine_atomic_sum_length": (_sz, [_vp, _vp, _vp]),
    "ucg_builtin_combine_check_reduction": (_int, [_vp, _vp]),
    "ucg_builtin_combine_dev_alloc": (_vp, [_vp, _sz]),
    "ucg_builtin_combine_dev_free": (None, [_vp, _vp]),
    "ucg_builtin_combine_dev_park": (None, [_vp, _vp]),
    "ucg_builtin_combine_dev_export": (_int, [_vp, _vp, _vp]),
    "ucg_builtin_combine_dev_import": (_int, [_vp, _vp, ctypes.POINTER(_vp)]),
    "ucg_builtin_combine_dev_release": (None, [_vp, _vp]),
    "ucg_builtin_combine_dev_fold": (_int, [_vp, _vp, _vp, _vp, ctypes.POINTER(_vp), _u,
                                            _sz]),
    "ucg_builtin_combine_dev_copy": (_int, [_vp, _vp, _vp, _sz]),
    "ucg_builtin_combine_dev_copy_n": (_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                              _u, _sz]),
    "ucg_builtin_combine_dev_butterfly": (_int, [_vp, _vp, _vp, _vp, ctypes.POINTER(_vp), _u,
                                                 _u, _sz]),
    # include/ucg_builtin_ops.h
    "ucg_builtin_shm_iface_open": (_int, [ctypes.c_char_p, _u, _u, _sz, _u,
                                          ctypes.POINTER(_vp)]),
    "ucg_builtin_shm_iface_close": (_int, [_vp]),
    "ucg_builtin_shm_job_token": (_u64, []),
    "ucg_builtin_shm_iface_max_short": (_sz, [_vp]),
    "ucg_builtin_shm_am_short": (_int, [_vp, _u, _u64, _vp, _sz]),
    "ucg_builtin_shm_progress": (_u, [_vp, _vp, _vp]),
    "ucg_builtin_shm_barrier": (_int, [_vp]),
    "ucg_builtin_shm_am_incast_batched": (_int, [_vp, _u, _u64, _u, _vp, _sz]),
    "ucg_builtin_shm_am_incast": (_int, [_vp, _u, _u64, _u, _sz, _vp, _vp, _int]),
    "ucg_builtin_lgroup_create": (_int, [_vp, ctypes.c_uint16, _u, _u, _vp,
                                         ctypes.POINTER(_vp)]),
    "ucg_builtin_lgroup_create_ex": (_int, [_vp, ctypes.c_uint16, _u, _u, _vp,
                                            ctypes.POINTER(GroupParams), ctypes.POINTER(_vp)]),
    "ucg_builtin_lgroup_destroy": (None, [_vp]),
    "ucg_builtin_lgroup_progress": (_u, [_vp]),
    "ucg_builtin_lgroup_stats": (None, [_vp, ctypes.POINTER(_u64)]),
    "ucg_builtin_lgroup_mem_alloc": (_vp, [_vp, _sz, _int]),
    "ucg_builtin_lgroup_mem_free": (None, [_vp, _vp]),
    "ucg_builtin_lcoll_allreduce": (_int, [_vp, _vp, _vp, _int, _vp, _vp,
                                           ctypes.POINTER(_vp)]),
    "ucg_builtin_lcoll_reduce": (_int, [_vp, _vp, _vp, _int, _vp, _vp, _u,
                                        ctypes.POINTER(_vp)]),
    "ucg_builtin_lcoll_start": (_int, [_vp]),
    "ucg_builtin_lcoll_start_as": (_int, [_vp, ctypes.c_uint8]),
    "ucg_builtin_lgroup_set_async_timer": (_int, [_vp, ctypes.c_double]),
    "ucg_builtin_lgroup_async_stats": (None, [_vp, ctypes.POINTER(_u64)]),
    "ucg_builtin_lcoll_test": (_int, [_vp, ctypes.POINTER(_int)]),
    "ucg_builtin_lcoll_wait": (_int, [_vp]),
    "ucg_builtin_lcoll_destroy": (None, [_vp]),
    "ucg_builtin_lcoll_describe": (_sz, [_vp, ctypes.c_char_p, _sz]),
    "ucg_builtin_lcoll_set_completion": (_int, [_vp, _vp, _vp, _sz, _sz]),
    # include/ucg_builtin_component.h
    "ucg_builtin_component_set_classifier": (None, [OP_FN, DT_FN]),
    "ucg_builtin_component_last_destroy_status": (_int, []),
}
