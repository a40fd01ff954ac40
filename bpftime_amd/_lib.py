"""ctypes binding of libbpftime_amd.so (the C ABI in include/ebpf-vm.h and
include/bpftime_amd.h).  The library is built in-tree by ``build()`` in
__graft_entry__.py (bpftime_amd/csrc/Makefile) and MUST be present: there is
no CPU fallback anywhere in the product path."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BPFTIME_AMD_LIB") or os.path.join(_HERE, "lib", "libbpftime_amd.so")

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)


class BpfMapAttr(C.Structure):  # runtime/include/bpftime_shm.hpp:27-46
    _fields_ = [("type", C.c_int), ("key_size", C.c_uint32), ("value_size", C.c_uint32),
                ("max_ents", C.c_uint32), ("flags", C.c_uint64), ("ifindex", C.c_uint32),
                ("btf_vmlinux_value_type_id", C.c_uint32), ("btf_id", C.c_uint32),
                ("btf_key_type_id", C.c_uint32), ("btf_value_type_id", C.c_uint32),
                ("map_extra", C.c_uint64), ("kernel_bpf_map_id", C.c_uint32),
                ("gpu_thread_count", C.c_uint64)]


class BpfLinkCreateArgs(C.Structure):  # bpftime_shm.hpp:250-301
    _fields_ = [("prog_fd", C.c_uint32), ("target_fd", C.c_uint32), ("attach_type", C.c_uint32),
                ("flags", C.c_uint32), ("attach_union", C.c_uint64 * 4)]


class EbpfBatch(C.Structure):  # include/ebpf-vm.h struct ebpf_batch
    _fields_ = [("ctx_kind", C.c_uint32), ("flags", C.c_uint32), ("count", C.c_uint64),
                ("data", C.c_void_p), ("stride", C.c_uint64), ("lens", C.c_void_p),
                ("fixed_len", C.c_uint32), ("ingress_ifindex", C.c_uint32),
                ("rx_queue_index", C.c_uint32), ("head", C.c_uint32), ("verdicts", C.c_void_p),
                ("rets", C.c_void_p), ("data_off_out", C.c_void_p), ("len_out", C.c_void_p),
                ("first_unit", C.c_uint64), ("stream", C.c_void_p), ("descs", C.c_void_p),
                ("umem_bytes", C.c_uint64), ("sys_nr", C.c_int64), ("sys_state", C.c_void_p),
                ("sys_ret", C.c_void_p), ("sys_phase", C.c_uint32), ("pid_tgid_off", C.c_int32),
                ("ktime_off", C.c_int32), ("pid_tgid_arr", C.c_void_p), ("pid_tgid_stride", C.c_uint64),
                ("ktime_arr", C.c_void_p), ("ktime_stride", C.c_uint64)]


class SysRecords(C.Structure):  # include/bpftime_amd.h struct bpftime_amd_sys_records
    _fields_ = [("enter", C.c_void_p), ("exit", C.c_void_p), ("clock", C.c_void_p), ("count", C.c_uint64)]


class PerfEvent(C.Structure):
    """struct bpftime_amd_perf_event (include/bpftime_amd.h)"""
    _fields_ = [("type", C.c_int), ("pid", C.c_int), ("enabled", C.c_int), ("tracepoint_id", C.c_int32),
                ("sys_nr", C.c_int64), ("offset", C.c_uint64), ("ref_ctr_off", C.c_uint64),
                ("module_name", C.c_char_p), ("cpu", C.c_int), ("sample_type", C.c_int32), ("config", C.c_int64)]


# (name, restype, argtypes) for every exported symbol of include/*.h
SIGNATURES = [
    # include/ebpf-vm.h
    ("ebpf_create", C.c_void_p, [C.c_char_p]),
    ("ebpf_destroy", None, [C.c_void_p]),
    ("ebpf_get_vm_name", C.c_char_p, [C.c_void_p]),
    ("ebpf_toggle_bounds_check", C.c_bool, [C.c_void_p, C.c_bool]),
    ("ebpf_set_error_print", None, [C.c_void_p, C.c_void_p]),
    ("ebpf_register", C.c_int, [C.c_void_p, C.c_uint, C.c_char_p, C.c_void_p]),
    ("ebpf_load", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("ebpf_unload_code", None, [C.c_void_p]),
    ("ebpf_exec", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, u64p]),
    ("ebpf_compile", C.c_void_p, [C.c_void_p, C.POINTER(C.c_void_p)]),
    ("ebpf_set_unwind_function_index", C.c_int, [C.c_void_p, C.c_uint]),
    ("ebpf_set_pointer_secret", C.c_int, [C.c_void_p, C.c_uint64]),
    ("ebpf_set_lddw_helpers", None, [C.c_void_p] + [C.c_void_p] * 5),
    ("ebpf_load_aot_object", C.c_void_p, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("ebpf_exec_batch", C.c_int, [C.c_void_p, C.POINTER(EbpfBatch)]),
    ("ebpf_set_ctx_kind", C.c_int, [C.c_void_p, C.c_uint32]),
    # include/bpftime_amd.h
    ("bpftime_maps_create", C.c_int, [C.c_int, C.c_char_p, BpfMapAttr]),
    ("bpftime_map_lookup_elem", C.c_void_p, [C.c_int, C.c_void_p]),
    ("bpftime_map_update_elem", C.c_long, [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64]),
    ("bpftime_map_delete_elem", C.c_long, [C.c_int, C.c_void_p]),
    ("bpftime_map_get_next_key", C.c_int, [C.c_int, C.c_void_p, C.c_void_p]),
    ("bpftime_map_value_size_from_syscall", C.c_uint32, [C.c_int]),
    ("bpftime_is_map_fd", C.c_int, [C.c_int]),
    ("bpftime_is_array_map", C.c_int, [C.c_int]),
    ("bpftime_is_prog_fd", C.c_int, [C.c_int]),
    ("bpftime_find_minimal_unused_fd", C.c_int, []),
    ("bpftime_close", None, [C.c_int]),
    ("bpftime_progs_create", C.c_int, [C.c_int, C.c_void_p, C.c_size_t, C.c_char_p, C.c_int]),
    ("bpftime_link_create", C.c_int, [C.c_int, C.POINTER(BpfLinkCreateArgs)]),
    ("bpftime_amd_map_ptr_by_fd", C.c_uint64, [C.c_uint32]),
    ("bpftime_amd_map_val", C.c_uint64, [C.c_uint64]),
    ("bpftime_amd_map_device_ptr", C.c_uint64, [C.c_int, u64p]),
    ("bpftime_amd_map_snapshot", C.c_int, [C.c_int, C.c_void_p, C.c_uint64]),
    ("bpftime_amd_map_restore", C.c_int, [C.c_int, C.c_void_p, C.c_uint64]),
    ("bpftime_amd_map_geometry", C.c_int, [C.c_int, u64p, u32p, u32p, u32p, u32p]),
    ("bpftime_amd_map_count", C.c_uint64, [C.c_int]),
    ("bpftime_amd_map_ack_error", C.c_int, [C.c_int]),
    ("bpftime_amd_set_ncpu", None, [C.c_uint32]),
    ("bpftime_amd_get_ncpu", C.c_uint32, []),
    ("bpftime_amd_reset", None, []),
    ("bpftime_amd_xdp_links", C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int), u32p, C.c_int]),
    ("bpftime_amd_prog_instantiate", C.c_void_p, [C.c_int, C.POINTER(C.c_void_p)]),
    ("bpftime_amd_register_default_helpers", C.c_int, [C.c_void_p]),
    ("bpftime_amd_vm_info", C.c_int, [C.c_void_p, u32p, C.POINTER(C.c_int), u32p, u32p]),
    ("bpftime_amd_set_step_limit", None, [C.c_void_p, C.c_uint64]),
    ("bpftime_amd_last_batch_ms", C.c_float, [C.c_void_p]),
    ("bpftime_amd_vm_fast_info", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    ("bpftime_amd_vm_counter_info", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32),
                                              C.POINTER(C.c_uint32)]),
    ("bpftime_import_global_shm_from_json", C.c_int, [C.c_char_p]),
    ("bpftime_export_global_shm_to_json", C.c_int, [C.c_char_p]),
    ("bpftime_import_shm_handler_from_json", C.c_int, [C.c_int, C.c_char_p]),
    ("bpftime_object_open", C.c_void_p, [C.c_char_p]),
    ("bpftime_object_open_mem", C.c_void_p, [C.c_void_p, C.c_size_t, C.c_char_p]),
    ("bpftime_object_error", C.c_char_p, [C.c_void_p]),
    ("bpftime_object_load_relocate_btf", C.c_int, [C.c_void_p, C.c_char_p]),
    ("bpftime_object_load_relocate_btf_mem", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("bpftime_object_map_count", C.c_int, [C.c_void_p]),
    ("bpftime_object_map_info", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(BpfMapAttr)]),
    ("bpftime_object_program_count", C.c_int, [C.c_void_p]),
    ("bpftime_object_program_info", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                              C.POINTER(C.c_int), C.POINTER(C.c_size_t)]),
    ("bpftime_object_program_insns", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_void_p, C.c_size_t]),
    ("bpftime_object_load", C.c_int, [C.c_void_p]),
    ("bpftime_object_find_program_by_name", C.c_int, [C.c_void_p, C.c_char_p]),
    ("bpftime_object_find_program_by_secname", C.c_int, [C.c_void_p, C.c_char_p]),
    ("bpftime_object_find_map_fd_by_name", C.c_int, [C.c_void_p, C.c_char_p]),
    ("bpftime_object_license", C.c_char_p, [C.c_void_p]),
    ("bpftime_object_close", None, [C.c_void_p]),
    ("bpftime_amd_ringbuf_fetch", C.c_int64, [C.c_int, C.c_void_p, C.c_uint64, u64p]),
    ("bpftime_amd_syscall_attach", C.c_int, [C.c_int, C.c_int64]),
    ("bpftime_amd_syscall_detach", C.c_int, [C.c_int]),
    ("bpftime_amd_syscall_dispatch", C.c_int64, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]),
    ("bpftime_amd_syscall_attach_ex", C.c_int, [C.c_int, C.c_int64, C.c_int]),
    ("bpftime_amd_syscall_dispatch_records", C.c_int64, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                                         C.c_uint32, C.c_void_p]),
    ("bpftime_amd_syscall_dispatch_plan", C.c_int, [C.c_uint32]),
    ("bpftime_amd_syscall_dispatch_soa", C.c_int64, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    ("bpftime_amd_handle_sysbpf", C.c_long, [C.c_int, C.c_void_p, C.c_uint32]),
    ("bpftime_map_get_info", C.c_int, [C.c_int, C.POINTER(BpfMapAttr), C.POINTER(C.c_char_p),
                                        C.POINTER(C.c_int)]),
    ("bpftime_get_array_map_raw_data", C.c_void_p, [C.c_int]),
    ("bpftime_amd_map_msync", C.c_int, [C.c_int]),
    ("bpftime_amd_perf_event_syscall", C.c_int, [C.c_int, C.c_int64]),
    ("bpftime_is_perf_event_fd", C.c_int, [C.c_int]),
    ("bpftime_attach_perf_to_bpf", C.c_int, [C.c_int, C.c_int]),
    ("bpftime_tracepoint_create", C.c_int, [C.c_int, C.c_int, C.c_int32]),
    ("bpftime_uprobe_create", C.c_int, [C.c_int, C.c_int, C.c_char_p, C.c_uint64, C.c_bool, C.c_size_t]),
    ("bpftime_perf_event_enable", C.c_int, [C.c_int]),
    ("bpftime_perf_event_disable", C.c_int, [C.c_int]),
    ("bpftime_amd_perf_event_record", C.c_int, [C.c_int, C.POINTER(PerfEvent)]),
    ("bpftime_amd_perf_event_get", C.c_int, [C.c_int, C.POINTER(PerfEvent)]),
    ("bpftime_amd_link_perf", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("bpftime_amd_link_attached", C.c_int, [C.c_int]),
    ("bpftime_amd_set_tracefs_events", C.c_int, [C.c_char_p]),
    ("bpftime_amd_tracepoint_resolve", C.c_int, [C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int)]),
    ("bpftime_amd_tracepoint_id", C.c_int32, [C.c_int64, C.c_int]),
    ("bpftime_amd_syscall_nr", C.c_int64, [C.c_char_p]),
    ("bpftime_amd_attach_create", C.c_void_p, [C.c_int, C.c_int]),
    ("bpftime_amd_attach_run", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64)]),
    ("bpftime_amd_attach_run_batch", C.c_int, [C.c_void_p, C.POINTER(EbpfBatch)]),
    ("bpftime_amd_attach_destroy", None, [C.c_void_p]),
    ("bpftime_amd_simple_attach_impl_create", C.c_int, [C.c_int, C.c_void_p]),
    ("bpftime_amd_simple_attach", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int]),
    ("bpftime_amd_simple_detach", C.c_int, [C.c_int, C.c_int]),
    ("bpftime_amd_simple_trigger", C.c_int, [C.c_int, C.c_void_p]),
    ("bpftime_amd_simple_attach_impl_destroy", C.c_int, [C.c_int]),
    ("bpftime_amd_merge_delta_u64", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    ("bpftime_amd_merge_delta", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32]),
    ("bpftime_amd_device_count", C.c_int, []),
    ("bpftime_amd_hip_runtime_version", C.c_int, []),
    ("bpftime_amd_dbg_counters", C.c_int, [C.POINTER(C.c_uint64), C.c_int, C.c_int]),
    ("bpftime_amd_set_device", C.c_int, [C.c_int]),
    ("bpftime_amd_dev_alloc", C.c_void_p, [C.c_uint64]),
    ("bpftime_amd_dev_free", None, [C.c_void_p]),
    ("bpftime_amd_memcpy_htod", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    ("bpftime_amd_memcpy_dtoh", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    ("bpftime_amd_memset", C.c_int, [C.c_void_p, C.c_int, C.c_uint64]),
    ("bpftime_amd_sync", C.c_int, []),
    ("bpftime_amd_memcpy_htod_async", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    ("bpftime_amd_memcpy_dtoh_async", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    ("bpftime_amd_stream_create", C.c_void_p, []),
    ("bpftime_amd_stream_destroy", None, [C.c_void_p]),
    ("bpftime_amd_stream_sync", C.c_int, [C.c_void_p]),
    ("bpftime_amd_host_alloc", C.c_void_p, [C.c_uint64]),
    ("bpftime_amd_host_free", None, [C.c_void_p]),
    ("bpftime_amd_event_create", C.c_void_p, []),
    ("bpftime_amd_event_destroy", None, [C.c_void_p]),
    ("bpftime_amd_event_record", C.c_int, [C.c_void_p, C.c_void_p]),
    ("bpftime_amd_stream_wait_event", C.c_int, [C.c_void_p, C.c_void_p]),
    ("bpftime_amd_event_elapsed_ms", C.c_float, [C.c_void_p, C.c_void_p]),
    ("bpftime_amd_last_error", C.c_char_p, []),
    ("bpftime_amd_gen_syscall_full", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p,
                                                C.c_uint32, C.c_void_p]),
    ("bpftime_amd_gen_syscall_soa", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64,
                                              C.c_void_p, C.c_uint32, C.c_void_p]),
    ("bpftime_amd_static_lds", C.c_size_t, [C.c_uint32, C.c_bool, C.c_bool, C.c_uint32]),
    ("bpftime_amd_lds_bytes", C.c_size_t, [C.c_uint32, C.c_bool, C.c_uint32, C.c_uint32, C.c_uint32, C.c_bool,
                                           C.c_bool, C.c_uint32]),
    ("bpftime_amd_gen_xdp", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64,
                                       C.c_uint64, C.c_void_p]),
    ("bpftime_amd_gen_flow", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                        C.c_void_p, C.c_uint32, C.c_void_p]),
    ("bpftime_amd_gen_syscall", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint32,
                                           C.c_void_p]),
]

# symbols outside include/*.h that the Python layer also uses
EXTRA = [
    ("bpftime_amd_vm_error", C.c_char_p, [C.c_void_p]),
]

_lib = None


def lib() -> C.CDLL:
    """Load the product library; raise loudly if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
        l = C.CDLL(LIB_PATH, use_errno=True)
        for name, res, args in SIGNATURES + EXTRA:
            if os.environ.get("BPFTIME_AMD_LIB") and not hasattr(l, name):
                continue  # an older build loaded for A/B timing
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib
