"""ctypes binding of libmzh.so (C ABI: include/mzh.h).

torch is imported first so the process has exactly one HIP runtime: libmzh.so's
DT_NEEDED libamdhip64.so.7 then resolves to the copy torch already loaded, and device pointers /
streams from torch are valid inside the library.  There is no fallback: if the library is missing
or has no device, every call raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede loading libmzh.so, see above)

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.join(HERE, "libmzh.so")
LIB_PATH = os.environ.get("MZH_LIB") or DEFAULT_LIB  # MZH_LIB: diagnostic builds

ABI_VERSION = 6
MZH_OK = 0
MZH_ERR_ARG = -1
MZH_ERR_HIP = -2
MZH_ERR_CAPACITY = -3
MZH_ERR_STATE = -4
MZH_ERR_TEMPERATURE = -5
MZH_FLAG_NP1_UCB = 1
MZH_FLAG_KERNEL_COOP = 2  # cooperative kernel (mzh_search.hip)
MZH_FLAG_KERNEL_WAVE = 4  # wave-independent kernel (mzh_wave.hip), 32 roots per wave
MZH_FLAG_KERNEL_WAVE16 = 8  # wave-independent kernel, 16 roots per wave
MZH_FLAG_COOP_TILE16 = 16  # cooperative kernel, 16 roots per workgroup
MZH_FLAG_COOP_TILE32 = 32  # cooperative kernel, 32 roots per workgroup
MZH_FLAG_COOP_OCC2 = 64  # cooperative kernel, 16-root tiles, two workgroups per CU (mzh_search_occ2_kernel)
MZH_FLAG_KERNEL_ONE = 128  # latency kernel: one root per workgroup, the network stationary on the CU (mzh_one.hip)

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32


class SearchPlan(ctypes.Structure):
    """mirror of struct mzh_search_plan (include/mzh.h)"""
    _fields_ = [("wave", _i32), ("roots_per_wave", _i32), ("roots_per_workgroup", _i32),
                ("threads_per_workgroup", _i32), ("workgroups", _i32), ("smem_bytes", ctypes.c_int64),
                ("kernel", ctypes.c_char * 96)]

    def as_dict(self):
        return {f: (getattr(self, f).decode() if f == "kernel" else getattr(self, f)) for f, _ in self._fields_}


class SearchArgs(ctypes.Structure):
    """mirror of struct mzh_search_args (include/mzh.h)"""
    _fields_ = [
        ("B", _i32), ("n_sims", _i32), ("discount", ctypes.c_double), ("eps", ctypes.c_double),
        ("temperature", ctypes.c_double), ("deterministic", _i32), ("flags", ctypes.c_uint32),
        ("obs", _vp), ("noise", _vp), ("tie_idx", _vp), ("action_u", _vp), ("minmax_in", _vp),
        ("rp_root_pi", _vp), ("rp_sim", _vp),
        ("visits", _vp), ("root_q", _vp), ("minmax_out", _vp), ("extra_ties", _vp), ("action", _vp),
        ("pi", _vp), ("latent", _vp), ("latent_len", _vp), ("sel_steps", _vp), ("pow_table", _vp), ("lockstep_levels", _vp),
        ("plan_out", ctypes.POINTER(SearchPlan)),
    ]


class TrainArgs(ctypes.Structure):
    """mirror of struct mzh_train_args (include/mzh.h)"""
    _f32 = ctypes.c_float
    _fields_ = [
        ("B", _i32), ("U", _i32), ("in_dim", _i32), ("support", _i32), ("rows", _i32),
        ("step_size", _f32), ("bc2_sqrt", _f32), ("beta1", _f32), ("beta2", _f32), ("eps", _f32),
        ("obs", _vp), ("rwds", _vp), ("actions", _vp), ("pi", _vp), ("returns", _vp), ("weights", _vp),
        ("param", _vp * 20), ("exp_avg", _vp * 20), ("exp_avg_sq", _vp * 20), ("wt", _vp * 10),
        ("scratch", _vp), ("scratch_bytes", ctypes.c_size_t), ("row_loss", _vp), ("new_prio", _vp),
    ]


class ReplayArgs(ctypes.Structure):
    """mirror of struct mzh_replay_args (include/mzh.h)"""
    _fields_ = [("n", _i32), ("m", _i32), ("d_state", _i32), ("U", _i32), ("A", _i32),
                ("prio", _vp), ("u", _vp), ("cdf", _vp), ("states", _vp), ("rwds", _vp), ("actions", _vp),
                ("pi", _vp), ("returns", _vp), ("indx", _vp), ("out_states", _vp), ("out_rwds", _vp),
                ("out_actions", _vp), ("out_pi", _vp), ("out_returns", _vp), ("status", _vp)]


# name -> (restype, argtypes); every symbol include/mzh.h declares
SIGNATURES = {
    "mzh_abi_version": (ctypes.c_int, []),
    "mzh_build_id": (ctypes.c_char_p, []),
    "mzh_last_error": (ctypes.c_char_p, []),
    "mzh_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "mzh_stream_synchronize": (ctypes.c_int, [_vp]),
    "mzh_host_device_pointer": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "mzh_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(_vp)]),
    "mzh_destroy": (ctypes.c_int, [_vp]),
    "mzh_weights_size": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "mzh_load_weights": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    "mzh_env_step": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [_vp] * 10 + [_vp]),
    "mzh_legal_mask": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]),
    "mzh_encode_obs": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]),
    "mzh_hanoi_solver": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]),
    "mzh_initial_inference": (ctypes.c_int, [_vp, ctypes.c_int] + [_vp] * 7 + [_vp]),
    "mzh_recurrent_inference": (ctypes.c_int, [_vp, ctypes.c_int] + [_vp] * 9 + [_vp]),
    "mzh_search": (ctypes.c_int, [_vp, ctypes.POINTER(SearchArgs), _vp]),
    "mzh_search_replay": (ctypes.c_int, [_vp, ctypes.POINTER(SearchArgs), _vp]),
    "mzh_search_plan_query": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                             ctypes.c_int, ctypes.POINTER(SearchPlan)]),
    "mzh_rng_predraw": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int,
                                       _vp, _vp, _vp]),
    "mzh_train_scratch_bytes": (ctypes.c_int, [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_size_t)]),
    "mzh_train_transpose": (ctypes.c_int, [ctypes.POINTER(TrainArgs), _vp]),
    "mzh_train_update": (ctypes.c_int, [ctypes.POINTER(TrainArgs), _vp]),
    "mzh_replay_sample": (ctypes.c_int, [ctypes.POINTER(ReplayArgs), _vp]),
    "mzh_replay_set_priorities": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, _vp, _vp]),
}

_lib = None


def lib():
    """Load libmzh.so (once). Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m muzero_hanoi_amd.build` "
                               "(there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.mzh_abi_version() != ABI_VERSION:
            raise RuntimeError(f"libmzh.so ABI version {L.mzh_abi_version()} != {ABI_VERSION}")
        if os.path.abspath(LIB_PATH) == DEFAULT_LIB and os.path.isdir(os.path.join(HERE, "csrc")):
            # provenance: the shipped library must be built from the checked-out sources
            from . import build as _build

            want, got = _build.source_hash(), L.mzh_build_id().decode()
            if got != want:
                raise RuntimeError(f"{LIB_PATH} was built from other sources or flags (build id {got}, the "
                                   f"checked-out sources hash to {want}): rebuild with "
                                   "`python -m muzero_hanoi_amd.build`")
        _lib = L
    return _lib


def build_id():
    return lib().mzh_build_id().decode()


def last_error():
    msg = lib().mzh_last_error()
    return msg.decode() if msg else ""


def check(status, what):
    """Map a status code to the reference's exception types."""
    if status == MZH_OK:
        return
    msg = f"{what}: {last_error()}"
    if status in (MZH_ERR_ARG, MZH_ERR_TEMPERATURE):
        raise ValueError(msg)
    raise RuntimeError(msg)


def search_plan(support, B, n_sims, flags=0, replay=False, minmax_in=False):
    """the kernel instantiation mzh_search / mzh_search_replay would launch (host-only query)"""
    out = SearchPlan()
    check(lib().mzh_search_plan_query(int(support), int(B), int(n_sims), int(flags), 1 if replay else 0,
                                      1 if minmax_in else 0, ctypes.byref(out)), "mzh_search_plan_query")
    return out.as_dict()


def device_count():
    n = ctypes.c_int(0)
    st = lib().mzh_device_count(ctypes.byref(n))
    return n.value if st == MZH_OK else 0


def host_device_pointer(addr):
    """the device address of page-locked host memory at `addr` (mzh_host_device_pointer)"""
    out = _vp()
    check(lib().mzh_host_device_pointer(addr, ctypes.byref(out)), "mzh_host_device_pointer")
    return out.value


def ptr(t):
    """device pointer of a tensor (None -> NULL)"""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_DEV_INDEX = {}


def _device_index(device):
    if device is None:
        return torch.cuda.current_device()
    i = _DEV_INDEX.get(device)
    if i is None:
        d = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
        i = d.index if d.index is not None else -1
        _DEV_INDEX[device] = i
    return torch.cuda.current_device() if i < 0 else i


def stream_handle(device=None):
    """torch's current stream on `device` as a raw hipStream_t (the launch stream of every call)"""
    if _RAW_STREAM is not None:
        return ctypes.c_void_p(_RAW_STREAM(_device_index(device)))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def synchronize(device=None):
    """wait for the current stream on `device` (mzh_stream_synchronize on the same raw handle the calls use)"""
    check(lib().mzh_stream_synchronize(stream_handle(device)), "mzh_stream_synchronize")
