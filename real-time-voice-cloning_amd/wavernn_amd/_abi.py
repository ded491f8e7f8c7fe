"""ctypes bindings of libwavernn_mi355x.so (include/wavernn_mi355x.h).

The library is the only compute path of this package: if it is missing, importing the model
raises immediately -- there is no CPU or eager-PyTorch fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = 'libwavernn_mi355x.so'
# WRNN_LIB: another build of the same library (kernel A/B experiments, tools/)
LIB_PATH = os.environ.get('WRNN_LIB') or os.path.join(_HERE, LIB_NAME)

WRNN_OK = 0
WRNN_ERR_INVALID = -1
WRNN_ERR_NOT_LOADED = -2
WRNN_ERR_HIP = -3
WRNN_ERR_OOM = -4
WRNN_ERR_ABORTED = -5
WRNN_ERR_CAPACITY = -6

WRNN_MODEL_FATCHORD = 0
WRNN_MODEL_RUNTIMERACER = 1
WRNN_MODEL_GENEING = 2
WRNN_MODE_RAW = 0
WRNN_MODE_MOL = 1
WRNN_MODE_BETA = 2

WRNN_ENGINE_AUTO = 0
WRNN_ENGINE_CHAIN = 1
WRNN_ENGINE_PERSIST = 2
ENGINES = {'auto': WRNN_ENGINE_AUTO, 'chain': WRNN_ENGINE_CHAIN, 'persist': WRNN_ENGINE_PERSIST}

EXPORTED = [
    'wrnn_version', 'wrnn_last_error', 'wrnn_device_count', 'wrnn_create', 'wrnn_destroy',
    'wrnn_load_tensor', 'wrnn_finalize', 'wrnn_set_seed', 'wrnn_set_stream', 'wrnn_fold_shape',
    'wrnn_generate', 'wrnn_generate_batch_device', 'wrnn_enable_stage_timing',
    'wrnn_stage_timing', 'wrnn_stage_info', 'wrnn_debug_noise', 'wrnn_debug_upsample',
    'wrnn_set_engine', 'wrnn_last_engine', 'wrnn_bin_read', 'wrnn_load_bin',
    'wrnn_de_emphasis', 'wrnn_post_overlaps', 'wrnn_post_assemble', 'wrnn_fallback_info',
    'wrnn_debug_beta', 'wrnn_debug_decide', 'wrnn_debug_rot_plan', 'wrnn_debug_slice_plan', 'wrnn_rot_info', 'wrnn_persist_steps', 'wrnn_plan_info', 'wrnn_debug_p1', 'wrnn_get_stream',
    'wrnn_set_utt_streams', 'wrnn_set_fold_ranges', 'wrnn_set_debug_steps', 'wrnn_debug_logits', 'wrnn_debug_wide_layout',
    'wrnn_sparse_info', 'wrnn_set_rates', 'wrnn_get_rates', 'wrnn_debug_plan',
]


class WrnnConfig(ctypes.Structure):
    _fields_ = [
        ('model_type', ctypes.c_int), ('mode', ctypes.c_int), ('bits', ctypes.c_int),
        ('rnn_dims', ctypes.c_int), ('fc_dims', ctypes.c_int), ('compute_dims', ctypes.c_int),
        ('res_out_dims', ctypes.c_int), ('res_blocks', ctypes.c_int), ('pad', ctypes.c_int),
        ('feat_dims', ctypes.c_int), ('hop_length', ctypes.c_int), ('n_upsample', ctypes.c_int),
        ('upsample_factors', ctypes.c_int * 4),
    ]


PROGRESS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_double)

TENSOR_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p,
                             ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64),
                             ctypes.c_int)

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def load_library(path=None):
    """Load (once) and type the C-ABI library. Raises NativeLibraryMissing if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f'{LIB_NAME} not found at {path}: build it with `make -C '
            f'real-time-voice-cloning_amd/csrc` or __graft_entry__.build(); the MI355X vocoder '
            f'has no CPU fallback')
    # WRNN_HOST_ONLY=1: a host-only build of the library (the sanitizer build of `make asan`,
    # tests/test_sanitizers.py) -- no HIP runtime to bind, only the host entry points exist
    host_only = os.environ.get('WRNN_HOST_ONLY') == '1'
    if not host_only:
        try:
            # One HIP runtime per process: when PyTorch is present its bundled libamdhip64.so.7
            # must be loaded first so this library binds to it (same SONAME) instead of pulling
            # in /opt/rocm's copy, after which torch.cuda cannot initialise.
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    c_int, c_void_p, c_size_t = ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    sig = {
        'wrnn_version': (ctypes.c_char_p, []),
        'wrnn_last_error': (ctypes.c_char_p, []),
        'wrnn_device_count': (c_int, [P(c_int)]),
        'wrnn_create': (c_int, [P(WrnnConfig), c_int, P(c_void_p)]),
        'wrnn_destroy': (None, [c_void_p]),
        'wrnn_load_tensor': (c_int, [c_void_p, ctypes.c_char_p, P(ctypes.c_float),
                                     P(ctypes.c_int64), c_int]),
        'wrnn_finalize': (c_int, [c_void_p]),
        'wrnn_bin_read': (c_int, [ctypes.c_char_p, c_size_t, P(WrnnConfig), TENSOR_FN, c_void_p]),
        'wrnn_load_bin': (c_int, [c_void_p, ctypes.c_char_p, c_size_t]),
        'wrnn_set_seed': (c_int, [c_void_p, ctypes.c_uint64]),
        'wrnn_set_stream': (c_int, [c_void_p, ctypes.c_uint32]),
        'wrnn_get_stream': (c_int, [c_void_p, P(ctypes.c_uint32)]),
        'wrnn_set_utt_streams': (c_int, [c_void_p, P(ctypes.c_uint32), c_int]),
        'wrnn_set_fold_ranges': (c_int, [c_void_p, P(c_int), P(c_int), c_int]),
        'wrnn_fold_shape': (c_int, [c_int, c_int, c_int, c_int, c_int, P(c_int), P(c_int)]),
        'wrnn_generate': (c_int, [c_void_p, P(ctypes.c_float), c_int, c_int, c_int, c_int,
                                  P(ctypes.c_int16), P(ctypes.c_float), c_size_t, P(c_int),
                                  P(c_int), PROGRESS_FN, c_void_p]),
        'wrnn_generate_batch_device': (c_int, [c_void_p, c_int, P(c_void_p), P(c_int), c_int,
                                               c_int, c_int, c_void_p, c_void_p, c_size_t,
                                               P(c_int), P(c_int), PROGRESS_FN, c_void_p]),
        'wrnn_set_engine': (c_int, [c_void_p, c_int]),
        'wrnn_last_engine': (c_int, [c_void_p, P(c_int)]),
        'wrnn_fallback_info': (c_int, [c_void_p, P(c_int), ctypes.c_char_p, c_size_t]),
        'wrnn_enable_stage_timing': (c_int, [c_void_p, c_int]),
        'wrnn_stage_timing': (c_int, [c_void_p, c_int, P(ctypes.c_double), P(c_int)]),
        'wrnn_stage_info': (c_int, [c_void_p, c_int, ctypes.c_char_p, c_size_t,
                                    P(ctypes.c_double), P(ctypes.c_double), P(c_int)]),
        'wrnn_de_emphasis': (c_int, [P(ctypes.c_double), P(ctypes.c_double), c_size_t,
                                     ctypes.c_double]),
        'wrnn_post_overlaps': (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                       c_void_p, c_void_p, c_void_p]),
        'wrnn_post_assemble': (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                       c_void_p, c_int, ctypes.c_double, c_void_p, c_size_t,
                                       c_void_p, c_size_t]),
        'wrnn_debug_noise': (c_int, [c_void_p, c_int, P(ctypes.c_float), c_size_t]),
        'wrnn_plan_info': (c_int, [c_void_p, P(c_int), P(c_int), P(c_int), P(c_int), c_int]),
        'wrnn_sparse_info': (c_int, [c_void_p, P(c_int), P(c_int), P(ctypes.c_double), P(c_int)]),
        'wrnn_set_rates': (c_int, [c_void_p, ctypes.c_char_p]),
        'wrnn_get_rates': (c_int, [c_void_p, ctypes.c_char_p, c_size_t]),
        'wrnn_debug_plan': (c_int, [ctypes.c_char_p, c_int, c_int, c_int, c_int, c_int, c_int, P(c_int),
                                    P(c_int), P(c_int), c_int, P(c_int)]),
        'wrnn_debug_beta': (c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_float, ctypes.c_float,
                                    P(ctypes.c_float)]),
        'wrnn_debug_rot_plan': (c_int, [c_int, c_int, ctypes.c_double, ctypes.c_double, P(c_int), P(c_int),
                                        P(c_int), P(c_int), c_size_t]),
        'wrnn_rot_info': (c_int, [c_void_p, P(c_int), P(c_int), P(c_int)]),
        'wrnn_debug_slice_plan': (c_int, [c_int, c_int, P(c_int), P(c_int), c_size_t, P(c_int), c_size_t]),
        'wrnn_persist_steps': (c_int, [c_void_p, c_int, P(ctypes.c_double)]),
        'wrnn_debug_decide': (c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, P(ctypes.c_float), c_int, P(c_int),
                                      P(ctypes.c_double)]),
        'wrnn_debug_upsample': (c_int, [c_void_p, P(ctypes.c_float), c_size_t,
                                        P(ctypes.c_float), c_size_t]),
        'wrnn_debug_p1': (c_int, [c_void_p, c_int, c_int, P(ctypes.c_float), c_size_t]),
        'wrnn_set_debug_steps': (c_int, [c_void_p, P(c_int), c_int]),
        'wrnn_debug_wide_layout': (c_int, [c_int]),
        'wrnn_debug_logits': (c_int, [c_void_p, c_int, c_int, P(ctypes.c_float), c_size_t]),
    }
    # (an A/B build given by WRNN_LIB may predate an entry point: it is left unbound)
    tolerant = host_only or bool(os.environ.get('WRNN_LIB'))
    unbound = []
    for name, (res, args) in sig.items():
        if tolerant and not hasattr(lib, name):
            unbound.append(name)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if unbound and not host_only:
        # a stale or wrong WRNN_LIB says so at load time, not as an AttributeError deep in a run
        import warnings
        warnings.warn(f'{path}: {len(unbound)} entry points missing, left unbound: '
                      + ', '.join(sorted(unbound)), RuntimeWarning, stacklevel=2)
    if path == LIB_PATH:
        _lib = lib
    return lib


def last_error():
    return load_library().wrnn_last_error().decode('utf-8', 'replace')


def check(rc, what=''):
    """Raise the reference's exception type for a failed call (WaveRNNVocoder.cpp:24-41)."""
    if rc == WRNN_OK:
        return
    msg = last_error()
    if what:
        msg = f'{what}: {msg}'
    if rc == WRNN_ERR_INVALID:
        raise ValueError(msg)
    if rc == WRNN_ERR_OOM:
        raise MemoryError(msg)
    if rc == WRNN_ERR_ABORTED:
        raise RuntimeError(msg)
    raise RuntimeError(msg)
