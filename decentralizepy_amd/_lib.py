"""ctypes binding of libdpzcodec.so (the C ABI declared in include/dpz_codec.h).

The shared library is built in-tree (``decentralizepy_amd/libdpzcodec.so``, see
``__graft_entry__.build()``).  There is no fallback: if the library is missing or fails to load,
every codec entry point raises.
"""
import ctypes
import glob
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DPZ_CODEC_LIB selects an alternative build (e.g. the stamped diagnostic build of tools/stamps.py)
LIB_PATH = os.environ.get("DPZ_CODEC_LIB") or os.path.join(_HERE, "libdpzcodec.so")
# The diagnostic build (csrc/dpz_knobs.h): the same sources with the tuning / forced-path
# switches read from DPZ_* environment variables.  The product library reads none.
DIAG_PATH = os.path.join(_HERE, "libdpzcodec_diag.so")

DPZ_ACC_NONE = 0
DPZ_ACC_ACCUMULATE = 1
DPZ_ACC_ADD = 2
DPZ_TOPK_EXACT = 0x1
DPZ_TOPK_ASYNC = 0x2
DPZ_TOPK_STREAM = 0x4
DPZ_TOPK_TAIL = 0x8
DPZ_TOPK_SHARED = 0x10
DPZ_TOPK_VAL_FP16 = 0x20
DPZ_TOPK_HINT = 0x40
DPZ_TOPK_KEEP_X = 0x80
DPZ_TOPK_SLICED = 0x100
DPZ_FOLD_SELF = 0x1
DPZ_FOLD_REPLACE_ONLY = 0x2
DPZ_FOLD_ZERO_BASE = 0x4
DPZ_FOLD_ADD_ONLY = 0x8
DPZ_FOLD_ACCUMULATE = 0x10
DPZ_FOLD_ALSO_LOCAL = 0x20
DPZ_FOLD_BASE_READY = 0x40
DPZ_BATCH_ENCODE = 0x1
DPZ_BATCH_DECODE = 0x2
DPZ_BATCH_HINT = 0x4
DPZ_BATCH_HINT_ALL = 0x8
DPZ_EW_SUB = 1
DPZ_EW_ADD = 2
DPZ_EW_CHOCO = 3
DPZ_EW_MHCOMBINE = 4
DPZ_COUNTER_AUTO = 0
DPZ_COUNTER_SCATTER = 1
DPZ_COUNTER_SWEEP = 2
DPZ_OK = 0
DPZ_ERR_ARG = 1001
DPZ_ERR_WORKSPACE = 1002
DPZ_ERR_UNSUPPORTED = 1003
DPZ_ERR_INTERNAL = 1004

_c_void_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_size = ctypes.c_size_t

# name -> (restype, argtypes); must match include/dpz_codec.h
SIGNATURES = {
    "dpz_abi_version": (_int, []),
    "dpz_build_id": (ctypes.c_char_p, []),
    "dpz_error_string": (ctypes.c_char_p, [_int]),
    "dpz_topk_workspace_bytes": (_size, [_i64, _i64]),
    "dpz_topk_encode": (_int, [_c_void_p, _c_void_p, _c_void_p, _int, _c_void_p, _i64, _i64,
                               _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size, _int, _c_void_p]),
    "dpz_topk_encode_status": (_int, [_c_void_p, _c_void_p, _c_void_p, _int, _c_void_p, _i64,
                                      _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size,
                                      _c_void_p, _int, _c_void_p]),
    "dpz_topk_encode_replace": (_int, [_c_void_p, _c_void_p, _c_void_p, _int, _c_void_p, _i64,
                                       _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size,
                                       _int, _c_void_p, _c_void_p, _c_void_p, _i64, _i64,
                                       _c_void_p, _c_void_p, _size, _c_void_p]),
    "dpz_topk_encode_foldbase": (_int, [_c_void_p, _c_void_p, _c_void_p, _int, _c_void_p, _i64,
                                        _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size,
                                        _int, _int, ctypes.POINTER(ctypes.c_float),
                                        ctypes.c_float, _c_void_p, _c_void_p]),
    "dpz_mask_words": (_i64, [_i64]),
    "dpz_topk_encode_sliced": (_int, [_c_void_p, _c_void_p, _c_void_p, _int, _c_void_p, _i64,
                                      _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                      _size, _c_void_p, _int, _c_void_p]),
    "dpz_counter_unslice": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    "dpz_counter_slice": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    "dpz_rewind_apply": (_int, [_c_void_p, _c_void_p, _i64, _c_void_p]),
    "dpz_counter_flush_workspace_bytes": (_size, [_i64]),
    "dpz_counter_flush": (_int, [_c_void_p, _i64, _c_void_p, ctypes.POINTER(_i64), _int, _int,
                                 _c_void_p, _size, _c_void_p]),
    "dpz_dwt_sym2_rewind": (_int, [_c_void_p, _c_void_p, _i64, _int, _c_void_p, _c_void_p,
                                   _c_void_p]),
    "dpz_dwt_haar_rewind": (_int, [_c_void_p, _c_void_p, _i64, _int, _c_void_p, _c_void_p,
                                   _c_void_p]),
    "dpz_topk_threshold": (_int, [_c_void_p, _i64, _i64, _c_void_p, _c_void_p, _i64, _c_void_p,
                                  _size, ctypes.POINTER(_i64), _c_void_p]),
    "dpz_mask_below_threshold": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p]),
    "dpz_elementwise": (_int, [_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_float, _i64,
                               _c_void_p, _c_void_p]),
    "dpz_gather_change": (_int, [_c_void_p, _c_void_p, _i64, _c_void_p, _i64, _c_void_p,
                                 _c_void_p]),
    "dpz_gather_u32": (_int, [_c_void_p, _i64, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "dpz_gather_u16": (_int, [_c_void_p, _i64, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "dpz_scatter_add_i32": (_int, [_c_void_p, _i64, _c_void_p, _i64, _i64, ctypes.c_int32,
                                   _c_void_p]),
    "dpz_topk_complete": (_int, [_c_void_p, _c_void_p, _c_void_p, _int, _c_void_p, _i64, _i64,
                                 _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size,
                                 ctypes.POINTER(_int), _c_void_p]),
    "dpz_decode_workspace_bytes": (_size, [_i64, _int]),
    "dpz_decode_average": (_int, [_c_void_p, _i64, _int, ctypes.POINTER(_c_void_p),
                                  ctypes.POINTER(_c_void_p), ctypes.POINTER(_i64),
                                  ctypes.POINTER(ctypes.c_float), ctypes.c_float, _int, _c_void_p,
                                  _c_void_p, _size, _c_void_p]),
    "dpz_wavedec_len": (_i64, [_i64, _int]),
    "dpz_dwt_sym2": (_int, [_c_void_p, _c_void_p, _i64, _int, _c_void_p, _c_void_p, _int,
                            _c_void_p]),
    "dpz_dwt_tile_width": (_i64, []),
    "dpz_idwt_tile_width": (_i64, []),
    "dpz_dwt_sym2_tiles": (_int, [_c_void_p, _c_void_p, _i64, _int, _i64, _i64, _c_void_p,
                                  _c_void_p, _int, _c_void_p]),
    "dpz_idwt_sym2_tiles": (_int, [_c_void_p, _i64, _int, _i64, _i64, _c_void_p, _c_void_p]),
    "dpz_idwt_sym2": (_int, [_c_void_p, _i64, _int, _c_void_p, _c_void_p]),
    "dpz_scatter_fill": (_int, [_c_void_p, _i64, _c_void_p, _i64, ctypes.c_float, _c_void_p]),
    "dpz_pack_fp16": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    "dpz_unpack_fp16": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    "dpz_timing_enable": (_int, [_int]),
    "dpz_timing_read": (_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i64), _int]),
    "dpz_kernel_name": (ctypes.c_char_p, [_int]),
    "dpz_replace_slice": (_int, [_c_void_p, _i64, _i64, _c_void_p, _c_void_p, _i64, _c_void_p,
                                 _c_void_p]),
    "dpz_topk_encode_batch": (_int, [_int, _c_void_p, _c_void_p, _i64, _i64, _c_void_p,
                                     _c_void_p, _c_void_p, _c_void_p, _size, _int, _c_void_p,
                                     _c_void_p]),
    "dpz_topk_encode_batch_ex": (_int, [_int, _c_void_p, _c_void_p, _i64, _i64, _c_void_p,
                                     _c_void_p, _c_void_p, _c_void_p, _size, _int, _c_void_p,
                                     _c_void_p, _int]),
    "dpz_topk_encode_nodes": (_int, [_int, _c_void_p, _i64, _i64, _size, _int, _c_void_p]),
    "dpz_decode_average_batch": (_int, [_int, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p,
                                        _c_void_p, _c_void_p, _c_void_p, _c_void_p, _int,
                                        _c_void_p, _size, _int, _c_void_p]),
    "dpz_decode_average_batch_guarded": (_int, [_int, _c_void_p, _c_void_p, _i64, _c_void_p,
                                                _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                                _c_void_p, _int, _c_void_p, _i64, _c_void_p]),
    "dpz_encode_replace_batch": (_int, [_int, _int, _c_void_p, _c_void_p, _i64, _i64, _c_void_p,
                                        _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                        _i64, _c_void_p, _c_void_p, _size, _c_void_p, _size,
                                        _int, _c_void_p]),
    "dpz_topk_sticky_status": (_int, [_c_void_p, _size, _int, ctypes.POINTER(ctypes.c_int32),
                                      _c_void_p]),
    "dpz_elias_max_bytes": (_i64, [_i64]),
    "dpz_elias_workspace_bytes": (_size, [_i64, _i64]),
    "dpz_elias_encode": (_int, [_c_void_p, _i64, _c_void_p, _i64, ctypes.POINTER(_i64),
                                _c_void_p, _size, _c_void_p]),
    "dpz_elias_decode": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _i64,
                                ctypes.POINTER(_i64), _c_void_p, _size, _c_void_p]),
    "dpz_elias_decode_async": (_int, [_c_void_p, _i64, _i64, _i64, _c_void_p, _c_void_p, _i64,
                                      _c_void_p, _c_void_p, _size, _c_void_p]),
    "dpz_fpz_max_bytes": (_i64, [_i64]),
    "dpz_fpz_workspace_bytes": (_size, [_i64]),
    "dpz_fpz_encode": (_int, [_c_void_p, _i64, _int, _c_void_p, _i64, ctypes.POINTER(_i64),
                              _c_void_p, _size, _c_void_p]),
    "dpz_fpz_decode": (_int, [_c_void_p, _i64, _i64, _int, _c_void_p, _c_void_p, _c_void_p]),
    "dpz_fft_workspace_bytes": (_i64, [_i64]),
    "dpz_fft_native": (_int, [_i64]),
    "dpz_rfft": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p, _size, _c_void_p]),
    "dpz_irfft": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p, _size, _c_void_p]),
    "dpz_cplx_key": (_int, [_c_void_p, _c_void_p, _int, _i64, _c_void_p, _c_void_p]),
    "dpz_cplx_gather": (_int, [_c_void_p, _i64, _c_void_p, _i64, _c_void_p, _c_void_p,
                               _c_void_p]),
    "dpz_cplx_pair_indices": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    "dpz_haar_wavedec_len": (_i64, [_i64, _int]),
    "dpz_dwt_haar": (_int, [_c_void_p, _c_void_p, _i64, _int, _c_void_p, _c_void_p, _int,
                            _c_void_p]),
    "dpz_idwt_haar": (_int, [_c_void_p, _i64, _int, _c_void_p, _c_void_p]),
    "dpz_wavedec_len_generic": (_i64, [_i64, _int, _int]),
    "dpz_wavelet_generic_workspace_bytes": (_size, [_i64, _int, _int]),
    "dpz_dwt_generic": (_int, [_c_void_p, _c_void_p, _i64, _int, _c_void_p, _int, _c_void_p,
                               _c_void_p, _int, _c_void_p, _c_void_p, _size, _c_void_p]),
    "dpz_idwt_generic": (_int, [_c_void_p, _i64, _int, _c_void_p, _int, _c_void_p, _c_void_p,
                                _size, _c_void_p]),
    "dpz_lz4_max_bytes": (_i64, [_i64]),
    "dpz_lz4_workspace_bytes": (_size, [_i64, _i64, _i64]),
    "dpz_lz4_compress": (_int, [_c_void_p, _i64, _c_void_p, _i64, ctypes.POINTER(_i64),
                                _c_void_p, _size, _c_void_p]),
    "dpz_lz4_frame_info": (_int, [ctypes.c_char_p, _i64, ctypes.POINTER(_i64),
                                  ctypes.POINTER(_i64), ctypes.POINTER(_int),
                                  ctypes.POINTER(_i64)]),
    "dpz_lz4_decompress": (_int, [_c_void_p, ctypes.c_char_p, _i64, _c_void_p, _i64,
                                  ctypes.POINTER(_i64), _c_void_p, _size, _c_void_p]),
    "dpz_delta_i32": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    "dpz_running_sum_workspace_bytes": (_size, [_i64]),
    "dpz_running_sum_i32": (_int, [_c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p, _size,
                                   _c_void_p]),
}

_lib = None


def source_build_id():
    """The build id the checked-out sources would produce (csrc/Makefile's BUILD_ID: sha256 of
    csrc/*.cpp, *.h, *.hip in name order, csrc/Makefile, include/dpz_codec.h; 16 hex digits)."""
    csrc = os.path.join(_HERE, "csrc")
    files = sorted(os.path.basename(p) for pat in ("*.cpp", "*.h", "*.hip")
                   for p in glob.glob(os.path.join(csrc, pat)))
    h = hashlib.sha256()
    for f in [os.path.join(csrc, f) for f in files] + [
            os.path.join(csrc, "Makefile"),
            os.path.join(os.path.dirname(_HERE), "include", "dpz_codec.h")]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load(path, check_build=True):
    """Load the codec library at ``path`` with every SIGNATURES binding; raises if it is missing
    or (check_build) was built from other sources than the checked-out ones."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"decentralizepy_amd: HIP codec library not found at {path}; "
            "build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C decentralizepy_amd/csrc`). There is no CPU fallback.")
    handle = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if not check_build and not hasattr(handle, name):
            continue  # a diagnostic build of other sources (A/B against an older tree)
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    if check_build:
        built = handle.dpz_build_id().decode()
        want = source_build_id()
        if built != want:
            raise RuntimeError(
                f"decentralizepy_amd: {path} was built from other sources (build id "
                f"{built}, checked-out sources {want}); rebuild it with "
                "`make -C decentralizepy_amd/csrc`")
    return handle


def lib():
    """Load (once) and return the codec library; raises if it is missing."""
    global _lib
    if _lib is None:
        # builds selected with DPZ_CODEC_LIB (diagnostic) are exempt from the build-id check
        _lib = load(LIB_PATH, check_build=not os.environ.get("DPZ_CODEC_LIB"))
    return _lib


def diag_lib():
    """The diagnostic build (DIAG_PATH), for forced-path tests: never the product path."""
    return load(DIAG_PATH)


class CodecError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        msg = lib().dpz_error_string(rc)
        raise CodecError(f"{what} failed: {rc} ({msg.decode() if msg else '?'})")
