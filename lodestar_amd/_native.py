"""ctypes binding of the C ABI in include/gbv.h (lodestar_amd/libgbv.so, built for gfx950).

There is deliberately no fallback: if the HIP library is missing or no GPU is visible, loading
raises.  The CPU oracle under oracle/ is test infrastructure and is never imported here.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LODESTAR_AMD_LIB selects an alternative in-tree build (A/B experiments with tools/build_variant.sh)
LIB_PATH = os.environ.get("LODESTAR_AMD_LIB") or os.path.join(_HERE, "libgbv.so")

GBV_OK = 0
GBV_E_ARG = -1
GBV_E_DEVICE = -2
GBV_E_EMPTY_AGGREGATE = -3
GBV_E_CLOSED = -4
GBV_E_OOM = -5
GBV_E_BAD_POINT = -6
GBV_CALL_REJECTED = 2

EXPORTED_SYMBOLS = (
    "gbv_init", "gbv_destroy", "gbv_last_error", "gbv_pubkeys_append", "gbv_pubkeys_count", "gbv_comb_enabled",
    "gbv_verify_sets", "gbv_verify_same_message", "gbv_verify_same_message_multi",
    "gbv_aggregate_pubkeys", "gbv_sm_batch_create", "gbv_sm_batch_verify", "gbv_sm_batch_destroy",
    "gbv_sm_batch_submit", "gbv_sm_batch_wait", "gbv_vs_partial", "gbv_fp12_check", "gbv_last_stats",
    "gbv_last_kernel_ms", "gbv_util_sk_to_pk", "gbv_util_sign", "gbv_util_hash_to_g2", "gbv_util_g1_mul_rand",
    "gbv_pubkeys_replicate", "gbv_sha256_digest64", "gbv_merkle_roots", "gbv_signing_roots",
    "gbv_attestation_signing_roots", "gbv_ssz_last_kernel_ms", "gbv_verify_sets_multi", "gbv_vs_batch_create",
    "gbv_vs_batch_submit", "gbv_vs_batch_wait", "gbv_vs_batch_destroy", "gbv_vs_last_kernel_ms",
    "gbv_aggregate_serialized_pubkeys", "gbv_signatures_validate", "gbv_aggregate_signatures",
    "gbv_sm_batch_fill", "gbv_vs_batch_fill", "gbv_vs_batch_partial", "gbv_vs_batch_partial_submit", "gbv_vs_batch_partial_wait", "gbv_tune", "gbv_last_ops",
)


class GbvSet(ctypes.Structure):
    """struct gbv_set (include/gbv.h)."""
    _fields_ = [
        ("idx_off", ctypes.c_uint32),
        ("idx_len", ctypes.c_uint32),
        ("raw_pk48", ctypes.c_void_p),
        ("msg32", ctypes.c_void_p),
        ("sig", ctypes.c_void_p),
        ("sig_len", ctypes.c_uint32),
    ]


class GbvError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("gbv error %d: %s" % (code, msg))
        self.code = code


class EmptyAggregateError(GbvError):
    """blst EMPTY_AGGREGATE_ARRAY: aggregatePublicKeys([]) throws (bls/utils.ts:12)."""


class QueueAbortedError(GbvError):
    """QueueError(QUEUE_ABORTED) (multithread/index.ts:303-305)."""


class BadPointError(GbvError):
    """A serialized point failed to deserialize where blst throws (BLST_BAD_ENCODING,
    BLST_POINT_NOT_ON_CURVE, ...), e.g. aggregateSerializedPublicKeys over a malformed key."""


_lib = None


def load_library(path=LIB_PATH):
    """Load libgbv.so and declare prototypes.  Raises OSError when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError("lodestar_amd: HIP library %s not built (run __graft_entry__.build())" % path)
    lib = ctypes.CDLL(path)
    vp, u32, sz, cp, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_int
    P = ctypes.POINTER
    sig = {
        "gbv_init": (i32, [i32, P(vp)]),
        "gbv_destroy": (None, [vp]),
        "gbv_last_error": (cp, [vp]),
        "gbv_pubkeys_append": (i32, [vp, u32, vp, sz, i32, vp]),
        "gbv_pubkeys_count": (sz, [vp]),
        "gbv_comb_enabled": (ctypes.c_int, [vp]),
        "gbv_verify_sets": (i32, [vp, P(GbvSet), sz, vp, vp, vp]),
        "gbv_verify_same_message": (i32, [vp, vp, vp, sz, vp, vp]),
        "gbv_verify_same_message_multi": (i32, [vp, sz, vp, vp, vp, vp, vp]),
        "gbv_aggregate_pubkeys": (i32, [vp, vp, sz, vp]),
        "gbv_sm_batch_create": (i32, [vp, sz, vp, vp, vp, vp, P(vp)]),
        "gbv_sm_batch_verify": (i32, [vp, vp, vp]),
        "gbv_sm_batch_submit": (i32, [vp, vp]),
        "gbv_vs_partial": (i32, [vp, P(GbvSet), sz, vp, vp, vp]),
        "gbv_fp12_check": (i32, [vp, vp, sz, vp]),
        "gbv_last_stats": (i32, [vp, vp, vp]),
        "gbv_sm_batch_wait": (i32, [vp, vp, vp]),
        "gbv_sm_batch_destroy": (None, [vp, vp]),
        "gbv_last_kernel_ms": (i32, [vp, P(ctypes.c_float), P(ctypes.c_int), i32]),
        "gbv_util_sk_to_pk": (i32, [vp, vp, sz, vp]),
        "gbv_util_sign": (i32, [vp, vp, sz, vp, vp, sz, vp]),
        "gbv_util_hash_to_g2": (i32, [vp, vp, sz, vp]),
        "gbv_util_g1_mul_rand": (i32, [vp, vp, vp, sz, ctypes.c_int, vp]),
        "gbv_pubkeys_replicate": (i32, [vp, u32, u32, u32, sz]),
        "gbv_sha256_digest64": (i32, [vp, vp, sz, vp]),
        "gbv_merkle_roots": (i32, [vp, vp, sz, u32, vp]),
        "gbv_signing_roots": (i32, [vp, vp, sz, vp, sz, vp, vp]),
        "gbv_attestation_signing_roots": (i32, [vp, vp, sz, vp, sz, vp, vp]),
        "gbv_ssz_last_kernel_ms": (i32, [vp, P(ctypes.c_float)]),
        "gbv_verify_sets_multi": (i32, [vp, sz, vp, P(GbvSet), vp, vp]),
        "gbv_vs_batch_create": (i32, [vp, sz, vp, P(GbvSet), vp, P(vp)]),
        "gbv_vs_batch_submit": (i32, [vp, vp]),
        "gbv_vs_batch_wait": (i32, [vp, vp, vp]),
        "gbv_vs_batch_destroy": (None, [vp, vp]),
        "gbv_vs_last_kernel_ms": (i32, [vp, P(ctypes.c_float)]),
        "gbv_aggregate_serialized_pubkeys": (i32, [vp, vp, sz, i32, vp]),
        "gbv_signatures_validate": (i32, [vp, vp, sz, u32, vp, vp]),
        "gbv_aggregate_signatures": (i32, [vp, vp, sz, u32, i32, vp]),
        "gbv_sm_batch_fill": (i32, [vp, vp, sz, vp, vp, vp, vp]),
        "gbv_vs_batch_fill": (i32, [vp, vp, sz, vp, P(GbvSet), vp]),
        "gbv_vs_batch_partial": (i32, [vp, vp, vp, vp]),
        "gbv_vs_batch_partial_submit": (i32, [vp, vp]),
        "gbv_vs_batch_partial_wait": (i32, [vp, vp, vp, vp]),
        "gbv_tune": (i32, [vp, cp, u32]),
        "gbv_last_ops": (i32, [vp, i32, vp, sz]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(lib, ctx, rc):
    if rc == GBV_OK:
        return
    msg = lib.gbv_last_error(ctx)
    msg = msg.decode() if msg else ""
    if rc == GBV_E_EMPTY_AGGREGATE:
        raise EmptyAggregateError(rc, msg)
    if rc == GBV_E_CLOSED:
        raise QueueAbortedError(rc, msg)
    if rc == GBV_E_BAD_POINT:
        raise BadPointError(rc, msg)
    raise GbvError(rc, msg)
