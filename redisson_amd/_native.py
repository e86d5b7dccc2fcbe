"""ctypes binding of libredisson_sketch.so (include/redisson_sketch.h).

This is the same boundary the Java JNI shim binds.  There is
no CPU fallback: if the library is missing, import of the engine fails loudly,
and opening a context without a GPU raises ``DeviceUnavailable``.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

LIB_PATH = os.environ.get("SK_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                       "libredisson_sketch.so")   # override: A/B builds

SK_OK = 0
SK_EWRONGTYPE = -1
SK_ERANGE = -2
SK_ECONFIG = -3
SK_ENOTINIT = -4
SK_EDEVICE = -5
SK_EINVAL = -6
SK_ENOMEM = -7
SK_ESYNTAX = -8
SK_ETOOBIG = -9
SK_ECORRUPT = -10
SK_ESTALE = -11
SK_EBUSYKEY = -12
SK_EPAYLOAD = -13

SK_TYPE_NONE, SK_TYPE_HLL, SK_TYPE_STRING, SK_TYPE_HASH = 0, 1, 2, 3
SK_BITOP = {"AND": 0, "OR": 1, "XOR": 2, "NOT": 3}


class SkConfig(ctypes.Structure):
    _fields_ = [
        ("device", c_int),
        ("redis_major", c_int),
        ("max_bit_offset", c_uint64),
        ("hll_capacity", c_uint64),
        ("max_batch", c_uint64),
    ]


P = c_void_p  # every pointer argument is passed as a raw address
_u8p, _u32p, _u64p, _i64p, _i32p = P, P, P, P, P

# name -> (restype, argtypes)
SIGNATURES = {
    "sk_open": (c_int, [POINTER(SkConfig), POINTER(c_void_p)]),
    "sk_close": (c_int, [P]),
    "sk_last_error": (c_char_p, [P]),
    "sk_strerror": (c_char_p, [c_int]),
    "sk_stream": (c_void_p, [P]),
    "sk_sync": (c_int, [P]),
    "sk_device_count": (c_int, []),
    "sk_crc16": (c_uint32, [_u8p, c_uint64]),
    "sk_calc_slot": (c_int32, [_u8p, c_uint64]),
    "sk_owner": (c_int32, [_u8p, c_uint64, c_int32]),
    "sk_owner_many": (c_int, [c_uint32, _u64p, _u8p, c_int32, _i32p]),
    "sk_bloom_optimal_bits": (c_int64, [c_int64, c_double]),
    "sk_bloom_optimal_k": (c_int32, [c_int64, c_int64]),
    "sk_hll_estimate_hist": (c_uint64, [_u32p, c_int]),
    "sk_type": (c_int, [P, _u8p, c_uint64, P]),
    "sk_type_many": (c_int, [P, c_uint32, _u64p, _u8p, _i32p]),
    "sk_del": (c_int, [P, c_uint32, _u64p, _u8p, _u64p]),
    "sk_hll_resolve": (c_int, [P, c_uint32, _u64p, _u8p, _u32p, _u8p]),
    "sk_hll_lookup": (c_int, [P, c_uint32, _u64p, _u8p, _u32p]),
    "sk_pfadd": (c_int, [P, c_uint32, _u64p, _u8p, _u32p, _u64p, _u8p, _u8p]),
    "sk_pfadd_ids": (c_int, [P, c_uint32, _u32p, _u32p, _u64p, _u8p, _u8p]),
    "sk_pfadd_dev": (c_int, [P, c_uint64, _u32p, _u64p, _u8p, c_uint64, _u8p]),
    "sk_pfcount": (c_int, [P, c_uint32, _u32p, _u64p, _u8p, _i64p]),
    "sk_pfcount_ids": (c_int, [P, c_uint64, _u32p, _i64p]),
    "sk_hll_histogram_dev": (c_int, [P, c_uint64, _u32p, _u32p]),
    "sk_hll_sum_dev": (c_int, [P, c_uint64, _u32p, _u64p]),
    "sk_pfmerge": (c_int, [P, _u8p, c_uint64, c_uint32, _u64p, _u8p]),
    "sk_hll_union_dev": (c_int, [P, c_uint64, _u32p, _u8p]),
    "sk_hll_epoch": (c_int, [P, P]),
    "sk_host_alloc": (c_int, [P, c_uint64, P]),
    "sk_host_free": (c_int, [P, P]),
    "sk_hll_count_registers_dev": (c_int, [P, _u8p, _i64p]),
    "sk_hll_union_keys": (c_int, [P, c_uint32, _u64p, _u8p, c_int32, c_int32, _u8p, _u32p]),
    "sk_hll_merge_registers_dev": (c_int, [P, _u8p, c_uint64, _u8p]),
    "sk_hll_registers": (c_int, [P, _u8p, c_uint64, _u8p]),
    "sk_setbit": (c_int, [P, c_uint32, _u64p, _u8p, _u64p, _u8p, _u8p]),
    "sk_getbit": (c_int, [P, c_uint32, _u64p, _u8p, _u64p, _u8p]),
    "sk_setbit_dev": (c_int, [P, _u8p, c_uint64, c_uint64, _u64p, c_uint8, _u8p]),
    "sk_getbit_dev": (c_int, [P, _u8p, c_uint64, c_uint64, _u64p, _u8p]),
    "sk_bitcount": (c_int, [P, _u8p, c_uint64, _u64p]),
    "sk_strlen": (c_int, [P, _u8p, c_uint64, _u64p]),
    "sk_bitop": (c_int, [P, c_int, _u8p, c_uint64, c_uint32, _u64p, _u8p, _u64p]),
    "sk_get": (c_int, [P, _u8p, c_uint64, _u8p, c_uint64, _i64p]),
    "sk_set": (c_int, [P, _u8p, c_uint64, _u8p, c_uint64]),
    "sk_get_dev": (c_int, [P, _u8p, c_uint64, _u8p, c_uint64, _i64p]),
    "sk_set_dev": (c_int, [P, _u8p, c_uint64, _u8p, c_uint64]),
    "sk_bitset_length": (c_int, [P, _u8p, c_uint64, _i64p]),
    "sk_bloom_try_init": (c_int, [P, _u8p, c_uint64, c_int64, c_double, P]),
    "sk_bloom_config": (c_int, [P, _u8p, c_uint64, P, P, P, P]),
    "sk_bloom_add": (c_int, [P, _u8p, c_uint64, c_int64, c_int32, c_uint32, _u64p, _u8p, _u8p]),
    "sk_bloom_contains": (c_int, [P, _u8p, c_uint64, c_int64, c_int32, c_uint32, _u64p, _u8p, _u8p]),
    "sk_bloom_add_dev": (c_int, [P, _u8p, c_uint64, c_uint64, _u64p, _u8p, c_uint64, _u8p]),
    "sk_bloom_contains_dev": (c_int, [P, _u8p, c_uint64, c_uint64, _u64p, _u8p, c_uint64, _u8p]),
    "sk_bloom_count": (c_int, [P, _u8p, c_uint64, P]),
    "sk_pfadd_ids_prefix": (c_int, [P, c_uint32, _u32p, _u8p, c_uint32, _u32p, _u8p, _u8p]),
    "sk_bloom_add_prefix": (c_int, [P, _u8p, c_uint64, c_int64, c_int32, c_uint32, _u8p, c_uint32, _u32p, _u8p, _u8p]),
    "sk_bloom_contains_prefix": (c_int, [P, _u8p, c_uint64, c_int64, c_int32, c_uint32, _u8p, c_uint32, _u32p, _u8p,
                                         _u8p]),
    "sk_gen_jackson_longs": (c_int, [c_uint64, c_uint64, _u64p, _u8p]),
    "sk_gen_jackson_longs_dev": (c_int, [P, c_uint64, P, c_uint64, c_uint64, P, P]),
    "sk_dev_alloc": (c_int, [P, c_uint64, P]),
    "sk_dev_free": (c_int, [P, P]),
    "sk_h2d": (c_int, [P, P, P, c_uint64]),
    "sk_d2h": (c_int, [P, P, P, c_uint64]),
    "sk_d2d": (c_int, [P, P, P, c_uint64]),
    "sk_dev_memset": (c_int, [P, P, c_int, c_uint64]),
    "sk_timer_record": (c_int, [P, c_int]),
    "sk_timer_elapsed": (c_int, [P, c_int, c_int, P]),
    "sk_set_async": (c_int, [P, c_int]),
    "sk_hll_exact_strings": (c_int, [P, c_int]),
    "sk_prof_enable": (c_int, [P, c_int]),
    "sk_prof_only": (c_int, [P, c_char_p]),
    "sk_set_bit_range": (c_int, [P, _u8p, c_uint64, c_int64, c_int64, c_int]),
    "sk_flushall": (c_int, [P]),
    "sk_ticket": (c_int, [P, P]),
    "sk_poll": (c_int, [P, c_uint64, P]),
    "sk_wait": (c_int, [P, c_uint64]),
    "sk_prof_reset": (c_int, [P]),
    "sk_prof_read": (c_int, [P, c_char_p, P, P]),
    "sk_comm_unique_id": (c_int, [P]),
    "sk_comm_init": (c_int, [P, c_int, c_int, P]),
    "sk_allreduce_max_u8": (c_int, [P, P, c_uint64]),
    "sk_allreduce_sum_u64": (c_int, [P, P, c_uint64]),
    "sk_allgather": (c_int, [P, P, P, c_uint64]),
    # persistence: SCAN / DUMP / RESTORE / SAVE / load (redis-server's formats)
    "sk_scan": (c_int, [P, c_uint64, c_uint32, P, P, P, P, c_uint64, P]),
    "sk_dbsize": (c_int, [P, P]),
    "sk_dump": (c_int, [P, _u8p, c_uint64, _u8p, c_uint64, _i64p]),
    "sk_restore": (c_int, [P, _u8p, c_uint64, _u8p, c_uint64, c_int]),
    "sk_save": (c_int, [P, c_char_p, c_uint32, P, P, P]),
    "sk_load": (c_int, [P, c_char_p, P, P, P]),
    "sk_alltoallv": (c_int, [P, P, _u64p, P, _u64p]),
    "sk_route_bits": (c_int, [P, c_uint64, _u64p, _u8p, c_uint64, c_int32, _u64p, _u8p, _u32p, _u64p]),
    "sk_unroute_u8": (c_int, [P, c_uint64, _u32p, _u8p, _u8p]),
    "sk_bloom_indexes_dev": (c_int, [P, c_uint64, _u64p, _u8p, c_int64, c_int32, c_int32, _u64p]),
    "sk_reduce_groups_u8": (c_int, [P, c_uint64, c_uint32, c_uint32, c_int, _u8p, _u8p]),
    "sk_setbit_values_dev": (c_int, [P, _u8p, c_uint64, c_uint64, _u64p, _u8p, _u8p]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load the in-tree native library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the sketch engine)"
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
