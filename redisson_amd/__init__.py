"""redisson_amd -- MI355X-native sketch engine for Redisson's probabilistic path.

The product is libredisson_sketch.so (HIP kernels + C ABI, include/redisson_sketch.h);
this package is the host-side mirror of the reference's RHyperLogLog / RBitSet /
RBloomFilter / RBatch interfaces over that ABI.
"""
from .codec import ByteArrayCodec, JInteger, JLong, JsonJacksonCodec, LongCodec, StringCodec  # noqa: F401
from .engine import (DeviceUnavailable, IllegalArgumentException, IllegalStateException,  # noqa: F401
                     RedisException, SketchEngine, bloom_optimal_bits, bloom_optimal_k, calc_slot, crc16, device_count,
                     gen_jackson_longs, owner)
from .redisson import Config, JBitSet, RBatch, RBitSet, RBloomFilter, Redisson, RHyperLogLog  # noqa: F401

__all__ = [
    "Redisson", "Config", "RBatch", "RBitSet", "RBloomFilter", "RHyperLogLog", "JBitSet",
    "SketchEngine", "RedisException", "IllegalStateException", "IllegalArgumentException", "DeviceUnavailable",
    "JsonJacksonCodec", "StringCodec", "LongCodec", "ByteArrayCodec", "JLong", "JInteger",
    "calc_slot", "crc16", "owner", "device_count", "bloom_optimal_bits", "bloom_optimal_k", "gen_jackson_longs",
]
