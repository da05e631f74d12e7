"""lambdafs_amd — MI355X-native Reed-Solomon engine for the hops EC codec path.

The product is libhrs.so (HIP kernels for gfx950 behind the C ABI in
include/hrs.h). This package is its host-side mirror of the reference plugin
interface (io.hops.erasure_coding.ErasureCode / Codec) plus device-batch
helpers; every byte is computed on the GPU.
"""
from .erasure_code import (ErasureCode, HipNativeReedSolomonCode, HipReedSolomonCode,  # noqa: F401
                           HipSimpleRegeneratingCode, HipXORCode,
                           TooManyErasedLocations)  # noqa: F401
from .codec import Codec, DEFAULT_CODECS_JSON  # noqa: F401
from ._lib import HrsError  # noqa: F401

__all__ = ["ErasureCode", "HipReedSolomonCode", "HipXORCode", "HipNativeReedSolomonCode",
           "HipSimpleRegeneratingCode", "TooManyErasedLocations", "Codec", "DEFAULT_CODECS_JSON",
           "HrsError"]
