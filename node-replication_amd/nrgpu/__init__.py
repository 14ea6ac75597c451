"""nrgpu — MI355X-native node-replication log replay (host side).

The data plane lives in libnrgpu.so (HIP kernels for gfx950 behind the C ABI of
include/nrgpu.h). This package mirrors the reference `nr` crate's API on top of it.
"""
from . import _lib
from ._lib import NrgError, load
from .combiner import Combiner
from .replica import (
    PUT_DTYPE,
    STACK_OP_DTYPE,
    SYNTH_OP_DTYPE,
    SYNTH_RD_DTYPE,
    AbstractDataStructure,
    DeviceReplica,
    Get,
    Log,
    NrHashMap,
    Peek,
    Pop,
    Push,
    Put,
    ReadOnly,
    ReadWrite,
    Replica,
    ReplicaToken,
    Stack,
    WriteOnly,
)

__all__ = [
    "_lib", "NrgError", "load", "Combiner", "PUT_DTYPE", "STACK_OP_DTYPE", "SYNTH_OP_DTYPE", "SYNTH_RD_DTYPE",
    "AbstractDataStructure", "DeviceReplica", "Get", "Log", "NrHashMap", "Peek", "Pop", "Push", "Put",
    "ReadOnly", "ReadWrite", "Replica", "ReplicaToken", "Stack", "WriteOnly",
]


def device_count() -> int:
    return int(load().nrg_device_count())
