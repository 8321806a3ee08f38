"""lodestar_amd -- MI355X-native BLS12-381 signature-set verifier for Lodestar's IBlsVerifier path.

The product is the gfx950 HIP library libgbv.so (C ABI: include/gbv.h) plus the host mirror of
IBlsVerifier in lodestar_amd.verifier.  Nothing here falls back to the CPU.
"""
from .verifier import (  # noqa: F401
    AggregatedSignatureSet,
    EmptyAggregateError,
    GbvError,
    GpuBlsVerifier,
    PackedSameMessageSets,
    QueueAbortedError,
    SingleSignatureSet,
    VerifySignatureOpts,
    chunkify_maximize_chunk_size,
)
