"""GpuBlsSingleThreadVerifier -- the BlsSingleThreadVerifier semantics on the gfx950 device.

Reference: packages/beacon-node/src/chain/bls/singleThread.ts:8-90 (the IBlsVerifier the node uses
with --chain.blsVerifyAllMainThread, and the one its unit tests construct).  It differs from the
worker pool (GpuBlsVerifier) in one observable way: verifySignatureSetsSameMessage checks the
UNRANDOMIZED aggregate

    verify(message, aggregatePublicKeys(pks), aggregateSignatures(sigs))      (singleThread.ts:41-57)

and answers every set true when it holds, so signatures whose errors cancel in the sum (the
`swapped_keys` fixture) all pass here while the pool's randomized check rejects them.  When the
aggregate fails, every set is verified on its own (singleThread.ts:62-71).

Every step runs on the device through the C ABI -- gbv_aggregate_pubkeys, gbv_signatures_validate,
gbv_aggregate_signatures, gbv_verify_sets (one raw-pubkey set) and gbv_verify_sets_multi (the
per-set retry); there is no CPU path.  verifySignatureSets is verifySignatureSetsMaybeBatch over all
sets (singleThread.ts:15-33); the device evaluates it in <=128-set randomized chunks, which returns
the same boolean as one unchunked batch (both are true iff every set verifies, up to the 2^-64
randomization bound the reference itself accepts).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

from . import _native
from .verifier import GpuBlsVerifier, ISignatureSet, SingleSignatureSet, VerifySignatureOpts  # noqa: F401

_PT_OK = 0


class GpuBlsSingleThreadVerifier:
    """IBlsVerifier with BlsSingleThreadVerifier semantics.  Owns (or borrows) a GpuBlsVerifier,
    whose HBM index2pubkey table holds the keys."""

    def __init__(self, device: int = 0, verifier: GpuBlsVerifier = None):
        self._owned = verifier is None
        self.v = verifier if verifier is not None else GpuBlsVerifier(device)

    # pubkey cache passthrough (syncPubkeys, pubkeyCache.ts:50-69)
    def add_pubkeys(self, first_index: int, pubkeys, validate: bool = False) -> bytes:
        return self.v.add_pubkeys(first_index, pubkeys, validate)

    def verify_signature_sets_sync(self, sets: Sequence[ISignatureSet]) -> bool:
        """singleThread.ts:15-33: verifySignatureSetsMaybeBatch(sets with aggregated pubkeys)."""
        return self.v.verify_signature_sets_sync(sets)

    def verify_signature_sets_same_message_sync(self, sets: Sequence[Tuple[int, bytes]], message: bytes) -> List[bool]:
        """singleThread.ts:36-80.  Raises EmptyAggregateError for an empty list (aggregatePublicKeys
        throws, singleThread.ts:41)."""
        message = bytes(message)
        if len(message) != 32:
            raise ValueError("message must be 32 bytes")
        pk_agg = self.v.aggregate_pubkeys([int(i) for i, _ in sets])                      # :41
        sigs = [bytes(s) for _, s in sets]
        # Signature.fromBytes(sig, true) per set (:44-52); a non-96-byte input throws there too
        # (the SSZ type is Bytes96), mapped to the all-zero encoding blst rejects.
        sigs96 = [s if len(s) == 96 else bytes(96) for s in sigs]
        status, _ = self.v.signatures_validate(sigs96)
        ok_sig = [st == _PT_OK for st in status]
        all_valid = all(ok_sig)
        if all_valid:                                                                       # :54-57
            sig_agg = self.v.aggregate_signatures(sigs96, validate=True)
            all_valid = self.v.verify_signature_sets_sync([SingleSignatureSet(0, message, sig_agg, pubkey=pk_agg)])
        if all_valid:
            return [True] * len(sets)
        # per-set verify(message, set.publicKey, sig) (:62-71), one device pass for all of them
        todo = [i for i, ok in enumerate(ok_sig) if ok]
        out = [False] * len(sets)
        if todo:
            res = self.v.verify_signature_sets_multi_sync([[SingleSignatureSet(int(sets[i][0]), message, sigs96[i])] for i in todo])
            for i, r in zip(todo, res):
                out[i] = r is True
        return out

    # ---- IBlsVerifier (async): the reference resolves synchronously computed results -----------
    async def verify_signature_sets(self, sets: Sequence[ISignatureSet], opts: VerifySignatureOpts = None) -> bool:
        return self.verify_signature_sets_sync(sets)

    async def verify_signature_sets_same_message(self, sets: Sequence[Tuple[int, bytes]], message: bytes,
                                                 opts: VerifySignatureOpts = None) -> List[bool]:
        return self.verify_signature_sets_same_message_sync(sets, message)

    async def close(self):
        if self._owned:
            self.v.close_sync()

    def close_sync(self):
        if self._owned:
            self.v.close_sync()

    def can_accept_work(self) -> bool:
        """singleThread.ts:86-89: no throttling mechanism, always true."""
        return True


__all__ = ["GpuBlsSingleThreadVerifier", "_native"]
