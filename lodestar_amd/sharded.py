"""Multi-GPU verification: one process per GPU, torch.distributed (RCCL over xGMI on MI355X,
gloo in CPU tests) -- SURVEY.md 8(e).

Two shapes, both keeping the reference's booleans:

* ``verify_signature_sets`` -- ONE large verifySignatureSets call (block range sync, epoch replay)
  sharded across ranks by cost-balanced contiguous ranges.  Each rank reduces its shard to one Fp12
  Miller product (``gbv_vs_partial``: its sets' pairs and its own (-g1, sum r_i sig_i) pair), the
  576-byte products are ALL-GATHERED (the only data-path collective: 577 B per GPU), and every rank
  runs ONE final exponentiation over all of them (``gbv_fp12_check``).  The answer is the AND over
  the reference's <=128-set jobs (multithread/index.ts:157-207), up to the 2^-64 error of
  randomised batch verification that each job check has as well.
* ``verify_same_message_multi`` -- many independent verifySignatureSetsSameMessage calls (the gossip
  stream): calls are split across ranks in contiguous ranges of near-equal SET count, with no
  collective on the data path; each rank verifies its
  own calls (per-set retries of failing chunks included, jobItem.ts:93-125) and the per-set booleans
  are all-gathered so every rank returns the full result.

The device is anything with the ``GpuBlsVerifier`` methods used here (``vs_partial``,
``fp12_check``, ``verify_same_message_multi_sync``); the CPU tests substitute an oracle-backed one.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

PARTIAL_BYTES = 576

# Cost model for balancing shards (Fp-multiplication equivalents per set):
# ~18k per set (decompress, subgroup, randomisation, hash_to_G2, Miller loop) + 11 per extra pubkey.
SET_COST = 18000
PUBKEY_COST = 11


def set_weight(s) -> int:
    k = len(getattr(s, "indices", ()) or ()) or 1
    return SET_COST + PUBKEY_COST * (k - 1)


def balanced_ranges(weights: Sequence[int], parts: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) ranges, one per part, with near-equal total weight (every set once).
    Part p ends where the running sum is closest to p+1 parts' share of the total: the next item is
    taken when that overshoots the share by no more than leaving it undershoots -- so an item larger
    than a share still starts on the first rank that reaches it instead of piling every later item on
    the last rank.  Ranges are empty only when there are fewer items than parts."""
    n = len(weights)
    total = sum(weights)
    out, lo, acc = [], 0, 0
    for p in range(parts):
        if p == parts - 1:
            out.append((lo, n))
            break
        target = total * (p + 1) / parts
        hi = lo
        while hi < n and acc + weights[hi] - target <= target - acc:
            acc += weights[hi]
            hi += 1
        out.append((lo, hi))
        lo = hi
    return out


class ShardedVerifier:
    """verifySignatureSets / verifySignatureSetsSameMessage over every GPU of the process group."""

    def __init__(self, device, group=None):
        import torch.distributed as dist
        self.device = device
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._tensor_device = "cpu"
        if dist.get_backend(group) == "nccl":  # RCCL on ROCm: the collective runs on the GPU
            import torch
            self._tensor_device = "cuda:%d" % torch.cuda.current_device()

    # ---- collectives ---------------------------------------------------------------------------
    def _all_gather_bytes(self, payload: bytes, size: int) -> List[bytes]:
        import torch
        assert len(payload) == size
        t = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(self._tensor_device)
        outs = [torch.empty(size, dtype=torch.uint8, device=self._tensor_device) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        return [o.cpu().numpy().tobytes() for o in outs]

    # ---- one large verifySignatureSets call ------------------------------------------------------
    def shard_of(self, sets: Sequence) -> Tuple[int, int]:
        return balanced_ranges([set_weight(s) for s in sets], self.world)[self.rank]

    def verify_signature_sets(self, sets: Sequence) -> bool:
        """AND over the whole call on every rank (same answer everywhere)."""
        from ._native import EmptyAggregateError, GBV_E_EMPTY_AGGREGATE, GbvError
        # every rank holds the same call: reject before any collective, on every rank alike
        for s in sets:
            if hasattr(s, "indices") and len(s.indices) == 0:
                raise EmptyAggregateError(GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY")
        if len(sets) == 0:  # verifySignatureSetsMaybeBatch([]) -> false (maybeBatch.ts:29-31)
            return False
        lo, hi = self.shard_of(sets)
        status, part = 2, bytes(PARTIAL_BYTES)
        try:
            part, ok = self.device.vs_partial(list(sets[lo:hi]))
            status = 1 if ok else 0
        finally:  # a device error still takes part in the collective, then raises everywhere
            blobs = self._all_gather_bytes(bytes(part) + bytes([status]), PARTIAL_BYTES + 1)
        if any(b[PARTIAL_BYTES] == 2 for b in blobs):
            raise GbvError(-2, "device error on a peer rank")
        if not all(b[PARTIAL_BYTES] == 1 for b in blobs):
            return False  # a malformed set somewhere: its job is false, so is the call
        return self.device.fp12_check([b[:PARTIAL_BYTES] for b in blobs])

    def verify_staged_shard(self, staged) -> bool:
        """The same exchange for a call whose shard this rank has staged in HBM beforehand
        (StagedSignatureSets over shard_of(call)): gbv_vs_batch_partial -> 577-byte all-gather ->
        one final exponentiation (gbv_fp12_check) on every rank.  Every rank must call it together."""
        status, part = 2, bytes(PARTIAL_BYTES)
        try:
            part, ok = staged.partial()
            status = 1 if ok else 0
        finally:  # a device error still takes part in the collective, then raises here
            blobs = self._all_gather_bytes(bytes(part) + bytes([status]), PARTIAL_BYTES + 1)
        return self._decide(blobs)

    def _exchange(self, part: bytes, status: int) -> bool:
        return self._decide(self._all_gather_bytes(bytes(part) + bytes([status]), PARTIAL_BYTES + 1))

    def _decide(self, blobs: List[bytes]) -> bool:
        from ._native import GbvError
        if any(b[PARTIAL_BYTES] == 2 for b in blobs):
            raise GbvError(-2, "device error on a peer rank")
        if not all(b[PARTIAL_BYTES] == 1 for b in blobs):
            return False
        return self.device.fp12_check([b[:PARTIAL_BYTES] for b in blobs])

    def verify_staged_shards(self, staged: Sequence, depth: int = 2) -> List[bool]:
        """verify_staged_shard over a sequence of staged shards (one per call, or the same shards
        re-verified: a range-sync stream of segments), streamed: up to `depth` shard passes in flight
        on this rank (gbv_vs_batch_partial_submit), so the all-gather and final exponentiation of
        pass k run while pass k + 1's kernels are on the device.  Pass k + depth is submitted before
        pass k's exchange.  A handle must not appear twice within `depth` consecutive entries.  Every
        rank calls it together with sequences of the same length; one answer per entry."""
        n = len(staged)
        depth = max(1, depth)
        out: List[bool] = []
        submitted = [False] * n
        failed = None  # a local device error: this rank still joins every exchange, then raises

        def submit(j):
            nonlocal failed
            if j < n and failed is None:
                try:
                    staged[j].partial_submit()
                    submitted[j] = True
                except Exception as e:  # noqa: BLE001 - reported after the collective
                    failed = e

        for j in range(min(depth, n)):
            submit(j)
        for k in range(n):
            status, part = 2, bytes(PARTIAL_BYTES)
            if submitted[k]:
                try:
                    part, ok = staged[k].partial_wait()
                    status = 1 if ok else 0
                except Exception as e:  # noqa: BLE001
                    failed = failed or e
                submitted[k] = False
            submit(k + depth)  # before the exchange: the next pass overlaps it
            try:
                out.append(self._exchange(part, status))
            except Exception as ex:
                for j in range(k + 1, n):  # drain what this rank still has in flight
                    if submitted[j]:
                        try:
                            staged[j].partial_wait()
                        except Exception:  # noqa: BLE001
                            pass
                if failed is not None:  # this rank's own error is the cause of the collective's
                    raise failed from ex
                raise
        if failed is not None:
            raise failed
        return out

    # ---- many same-message calls (gossip stream / epoch replay) ----------------------------------
    def call_ranges(self, sizes: Sequence[int]) -> List[Tuple[int, int]]:
        """Contiguous call ranges, one per rank, balanced by SET count (the per-set work is what the
        device does; call counts would give a rank of 128-set calls 4x the work of a rank of 32-set
        ones)."""
        return balanced_ranges([max(1, int(x)) for x in sizes], self.world)

    def calls_of(self, n_calls: int, sizes: Optional[Sequence[int]] = None) -> Tuple[int, int]:
        if sizes is not None:
            return self.call_ranges(sizes)[self.rank]
        per = (n_calls + self.world - 1) // self.world
        return min(self.rank * per, n_calls), min((self.rank + 1) * per, n_calls)

    def verify_same_message_multi(self, calls: Sequence[Tuple[Sequence[Tuple[int, bytes]], bytes]]) -> List[List[bool]]:
        from ._native import GbvError
        sizes = [len(c[0]) for c in calls]
        ranges = self.call_ranges(sizes)
        lo, hi = ranges[self.rank]
        # gather per-set booleans: fixed-size payload = all sets of the widest rank's range, plus a
        # status byte (1 ok, 2 this rank raised) so a rank whose device call raises still joins the
        # collective and every rank raises together instead of the others blocking in all_gather
        width = max((sum(sizes[a:b]) for a, b in ranges), default=0)
        flat, status = b"", 2
        try:
            mine = self.device.verify_same_message_multi_sync(list(calls[lo:hi])) if hi > lo else []
            flat = bytes(1 if b else 0 for res in mine for b in res)
            status = 1
        finally:
            blobs = self._all_gather_bytes(bytes([status]) + flat + bytes(width - len(flat)), width + 1)
        if any(b[0] != 1 for b in blobs):
            raise GbvError(-2, "device error on a peer rank")
        blobs = [b[1:] for b in blobs]
        out: List[List[bool]] = []
        for r, (clo, chi) in enumerate(ranges):
            pos = 0
            for g in range(clo, chi):
                out.append([x == 1 for x in blobs[r][pos:pos + sizes[g]]])
                pos += sizes[g]
        return out
