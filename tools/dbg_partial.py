"""Debug helper: one gbv_vs_partial call with GBV_SYNC_DEBUG tracing (GPU box)."""
import faulthandler
import hashlib
import sys

faulthandler.enable()
sys.path.insert(0, ".")
from lodestar_amd import GpuBlsVerifier, SingleSignatureSet  # noqa: E402

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
v = GpuBlsVerifier(0)
sks = [(int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R).to_bytes(32, "big") for i in range(8)]
pks = v.util_sk_to_pk(sks)
v.add_pubkeys(0, pks, validate=True)
msgs = [hashlib.sha256(bytes([i])).digest() for i in range(8)]
sets = [SingleSignatureSet(i, msgs[i], v.util_sign([sks[i]], [0], [msgs[i]])[0]) for i in range(8)]
print("verify", v.verify_signature_sets_sync(sets), flush=True)
for n in (1, 2, 8):
    print("partial", n, flush=True)
    p, ok = v.vs_partial(sets[:n])
    print(" ->", ok, p[:16].hex(), flush=True)
print("check", v.fp12_check([v.vs_partial(sets[:3])[0], v.vs_partial(sets[3:])[0]]), flush=True)
