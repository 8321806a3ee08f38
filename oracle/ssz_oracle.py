"""CPU oracle for the signing-root row.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (lodestar_amd) never does.

Restates, with hashlib's SHA-256:
  * persistent-merkle-tree hasher.digest64(a, b) = sha256(a || b) (@chainsafe/persistent-merkle-tree
    0.8.0 / @chainsafe/as-sha256 0.5.0, yarn.lock:598,360; neither is vendored; call site
    light-client/src/utils/verifyMerkleBranch.ts:23);
  * ContainerType.hashTreeRoot (@chainsafe/ssz 0.11.1, yarn.lock:661, not vendored): basic fields packed
    into 32-byte chunks (uint64 little-endian, zero padded), composite fields by their own roots, chunks
    merkleized as a binary tree zero-padded to the next power of two (the consensus-spec
    merkleization that library implements);
  * computeSigningRoot (state-transition/src/util/signingRoot.ts:7-13) and computeDomain /
    computeForkDataRoot (state-transition/src/util/domain.ts:7-13,25-31);
  * getAttestationDataSigningRoot (beacon-node/src/chain/validation/attestation.ts:657-665) over phase0
    AttestationData (types/src/phase0/sszTypes.ts:247-256) given as its 128-byte SSZ serialisation.

Pinned by K1: the interop deposit signature in beacon-node/test/e2e/interop/
genesisState.test.ts:50-54 signs the DepositMessage signing root built with these same rules, so a
merkleization error would change the signature (tests/test_ssz.py::test_k1_deposit_root_pins_merkleization).
"""
import hashlib
import struct


def sha256(b):
    return hashlib.sha256(b).digest()


def digest64(b64):
    assert len(b64) == 64
    return sha256(b64)


ZERO_CHUNK = bytes(32)


def merkleize(chunks):
    """Root of the chunk list zero-padded to the next power of two (at least one chunk)."""
    nodes = list(chunks) or [ZERO_CHUNK]
    width = 1
    while width < len(nodes):
        width *= 2
    nodes += [ZERO_CHUNK] * (width - len(nodes))
    while len(nodes) > 1:
        nodes = [sha256(nodes[i] + nodes[i + 1]) for i in range(0, len(nodes), 2)]
    return nodes[0]


def merkle_root_fixed(chunks, depth):
    """Root of exactly 2**depth chunks (the layout gbv_merkle_roots takes)."""
    assert len(chunks) == 1 << depth
    return merkleize(chunks)


def uint64_chunk(v):
    return struct.pack("<Q", v) + bytes(24)


def bytes_root(b):
    """hash_tree_root of a fixed-length byte vector (Bytes32 / Bytes48 / Bytes96 ...)."""
    b = bytes(b)
    if len(b) % 32:
        b += bytes(32 - len(b) % 32)
    return merkleize([b[i:i + 32] for i in range(0, len(b), 32)])


def checkpoint_root(epoch, root):
    return merkleize([uint64_chunk(epoch), bytes(root)])


def attestation_data_serialize(slot, index, beacon_block_root, source, target):
    """phase0 AttestationData SSZ bytes: slot | index | beaconBlockRoot | source | target (128 B)."""
    return (struct.pack("<QQ", slot, index) + bytes(beacon_block_root) + struct.pack("<Q", source[0]) + bytes(source[1])
            + struct.pack("<Q", target[0]) + bytes(target[1]))


def attestation_data_root(data128):
    data128 = bytes(data128)
    assert len(data128) == 128
    slot, index = struct.unpack_from("<QQ", data128, 0)
    bbr = data128[16:48]
    src = checkpoint_root(struct.unpack_from("<Q", data128, 48)[0], data128[56:88])
    tgt = checkpoint_root(struct.unpack_from("<Q", data128, 88)[0], data128[96:128])
    return merkleize([uint64_chunk(slot), uint64_chunk(index), bbr, src, tgt])


def compute_signing_root(object_root, domain):
    """hash_tree_root(SigningData{objectRoot, domain}) (signingRoot.ts:7-13)."""
    return merkleize([bytes(object_root), bytes(domain)])


def compute_fork_data_root(current_version, genesis_validators_root):
    return merkleize([bytes(current_version) + bytes(28), bytes(genesis_validators_root)])


def compute_domain(domain_type, fork_version, genesis_validators_root):
    return bytes(domain_type) + compute_fork_data_root(fork_version, genesis_validators_root)[:28]


def attestation_signing_root(data128, domain):
    return compute_signing_root(attestation_data_root(data128), domain)


def deposit_message_root(pubkey48, withdrawal_credentials, amount):
    """hash_tree_root(DepositMessage{pubkey, withdrawalCredentials, amount}) (phase0 sszTypes.ts:117-124)."""
    return merkleize([bytes_root(pubkey48), bytes(withdrawal_credentials), uint64_chunk(amount)])
